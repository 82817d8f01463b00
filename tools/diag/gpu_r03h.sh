#!/bin/bash
# DIAGNOSTIC round-3 call h: FULL4 with the obs rows through the ring too
# (oring12: 12 slots, drift 12; oring8: 8 slots, drift 8) against the
# product (narrow ring, drift 16 = nring2_d16): sustained A/B, the FULL4
# tests on both obs-ring builds, PMC of both.
set -o pipefail
bash tools/diag/gpu_ab_f4.sh nring2_d16 oring12 oring8 || exit 1
bash tools/diag/gpu_ab_f4.sh oring12 > /dev/null || exit 1
tail -1 gpurun_out/abf4/pytest_full4_oring12.log
bash tools/diag/gpu_pmc_full4.sh oring12 oring8 | grep -v '^ \|^{\|^}' || exit 1
for t in oring12 oring8; do python3 -c "import json; d=json.load(open('gpurun_out/pmcf4_$t.json')); print('$t', d['traffic_over_algorithmic'])"; done
