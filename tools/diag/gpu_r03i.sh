#!/bin/bash
# DIAGNOSTIC round-3 call i: FULL4 with each obs row's shared 64-B granule
# (32 B of each of two adjacent rows) stored at the flush (hring) against the
# product (narrow ring, drift 16 = nring2_d16): sustained A/B x3, the FULL4
# tests on hring, PMC of hring.
set -o pipefail
bash tools/diag/gpu_ab_f4.sh nring2_d16 hring || exit 1
bash tools/diag/gpu_ab_f4.sh nring2_d16 hring | grep -v passed || exit 1
bash tools/diag/gpu_pmc_full4.sh hring | grep -v '^ \|^{\|^}' || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/pmcf4_hring.json')); print('hring', d['traffic_over_algorithmic'])"
