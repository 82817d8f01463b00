#!/bin/bash
# DIAGNOSTIC round-3 call g: FULL4 narrow-output ring, 16 slots (nring2)
# at drift 10 / 13 / 16 against the product (base): sustained A/B, the
# FULL4 tests on nring2 and on d16, PMC of nring2 and d16.
set -o pipefail
bash tools/diag/gpu_ab_f4.sh base nring2 nring2_d13 nring2_d16 || exit 1
bash tools/diag/gpu_ab_f4.sh nring2 > /dev/null || exit 1
tail -1 gpurun_out/abf4/pytest_full4_nring2.log
bash tools/diag/gpu_pmc_full4.sh nring2 nring2_d16 | grep -v '^ \|^{\|^}' || exit 1
