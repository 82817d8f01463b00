#!/bin/bash
# round 5, call O: FULL4 consumer precomputes each ply's dice, pick words and
# reset side (ply_dice_word) for the producer: FULL4 tests on the product
# build, sustained A/B against the previous build (wfx)
set -o pipefail
OUT=gpurun_out/r05o
mkdir -p $OUT
export TMPDIR=/tmp
echo "[r05o] $(date +%T) full4 tests"
timeout -k 10 700 python -u -m pytest tests/test_gpu_full4.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 \
  && echo "[r05o] $(date +%T) sustained A/B" \
  && timeout -k 10 600 bash tools/diag/gpu_sus20.sh wfx pre wfx pre > $OUT/sus_ab.log 2>&1
rc=$?
tail -3 $OUT/tests.log; cat $OUT/sus_ab.log
echo "[r05o] rc=$rc"
exit $rc
