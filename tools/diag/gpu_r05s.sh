#!/bin/bash
# round 5, call S: the new launch-edge tests (REF2 barrier blocks, FULL4 ring depth)
set -o pipefail
OUT=gpurun_out/r05s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full4.py -k "block_boundaries or ring_boundaries" -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -6 $OUT/tests.log
echo "[r05s] rc=$rc"
exit $rc
