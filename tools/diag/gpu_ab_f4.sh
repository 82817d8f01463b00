#!/bin/bash
# FULL4 A/B of tools/diag/build/libnarde_<tag>.so variants: sustained
# 1,000-ply and 20-ply launches, two rounds; then the FULL4 GPU tests on the
# last tag's library.  DIAGNOSTIC.
set -o pipefail
OUT=gpurun_out/abf4; mkdir -p $OUT
for rep in 1 2; do
  for tag in "$@"; do
    echo -n "$tag "; NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 60 python tools/diag/sustained_rollout.py 1000,20 full4 2>/dev/null | python3 -c "import sys,json; print(' '.join(str(json.loads(l)['ms_per_100_plies']) for l in sys.stdin))" || exit 1
  done
done
last=${@: -1}
NARDE_LIB=$PWD/tools/diag/build/libnarde_$last.so timeout -k 10 400 python -u -m pytest tests/test_gpu_full4.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_full4_$last.log 2>&1; rc=$?; tail -2 $OUT/pytest_full4_$last.log; exit $rc
