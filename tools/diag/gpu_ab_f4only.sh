#!/bin/bash
# DIAGNOSTIC: FULL4-only A/B (sustained 1,000 / 20-ply launches, three
# rounds, one box) of tools/diag/build/libnarde_<tag>.so variants, then the
# FULL4 parity tests on every tag.
#   tools/diag/gpu_ab_f4only.sh <outdir> <tag>...
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for rep in 1 2 3; do
  for tag in "$@"; do
    L=$PWD/tools/diag/build/libnarde_$tag.so
    echo -n "$tag full4 "
    NARDE_LIB=$L timeout -k 5 90 python tools/diag/sustained_rollout.py 1000,20 full4 2>/dev/null | python3 -c "import sys,json; print(' '.join(str(json.loads(l)['ms_per_100_plies']) for l in sys.stdin))" || exit 1
  done
done | tee $OUT/ab.txt
for tag in "$@"; do
  NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 300 python -u -m pytest tests/test_gpu_full4.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$tag.log 2>&1
  rc=$?
  echo "$tag tests rc=$rc $(tail -1 $OUT/pytest_$tag.log)"
  [ $rc -eq 0 ] || exit $rc
done
