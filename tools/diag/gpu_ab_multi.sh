#!/bin/bash
# DIAGNOSTIC: REF2 (single 20-ply launch + sustained 1,000-ply) and FULL4
# (sustained 1,000 / 20-ply) A/B of tools/diag/build/libnarde_<tag>.so
# variants, two rounds, one box; then the rollout parity tests
# (test_gpu_parity, test_gpu_full4) on every tag.
#   tools/diag/gpu_ab_multi.sh <outdir> <tag>...
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for rep in 1 2; do
  for tag in "$@"; do
    L=$PWD/tools/diag/build/libnarde_$tag.so
    echo -n "$tag ref2 "
    NARDE_LIB=$L NARDE_EVENTS=nofence timeout -k 5 90 python tools/diag/single_launch.py 20 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read())['20']; print('b2b', d['b2b_us'], 'span_min', d['span_min_us'], end=' ')" || exit 1
    NARDE_LIB=$L timeout -k 5 60 python tools/diag/sustained_rollout.py 1000,20 ref2 2>/dev/null | python3 -c "import sys,json; print(' '.join(str(json.loads(l)['ms_per_100_plies']) for l in sys.stdin), end=' ')" || exit 1
    echo -n " full4 "
    NARDE_LIB=$L timeout -k 5 90 python tools/diag/sustained_rollout.py 1000,20 full4 2>/dev/null | python3 -c "import sys,json; print(' '.join(str(json.loads(l)['ms_per_100_plies']) for l in sys.stdin))" || exit 1
  done
done
for tag in "$@"; do
  NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full4.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$tag.log 2>&1
  echo "$tag tests rc=$? $(tail -1 $OUT/pytest_$tag.log)"
done
