#!/bin/bash
# REF2 A/B of tools/diag/build/libnarde_<tag>.so variants at the driver's
# shape: single 20-ply launches after a ramp (median of 30: round trip,
# event span), sustained 1,000-ply rate; three rounds, alternating; then
# the REF2 parity tests on the last tag's library.  DIAGNOSTIC.
set -o pipefail
OUT=gpurun_out/abref2; mkdir -p $OUT
for rep in 1 2 3; do
  for tag in "$@"; do
    echo -n "$tag "
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so NARDE_EVENTS=nofence timeout -k 5 90 python tools/diag/single_launch.py 20 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['20'], end=' ')" || exit 1
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 60 python tools/diag/sustained_rollout.py 1000 ref2 2>/dev/null | python3 -c "import sys,json; print(json.loads(sys.stdin.read())['ms_per_100_plies'])" || exit 1
  done
done
last=${@: -1}
NARDE_LIB=$PWD/tools/diag/build/libnarde_$last.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$last.log 2>&1; rc=$?; tail -2 $OUT/pytest_$last.log; exit $rc
