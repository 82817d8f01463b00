#!/bin/bash
# DIAGNOSTIC: FULL4 GPU tests on the product build, then sustained FULL4
# (1,000-ply launches) and REF2 rates of tools/diag/build/libnarde_<tag>.so
# for each tag, interleaved twice (A/B inside one call, one box).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_full4.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/full4_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/full4_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for tag in "$@"; do
    echo -n "$tag "
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 45 python tools/diag/sustained_rollout.py 1000 full4 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
for tag in "$@"; do
  echo -n "$tag "
  NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 45 python tools/diag/sustained_rollout.py 1000 ref2 2>&1 | grep -v amdgpu.ids || exit 1
done
