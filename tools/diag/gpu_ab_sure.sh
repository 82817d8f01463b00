#!/bin/bash
# FULL4 A/B: HEAD (base) vs the working tree (sure two-dice block-bound turns
# played by the rule wave), sustained 1,000-ply and 20-ply launches, then the
# FULL4 GPU tests on the working tree.  DIAGNOSTIC.
set -o pipefail
OUT=gpurun_out/absure; mkdir -p $OUT
for rep in 1 2; do
  for tag in base sure; do
    echo -n "$tag "; NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 60 python tools/diag/sustained_rollout.py 1000,20 full4 2>/dev/null | tr '\n' ' ' || exit 1; echo
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_full4.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_full4.log 2>&1; rc=$?; tail -2 $OUT/pytest_full4.log; exit $rc
