#!/bin/bash
# DIAGNOSTIC: FULL4 GPU parity tests on the product build, then the sustained
# FULL4 rates (all 36 / non-doubles) of the builds named on the command line.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_full4.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/full4_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/diag/gpu_full4_modes.sh "$@"
