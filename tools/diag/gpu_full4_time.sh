#!/bin/bash
# DIAGNOSTIC: FULL4 rollout timing (+ GPU FULL4 parity tests first).
set -o pipefail
cd "$(dirname "$0")/../.."
timeout -k 10 300 python -m pytest tests/test_gpu_full4.py -x -q 2>&1 | tail -2 || exit 1
for spec in "full4 all36" "full4 nodoubles" "ref2 all36" "ref2 nodoubles"; do
  timeout -k 10 120 python tools/diag/time_rollout.py 65536 $spec 2>&1 | grep -v amdgpu.ids || exit 1
done
