#!/bin/bash
# GPU tests only (optionally a subset): bash tools/diag/gpu_tests_only.sh <tag> [pytest args]
set -o pipefail
TAG=${1:?tag}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
tail -15 gpurun_out/$TAG/pytest.log
exit $rc
