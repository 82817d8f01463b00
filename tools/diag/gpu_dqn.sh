#!/bin/bash
# Config-4 loop on the box: DQN GPU tests, eager/graph step timing, kernel trace.
#   gpurun -- bash tools/diag/gpu_dqn.sh [tag]
set -o pipefail
TAG=${1:-dqn}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_dqn.py -x -q > "$OUT/pytest.log" 2>&1 \
  && tail -2 "$OUT/pytest.log" \
  && timeout -k 10 200 python tools/dqn_target.py 65536 30 eager \
  && timeout -k 10 200 python tools/dqn_target.py 65536 30 \
  && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o dqn \
        -- python3 "$R/tools/dqn_target.py" 65536 20 > "$OUT/prof.log" 2>&1)
rc=$?
[ $rc -ne 0 ] && tail -30 "$OUT/pytest.log"
exit $rc
