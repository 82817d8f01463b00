#!/bin/bash
# round 5, call F: the full GPU suite on the current build (k_step straight-line
# ply + non-temporal API stores, the pairwise FULL4 rollout), the API kernels
# timed and traced, the smoke
set -o pipefail
OUT=gpurun_out/r05f
mkdir -p $OUT
export TMPDIR=/tmp
echo "[r05f] $(date +%T) pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  && echo "[r05f] $(date +%T) smoke" \
  && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
  && echo "[r05f] $(date +%T) api kernels" \
  && timeout -k 10 120 python3 tools/api_target.py > $OUT/api.json \
  && (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/api_trace -o api \
        -- python3 $GRAFT_REPO_ROOT/tools/api_target.py > $GRAFT_REPO_ROOT/$OUT/api_trace.log 2>&1)
rc=$?
tail -3 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log; cat $OUT/api.json
echo "[r05f] rc=$rc"
exit $rc
