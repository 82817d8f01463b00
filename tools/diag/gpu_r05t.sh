#!/bin/bash
# round 5, call T: k_step<false> against a 1-ply producer/consumer rollout
set -o pipefail
OUT=gpurun_out/r05t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/diag/step_vs_rollout1.py > $OUT/step_vs_rollout1.json 2> $OUT/err.log
rc=$?
cat $OUT/step_vs_rollout1.json; tail -3 $OUT/err.log
echo "[r05t] rc=$rc"
exit $rc
