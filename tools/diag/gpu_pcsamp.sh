#!/bin/bash
# PC sampling of the FULL4 rollout (k_rollout_full, 100 plies per launch):
# where the rule waves' issue goes.  DIAGNOSTIC.
set -o pipefail
OUT=gpurun_out/pcs; mkdir -p $OUT; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $R/$OUT/list.txt 2>&1); grep -i -B2 -A12 "pc_sampling\|PC Sampling" $OUT/list.txt | head -60
M=${1:-stochastic}; U=${2:-cycles}; I=${3:-65536}
echo "[pcs] $(date +%T) method $M unit $U interval $I"
(cd /tmp && timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit $U \
   --pc-sampling-interval $I --output-format csv -d $R/$OUT/run -o pcs -- python3 $R/tools/diag/sq_target.py full4 100 \
   > $R/$OUT/run.log 2>&1); rc=$?
echo "rc=$rc"; tail -5 $OUT/run.log; find $OUT/run -type f | head; exit $rc
