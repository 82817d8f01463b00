#!/bin/bash
# round 5, call K: k_rollout_pp_full's consumer without the per-store
# readfirstlane/exec loops (pc_rsrc_u): FULL4 tests, sustained A/B against
# the previous build, the FULL4 driver-shape bench line
set -o pipefail
OUT=gpurun_out/r05k
mkdir -p $OUT
export TMPDIR=/tmp
echo "[r05k] $(date +%T) full4 tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_full4.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "full4 or rollout_writes or totals" -x -v --timeout 300 --timeout-method thread > $OUT/full4_tests.log 2>&1 \
  && echo "[r05k] $(date +%T) sustained A/B" \
  && timeout -k 10 500 bash tools/diag/gpu_sus20.sh f4base wfx > $OUT/sus_ab.log 2>&1 \
  && echo "[r05k] $(date +%T) bench full4 driver shape" \
  && for k in 1 2; do timeout -k 10 300 python bench.py --rules full4 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_full4_driver_$k.json 2> $OUT/bench_full4_driver_$k.err || exit 1; done
rc=$?
tail -3 $OUT/full4_tests.log; cat $OUT/sus_ab.log
for k in 1 2; do python3 -c "
import json
l=[x for x in open('$OUT/bench_full4_driver_$k.json') if x.startswith('{')][-1]; d=json.loads(l); print('full4 driver kernel_ms', d['roofline']['kernel_ms'], d['roofline']['frac'])" 2>/dev/null; done
echo "[r05k] rc=$rc"
exit $rc
