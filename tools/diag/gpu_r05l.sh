#!/bin/bash
# round 5, call L: consumers stage each ply's obs rows in LDS (obs_stage)
# instead of extracting every quad from the ply results per lane: rollout
# parity tests on the product build, sustained REF2 + FULL4 A/B, REF2 bench
# lines at the driver's shape alternating the two builds
set -o pipefail
OUT=gpurun_out/r05l
mkdir -p $OUT
export TMPDIR=/tmp
echo "[r05l] $(date +%T) rollout tests"
timeout -k 10 700 python -u -m pytest tests/test_gpu_full4.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 \
  && echo "[r05l] $(date +%T) sustained A/B" \
  && timeout -k 10 600 bash tools/diag/gpu_sus_both.sh wfx stage > $OUT/sus_ab.log 2>&1 \
  && echo "[r05l] $(date +%T) bench ref2 driver shape A/B" \
  && for rep in 1 2 3; do for tag in wfx stage; do NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${tag}_$rep.json 2> $OUT/bench_${tag}_$rep.err || exit 1; done; done
rc=$?
tail -3 $OUT/tests.log; cat $OUT/sus_ab.log
for f in $OUT/bench_wfx_*.json $OUT/bench_stage_*.json; do python3 -c "
import json
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" 2>/dev/null; done
echo "[r05l] rc=$rc"
exit $rc
