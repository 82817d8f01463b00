#!/bin/bash
# round 5, call I: REF2 short launches with whole-row narrow stores per workgroup (lib r2rows) against the per-wave rows (r2base):
# r2rows) against the barrier-block producer/consumer k_rollout_pc (r2base):
# parity of the pp build, sustained 20/1,000-ply A/B, driver-shape bench lines
set -o pipefail
OUT=gpurun_out/r05i
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/tools/diag/build
echo "[r05i] $(date +%T) parity (r2rows)"
NARDE_LIB=$L/libnarde_r2rows.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $OUT/parity_r2rows.log 2>&1 \
  && echo "[r05i] $(date +%T) sustained A/B" \
  && for rep in 1 2; do for tag in r2base r2rows; do echo -n "$tag "; NARDE_LIB=$L/libnarde_$tag.so timeout -k 5 90 python tools/diag/sustained_rollout.py 20,1000 ref2 2>&1 | grep -v amdgpu.ids | tr '\n' ' ' || exit 1; echo; done; done > $OUT/sus_ab.log \
  && echo "[r05i] $(date +%T) driver-shape bench A/B" \
  && for rep in 1 2 3; do for tag in r2base r2rows; do NARDE_LIB=$L/libnarde_$tag.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${tag}_$rep.json 2> $OUT/bench_${tag}_$rep.err || exit 1; done; done
rc=$?
tail -3 $OUT/parity_r2rows.log; cat $OUT/sus_ab.log
for f in $OUT/bench_*.json; do python3 -c "
import json,sys
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" 2>/dev/null; done
echo "[r05i] rc=$rc"
exit $rc
