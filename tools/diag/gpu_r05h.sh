#!/bin/bash
# round 5, call H: REF2 through the pairwise kernel (k_rollout_pp_ref2, lib
# r2pp) against the barrier-block producer/consumer k_rollout_pc (r2pc):
# parity of the pp build, sustained 20/1,000-ply A/B, driver-shape bench lines
set -o pipefail
OUT=gpurun_out/r05h
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/tools/diag/build
echo "[r05h] $(date +%T) parity (r2pp)"
NARDE_LIB=$L/libnarde_r2pp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $OUT/parity_r2pp.log 2>&1 \
  && echo "[r05h] $(date +%T) sustained A/B" \
  && for rep in 1 2; do for tag in r2pc r2pp; do echo -n "$tag "; NARDE_LIB=$L/libnarde_$tag.so timeout -k 5 90 python tools/diag/sustained_rollout.py 20,1000 ref2 2>&1 | grep -v amdgpu.ids | tr '\n' ' ' || exit 1; echo; done; done > $OUT/sus_ab.log \
  && echo "[r05h] $(date +%T) driver-shape bench A/B" \
  && for rep in 1 2 3; do for tag in r2pc r2pp; do NARDE_LIB=$L/libnarde_$tag.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${tag}_$rep.json 2> $OUT/bench_${tag}_$rep.err || exit 1; done; done
rc=$?
tail -3 $OUT/parity_r2pp.log; cat $OUT/sus_ab.log
for f in $OUT/bench_*.json; do python3 -c "
import json,sys
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" 2>/dev/null; done
echo "[r05h] rc=$rc"
exit $rc
