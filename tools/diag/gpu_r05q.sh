#!/bin/bash
# round 5, call Q: REF2 consumer cost -- the ply's board as one 32-B record per
# env (lay: own and opponent words three dwords apart, one ds_read2 and one
# address per obs quad) and, on top, the Philox draws on the rule waves
# instead of the consumers (layphx): tests on the product (lay) and on
# layphx, sustained A/B and bench lines at the driver's shape
set -o pipefail
OUT=gpurun_out/r05q
mkdir -p $OUT
export TMPDIR=/tmp
echo "[r05q] $(date +%T) tests"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_bench_line.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 \
  && NARDE_LIB=$PWD/tools/diag/build/libnarde_layphx.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $OUT/tests_layphx.log 2>&1 \
  && echo "[r05q] $(date +%T) sustained A/B" \
  && for rep in 1 2 3; do for tag in pre lay layphx; do echo -n "$tag "; NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 90 python tools/diag/sustained_rollout.py 20,1000 ref2 2>&1 | grep -v amdgpu.ids | tr '\n' ' ' || exit 1; echo; done; done > $OUT/sus_ab.log 2>&1 \
  && echo "[r05q] $(date +%T) bench ref2 driver shape A/B" \
  && for rep in 1 2 3; do for tag in pre lay layphx; do NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${tag}_$rep.json 2> $OUT/bench_${tag}_$rep.err || exit 1; done; done
rc=$?
tail -2 $OUT/tests.log; tail -2 $OUT/tests_layphx.log; cat $OUT/sus_ab.log
for f in $OUT/bench_*.json; do python3 -c "
import json
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f'.split('/')[-1], 'value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])" 2>/dev/null; done
echo "[r05q] rc=$rc"
exit $rc
