#!/bin/bash
# round 5, call AA: per-env statistics read at the launch's start (prest)
# instead of after the last ply -- rollout tests on the product, sustained
# 20-ply A/B, driver-shape lines for both rules alternating
set -o pipefail
OUT=gpurun_out/r05aa
mkdir -p $OUT
export TMPDIR=/tmp
echo "[r05aa] $(date +%T) tests"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full4.py tests/test_gpu_configs.py tests/test_gpu_bench_line.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 \
  && echo "[r05aa] $(date +%T) sustained A/B" \
  && for rep in 1 2; do for tag in cur prest; do for rules in ref2 full4; do echo -n "$tag "; NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 90 python tools/diag/sustained_rollout.py 20 $rules 2>&1 | grep -v amdgpu.ids | tr '\n' ' ' || exit 1; echo; done; done; done > $OUT/sus_ab.log 2>&1 \
  && echo "[r05aa] $(date +%T) driver-shape A/B" \
  && for rep in 1 2 3 4; do for tag in cur prest; do for rules in ref2 full4; do NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 300 python bench.py --rules $rules --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${rules}_${tag}_$rep.json 2> $OUT/bench_${rules}_${tag}_$rep.err || exit 1; done; done; done
rc=$?
tail -2 $OUT/tests.log; cat $OUT/sus_ab.log
for f in $OUT/bench_*.json; do python3 -c "
import json
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f'.split('/')[-1], 'value', round(d['value']/1e9,2), 'kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])" 2>/dev/null; done
echo "[r05aa] rc=$rc"
exit $rc
