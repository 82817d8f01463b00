#!/bin/bash
# round 5, call Y: short launches' narrow outputs stored through empty
# resources when absent instead of behind a branch per output (nobr) --
# rollout tests on the product build, sustained A/B, REF2 driver-shape lines
set -o pipefail
OUT=gpurun_out/r05y2
mkdir -p $OUT
export TMPDIR=/tmp
echo "[r05y] $(date +%T) tests"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full4.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 \
  && echo "[r05y] $(date +%T) sustained A/B" \
  && for rep in 1 2 3; do for tag in cur nobr; do for rules in ref2 full4; do echo -n "$tag "; NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 90 python tools/diag/sustained_rollout.py 20 $rules 2>&1 | grep -v amdgpu.ids | tr '\n' ' ' || exit 1; echo; done; done; done > $OUT/sus_ab.log 2>&1 \
  && echo "[r05y] $(date +%T) bench ref2 driver shape A/B" \
  && for rep in 1 2 3 4; do for tag in cur nobr; do NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${tag}_$rep.json 2> $OUT/bench_${tag}_$rep.err || exit 1; done; done
rc=$?
tail -2 $OUT/tests.log; cat $OUT/sus_ab.log
for f in $OUT/bench_*.json; do python3 -c "
import json
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f'.split('/')[-1], 'value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])" 2>/dev/null; done
echo "[r05y] rc=$rc"
exit $rc
