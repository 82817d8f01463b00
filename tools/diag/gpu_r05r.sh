#!/bin/bash
# round 5, call R: REF2 with the Philox draws on the rule waves (phx) against
# the product (pre): parity tests on phx, sustained A/B, driver-shape bench
set -o pipefail
OUT=gpurun_out/r05r
mkdir -p $OUT
export TMPDIR=/tmp
echo "[r05r] $(date +%T) tests (phx)"
NARDE_LIB=$PWD/tools/diag/build/libnarde_phx.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $OUT/tests_phx.log 2>&1 \
  && echo "[r05r] $(date +%T) sustained A/B" \
  && for rep in 1 2 3; do for tag in pre phx; do echo -n "$tag "; NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 90 python tools/diag/sustained_rollout.py 20,1000 ref2 2>&1 | grep -v amdgpu.ids | tr '\n' ' ' || exit 1; echo; done; done > $OUT/sus_ab.log 2>&1 \
  && echo "[r05r] $(date +%T) bench ref2 driver shape A/B" \
  && for rep in 1 2 3 4; do for tag in pre phx; do NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${tag}_$rep.json 2> $OUT/bench_${tag}_$rep.err || exit 1; done; done
rc=$?
tail -2 $OUT/tests_phx.log; cat $OUT/sus_ab.log
for f in $OUT/bench_*.json; do python3 -c "
import json
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f'.split('/')[-1], 'value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])" 2>/dev/null; done
echo "[r05r] rc=$rc"
exit $rc
