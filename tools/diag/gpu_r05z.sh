#!/bin/bash
# round 5, call Z: the pair pass (coop_pair_w: the block-bound doubles
# search's root and sub-move-1 check in one cooperative pass) -- FULL4 GPU
# tests on the product build, sustained A/B, k_step<true>, driver-shape lines
set -o pipefail
OUT=gpurun_out/r05z2
mkdir -p $OUT
export TMPDIR=/tmp
echo "[r05z] $(date +%T) full4 tests"
timeout -k 10 700 python -u -m pytest tests/test_gpu_full4.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "full4 or rollout_writes or totals" -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 \
  && echo "[r05z] $(date +%T) sustained A/B" \
  && timeout -k 10 600 bash tools/diag/gpu_sus20.sh cur pair cur pair > $OUT/sus_ab.log 2>&1 \
  && echo "[r05z] $(date +%T) api A/B" \
  && for rep in 1 2; do for tag in cur pair; do echo -n "$tag "; NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 120 python tools/api_target.py 2>/dev/null | tail -1 || exit 1; done; done > $OUT/api_ab.log 2>&1 \
  && echo "[r05z] $(date +%T) bench full4 driver shape A/B" \
  && for rep in 1 2 3; do for tag in cur pair; do NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 300 python bench.py --rules full4 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${tag}_$rep.json 2> $OUT/bench_${tag}_$rep.err || exit 1; done; done
rc=$?
tail -2 $OUT/tests.log; cat $OUT/sus_ab.log
python3 - <<PY
import json
for l in open("$OUT/api_ab.log"):
    tag, js = l.split(" ", 1)
    d = json.loads(js); print(tag, "k_step_full4", d["k_step_full4"]["graph_us"], "k_step_ref2", d["k_step_ref2"]["graph_us"])
PY
for f in $OUT/bench_*.json; do python3 -c "
import json
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f'.split('/')[-1], 'value', d['value'], 'kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])" 2>/dev/null; done
echo "[r05z] rc=$rc"
exit $rc
