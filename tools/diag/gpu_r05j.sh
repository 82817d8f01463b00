#!/bin/bash
# round 5, call J: FULL4 pairwise kernel variants (producer priority, consumer sleep, ring depth)
# FULL4 GPU tests + the host-check-mirrored parity, sustained A/B against the
# committed pairwise kernel, the FULL4 driver-shape bench line
set -o pipefail
OUT=gpurun_out/r05j
mkdir -p $OUT
export TMPDIR=/tmp
echo "[r05j] $(date +%T) full4 tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_full4.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "full4 or rollout_writes or totals" -x -v --timeout 300 --timeout-method thread > $OUT/full4_tests.log 2>&1 \
  && echo "[r05j] $(date +%T) sustained A/B" \
  && timeout -k 10 500 bash tools/diag/gpu_sus20.sh f4base f4prio f4sl16 f4r4 > $OUT/sus_ab.log 2>&1 \
  && echo "[r05j] $(date +%T) api kernels A/B (one workgroup per CU)" \
  && for rep in 1 2; do for tag in f4base lds1; do echo -n "$tag "; NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 120 python tools/api_target.py 2>/dev/null | tail -1 || exit 1; done; done > $OUT/api_ab.log 2>&1 \
  && echo "[r05j] $(date +%T) timed launch as a graph: bench A/B" \
  && NARDE_LIB=$PWD/tools/diag/build/libnarde_tgraph.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_line.py -x -v --timeout 280 --timeout-method thread > $OUT/tgraph_test.log 2>&1 \
  && for rep in 1 2 3; do for tag in f4base tgraph; do NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${tag}_$rep.json 2> $OUT/bench_${tag}_$rep.err || exit 1; done; done \
  && echo "[r05j] $(date +%T) bench full4 driver shape" \
  && for k in 1; do timeout -k 10 300 python bench.py --rules full4 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_full4_driver_$k.json 2> $OUT/bench_full4_driver_$k.err || exit 1; done
rc=$?
tail -3 $OUT/full4_tests.log; cat $OUT/sus_ab.log; cat $OUT/api_ab.log
for k in 1 2; do python3 -c "
import json,sys
l=[x for x in open('$OUT/bench_full4_driver_$k.json') if x.startswith('{')][-1]; d=json.loads(l); print('full4 driver kernel_ms', d['roofline']['kernel_ms'], d['roofline']['frac'])" 2>/dev/null; done
tail -2 $OUT/tgraph_test.log
for f in $OUT/bench_f4base_*.json $OUT/bench_tgraph_*.json; do python3 -c "
import json
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['timed_region_host_us'])" 2>/dev/null; done
echo "[r05j] rc=$rc"
exit $rc
