#!/bin/bash
# round 3: all GPU tests, three driver-shape bench lines, the launch-after-
# marker diagnostic.
set -o pipefail
OUT=gpurun_out/r03c; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r03c] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench$r.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$OUT/bench$r.json')); print(round(d['value']/1e9,2), d['timed_region_host_us'], d['roofline']['kernel_ms'], d['config']['rank_totals'])"
done
echo "[r03c] $(date +%T) launch after marker"
timeout -k 10 200 python tools/diag/launch_after_marker.py 20 > $OUT/lam.json 2> $OUT/lam.err && cat $OUT/lam.json
