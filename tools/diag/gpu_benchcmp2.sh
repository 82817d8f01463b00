#!/bin/bash
# current bench.py at the driver's shape: where the timed region's host time
# goes (submit / totals call / wait / close).  DIAGNOSTIC.
set -o pipefail
OUT=gpurun_out/bcmp2; mkdir -p $OUT
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --dqn-steps 0 > $OUT/new$r.json 2>/dev/null || exit 1
done
for r in 1 2 3; do python3 -c "import json; d=json.load(open('$OUT/new$r.json')); print(round(d['value']/1e9,2), d['timed_region_host_us'], d['roofline']['kernel_ms'])"; done
