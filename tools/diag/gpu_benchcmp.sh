#!/bin/bash
# the round-2 bench.py against the current one at the driver's shape, same
# box, alternating, 3 runs each.  DIAGNOSTIC.
set -o pipefail
OUT=gpurun_out/bcmp; mkdir -p $OUT
for r in 1 2 3; do
  timeout -k 10 200 python tools/diag/bench_r02.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --dqn-steps 0 > $OUT/old$r.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --dqn-steps 0 > $OUT/new$r.json 2>/dev/null || exit 1
done
python3 - <<'PY'
import json
for k in ("old", "new"):
    for r in (1, 2, 3):
        d = json.load(open(f"gpurun_out/bcmp/{k}{r}.json"))
        print(k, r, round(d["value"] / 1e9, 2), d["timed_region_host_us"], d["roofline"]["kernel_ms"])
PY
