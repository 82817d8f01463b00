#!/bin/bash
# DIAGNOSTIC call: GPU tests + the driver-shape evidence (tools/gpu_driver_shape.sh),
# the host-overhead probe, and the default (1,000-ply) bench for the sustained rate.
set -o pipefail
TAG=${1:?tag}
bash tools/gpu_driver_shape.sh "$TAG" || exit $?
OUT=gpurun_out/$TAG
timeout -k 10 120 python tools/diag/host_overheads.py > "$OUT/host_overheads.txt" 2>&1 && cat "$OUT/host_overheads.txt" \
  && timeout -k 10 300 python bench.py --no-cpu-baseline --dqn-steps 0 > "$OUT/bench_n1_default.json" 2> "$OUT/bench_n1_default.err" \
  && cat "$OUT/bench_n1_default.json"
