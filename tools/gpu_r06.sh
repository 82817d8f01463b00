#!/bin/bash
# Round 6's GPU calls (run on the MI355X box from the repo root):
#   gpurun -- bash tools/gpu_r06.sh TAG PHASE
# Every GPU step has its own time limit, the steps are chained with &&.
set -o pipefail
TAG=${1:-r06}
PHASE=${2:-parity}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
case "$PHASE" in
parity)  # the full-batch parity tests and the self-checking bench line
  timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_full4.py -m gpu > "$OUT/pytest.log" 2>&1 \
    && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" \
    && timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
  rc=$?; tail -3 "$OUT/pytest.log"; exit $rc ;;
drv)  # the driver's command, with and without the checker leg, alternating
  for k in 1 2 3; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/drv_chk_$k.json" 2> "$OUT/drv_chk_$k.err" \
      && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-parity-check --no-cpu-baseline \
           > "$OUT/drv_nochk_$k.json" 2> "$OUT/drv_nochk_$k.err" || exit 1
  done ;;
*) echo "unknown phase $PHASE"; exit 2 ;;
esac
