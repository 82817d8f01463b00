#!/bin/bash
# round 3: the config / DQN GPU tests, the launch-after-marker diagnostic
# (with RCCL's own all-gather), three driver-shape bench lines, and the
# N-rank path rehearsed on one GPU (bench.py --gpus 2 spawning its ranks,
# gloo) -- correctness, not a measurement.
set -o pipefail
OUT=gpurun_out/r03d; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r03d] $(date +%T) pytest"
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "[r03d] $(date +%T) launch after marker"
timeout -k 10 200 python tools/diag/launch_after_marker.py 20 > $OUT/lam.json 2> $OUT/lam.err && cat $OUT/lam.json || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench$r.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$OUT/bench$r.json')); print(round(d['value']/1e9,2), d['timed_region_host_us'], d['roofline']['kernel_ms'])"
done
echo "[r03d] $(date +%T) FULL4 loop counters"
timeout -k 10 120 python tools/diag/f4_counts.py 1000 > $OUT/f4counts.json 2> $OUT/f4counts.err && cat $OUT/f4counts.json || exit 1
echo "[r03d] $(date +%T) rehearsal --gpus 2"
NARDE_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --dqn-steps 3 --api-steps 20 --other-launches 3 --fused-launches 2 > $OUT/rehearse2.json 2> $OUT/rehearse2.err; rc=$?
tail -3 $OUT/rehearse2.err; cut -c1-600 $OUT/rehearse2.json; exit $rc
