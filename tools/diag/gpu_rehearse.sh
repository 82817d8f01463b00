#!/bin/bash
# DIAGNOSTIC: the N-rank bench path (torchrun, env-id shards, barrier +
# max-over-ranks timing, the statistics all-gather) on a ONE-GPU box: every
# rank on GPU 0 over gloo (NARDE_REHEARSAL=1).  Correctness of the path, not
# a measurement.  Usage: gpurun -- bash tools/diag/gpu_rehearse.sh [N]
set -o pipefail
N=${1:-2}
mkdir -p gpurun_out/rehearse
export NARDE_REHEARSAL=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus "$N" --steps 2000 --warmup 200 \
  --dqn-steps 5 --api-steps 50 --other-launches 5 > gpurun_out/rehearse/bench_n$N.json \
  2> gpurun_out/rehearse/bench_n$N.err
rc=$?
tail -5 gpurun_out/rehearse/bench_n$N.err
cat gpurun_out/rehearse/bench_n$N.json | cut -c1-400
exit $rc
