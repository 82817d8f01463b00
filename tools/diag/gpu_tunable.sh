#!/bin/bash
# DIAGNOSTIC: config-4 step with TunableOp GEMM selection (tune once into a
# results file, then replay with the file) vs the default heuristics.
set -o pipefail
mkdir -p gpurun_out/tun
export PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tun/tunableop_results%d.csv
timeout -k 10 200 python tools/dqn_target.py 65536 30 \
  && PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 \
     timeout -k 10 400 python tools/dqn_target.py 65536 30 \
  && PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 200 python tools/dqn_target.py 65536 30 \
  && timeout -k 10 200 python tools/dqn_target.py 65536 30 \
  && ls -la gpurun_out/tun && head -30 gpurun_out/tun/*.csv
