#!/bin/bash
# A/B of the REF2 rollout kernel: producer/consumer (default build) vs the
# one-wave-per-64-envs k_rollout (-DNARDE_ROLLOUT_PC=0), same box, same run.
#   bash tools/diag/ab_rollout.sh [build|run]
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/diag/build
if [ "$1" != "run" ]; then
  for v in 0 1; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -DNARDE_ROLLOUT_PC=$v \
      -o tools/diag/build/libnarde_pc$v.so gym-narde_amd/csrc/narde.hip gym-narde_amd/csrc/dqn_learner.hip
  done
fi
if [ "$1" != "build" ]; then
  for v in 0 1 0 1; do
    NARDE_LIB=$PWD/tools/diag/build/libnarde_pc$v.so timeout -k 10 120 python tools/diag/time_rollout.py
  done
fi
