#!/bin/bash
# Build libnarde with each NARDE_OBS_STORE strategy (DIAGNOSTIC) and time
# k_rollout with each: bash tools/diag/variants.sh [build|run]
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/diag/build
if [ "$1" != "run" ]; then
  for v in 0 1 2; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -DNARDE_OBS_STORE=$v \
      -o tools/diag/build/libnarde_v$v.so gym-narde_amd/csrc/narde.hip gym-narde_amd/csrc/dqn_learner.hip
  done
fi
if [ "$1" != "build" ]; then
  for v in 0 1 2; do
    NARDE_LIB=$PWD/tools/diag/build/libnarde_v$v.so timeout -k 10 120 python tools/diag/time_rollout.py
  done
fi
