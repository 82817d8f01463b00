#!/bin/bash
# DIAGNOSTIC: in-kernel clock of k_rollout_pc for each -DNARDE_DIAG_CLOCK=1
# build tools/diag/build/libnarde_<tag>.so named on the command line.
set -o pipefail
cd "$(dirname "$0")/../.."
for tag in "$@"; do
  for mode in rollout selfplay; do
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 120 python tools/diag/clock_rollout.py $mode 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
