#!/bin/bash
# DIAGNOSTIC: FULL4 at 20 plies per launch (the driver's shape; k_rollout_wave):
# sustained and single launches of each tools/diag/build/libnarde_<tag>.so.
set -o pipefail
cd "$(dirname "$0")/../.."
for rep in 1 2; do
  for tag in "$@"; do
    echo -n "$tag "
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 60 python tools/diag/sustained_rollout.py 20 full4 2>&1 | grep -v amdgpu.ids || exit 1
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 90 python tools/diag/single_launch.py full4 20 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
