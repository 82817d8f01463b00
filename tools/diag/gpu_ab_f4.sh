#!/bin/bash
# DIAGNOSTIC (round 4): FULL4 sustained 20 / 1000-ply rollouts of
# libnarde_<tag>.so builds, alternating, 2 rounds.
set -o pipefail
cd "$(dirname "$0")/../.."
for rep in 1 2; do
  for tag in "$@"; do
    echo -n "$tag "
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 60 python tools/diag/sustained_rollout.py 20,1000 full4 2>&1 | grep -v amdgpu.ids | tr '\n' ' ' || exit 1
    echo
  done
done
