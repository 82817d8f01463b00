#!/bin/bash
# DIAGNOSTIC (round 4): A/B of libnarde_<tag>.so builds in one call --
# FULL4 and REF2 sustained 20 / 1000-ply rollouts and the API kernels,
# alternating, 2 rounds.
set -o pipefail
cd "$(dirname "$0")/../.."
for rep in 1 2; do
  for tag in "$@"; do
    for rules in full4 ref2; do
      echo -n "$tag $rules "
      NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 60 python tools/diag/sustained_rollout.py 20,1000 $rules 2>&1 | grep -v amdgpu.ids | tr '\n' ' ' || exit 1
      echo
    done
    echo -n "$tag api "
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 60 python tools/api_target.py --reps 200 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
