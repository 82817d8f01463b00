#!/bin/bash
# DIAGNOSTIC (round 4): sustained REF2 and FULL4 rollouts at 20 and 1,000
# plies per launch for libnarde_<tag>.so builds, 2 rounds alternating.
set -o pipefail
cd "$(dirname "$0")/../.."
for rep in 1 2; do
  for tag in "$@"; do
    for rules in ref2 full4; do
      echo -n "$tag "
      NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 90 python tools/diag/sustained_rollout.py 20,1000 $rules 2>&1 | grep -v amdgpu.ids | tr '\n' ' ' || exit 1
      echo
    done
  done
done
