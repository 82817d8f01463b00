#!/bin/bash
# DIAGNOSTIC (round 4): FULL4 rollouts (outputs) and self-play (stats only)
# at 20 / 100 / 1000 plies per launch for libnarde_<tag>.so builds,
# alternating, 2 rounds.
set -o pipefail
cd "$(dirname "$0")/../.."
for rep in 1 2; do
  for tag in "$@"; do
    for s in sustained_rollout.py sustained_selfplay.py; do
      echo -n "$tag $s "
      NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 90 python tools/diag/$s 20,100,1000 full4 2>&1 | grep -v amdgpu.ids | tr '\n' ' ' || exit 1
      echo
    done
  done
done
