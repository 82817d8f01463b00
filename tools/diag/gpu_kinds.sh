#!/bin/bash
# DIAGNOSTIC (round 4): FULL4 cost by turn kind -- all 36 rolls, no doubles,
# doubles only (libnarde_dblonly: the 'nodoubles' law patched to doubles),
# sustained launches of 20 and 1000 plies.
set -o pipefail
cd "$(dirname "$0")/../.."
for rep in 1 2; do
for spec in head:all36 head:nodoubles dblonly:nodoubles; do
  tag=${spec%%:*}; dm=${spec##*:}
  echo -n "$tag $dm "
  NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 60 python tools/diag/sustained_rollout.py 20,1000 full4 $dm 2>&1 | grep -v amdgpu.ids | tr '\n' ' ' || exit 1
  echo
done
done
NARDE_LIB=$PWD/tools/diag/build/libnarde_head.so timeout -k 5 60 python tools/diag/sustained_rollout.py 20,1000 ref2 all36 2>&1 | grep -v amdgpu.ids
