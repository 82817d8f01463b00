#!/bin/bash
# DIAGNOSTIC: REF2 store-policy A/B: single 20-ply launches and sustained
# 1,000-ply launches for each tools/diag/build/libnarde_<tag>.so named.
set -o pipefail
cd "$(dirname "$0")/../.."
for tag in "$@"; do
  NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 90 python tools/diag/single_launch.py ref2 ${PLIES:-5 20} 2>&1 | grep -v amdgpu.ids || exit 1
done
for tag in "$@"; do
  echo -n "$tag "
  NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 60 python tools/diag/sustained_rollout.py 20,1000 ref2 2>&1 | grep -v amdgpu.ids | tr '\n' ' ' || exit 1
  echo
done
