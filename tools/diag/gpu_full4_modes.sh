#!/bin/bash
# DIAGNOSTIC: sustained FULL4 rate, all 36 rolls and non-doubles only, for
# each tools/diag/build/libnarde_<tag>.so named on the command line.
set -o pipefail
for tag in "$@"; do
  for dm in all36 nodoubles; do
    echo -n "$tag "
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 120 python tools/diag/sustained_rollout.py 1000 full4 $dm 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
