#!/bin/bash
# DIAGNOSTIC: sustained REF2 rollout rate (1,000 plies per launch) for each
# tools/diag/build/libnarde_<tag>.so named on the command line, twice each.
set -o pipefail
cd "$(dirname "$0")/../.."
for rep in 1 2; do
  for tag in "$@"; do
    echo -n "$tag "
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 120 python tools/diag/sustained_rollout.py ${SUS_P:-1000} 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
