#!/bin/bash
# DIAGNOSTIC: time the REF2 rollout for each tools/diag/build/libnarde_<tag>.so
# named on the command line, twice each, interleaved.
set -o pipefail
cd "$(dirname "$0")/../.."
for rep in 1 2; do
  for tag in "$@"; do
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 120 python tools/diag/time_rollout.py 65536 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
