#!/bin/bash
# DIAGNOSTIC: sustained FULL4 rollout (1,000 plies per launch) and stats-only
# rate for each tools/diag/build/libnarde_<tag>.so named on the command line.
set -o pipefail
cd "$(dirname "$0")/../.."
for tag in "$@"; do
  echo -n "$tag "
  NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 120 python tools/diag/sustained_rollout.py 1000 full4 2>&1 | grep -v amdgpu.ids || exit 1
done
