#!/bin/bash
# DIAGNOSTIC: sustained FULL4 stats-only and with-outputs rates of
# tools/diag/build/libnarde_<tag>.so for each tag (A/B inside one call).
set -o pipefail
cd "$(dirname "$0")/../.."
for tag in "$@"; do
  for s in sustained_selfplay.py sustained_rollout.py; do
    echo -n "$tag "
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 45 python tools/diag/$s 1000 full4 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
