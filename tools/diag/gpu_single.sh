#!/bin/bash
# DIAGNOSTIC: single-launch anatomy (tools/diag/single_launch.py) for each
# tools/diag/build/libnarde_<tag>.so named, in one call on one box.
#   gpurun -- bash tools/diag/gpu_single.sh <tag>... (RULES=full4 PLIES="1 20")
set -o pipefail
cd "$(dirname "$0")/../.."
for tag in "$@"; do
  NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 90 python tools/diag/single_launch.py ${RULES:-ref2} ${PLIES:-} 2>&1 \
    | grep -v amdgpu.ids || exit 1
done
