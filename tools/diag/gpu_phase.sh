#!/bin/bash
# DIAGNOSTIC (round 4): one 20-ply FULL4 launch by game phase
# (phase_time.py) for libnarde_<tag>.so builds.
set -o pipefail
cd "$(dirname "$0")/../.."
for tag in "$@"; do
  NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 120 python tools/diag/phase_time.py 0,40,60,70,80 2>&1 | grep -v amdgpu.ids || exit 1
done
