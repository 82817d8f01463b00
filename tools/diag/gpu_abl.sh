#!/bin/bash
# DIAGNOSTIC: FULL4 ablation timings for tools/diag/build/libnarde_abl<k>.so,
# k given on the command line (build them with -DNARDE_DIAG_ABLATE=k).
set -o pipefail
cd "$(dirname "$0")/../.."
for v in "$@"; do
  for dm in all36 nodoubles; do
    NARDE_LIB=$PWD/tools/diag/build/libnarde_abl$v.so timeout -k 10 120 python tools/diag/time_rollout.py 65536 full4 $dm 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
