#!/bin/bash
# DIAGNOSTIC: FULL4 ablation timings (tools/diag/build/libnarde_abl<k>.so).
set -o pipefail
cd "$(dirname "$0")/../.."
for v in 0 1 2 4 7; do
  for dm in all36 nodoubles; do
    NARDE_LIB=$PWD/tools/diag/build/libnarde_abl$v.so timeout -k 10 120 python tools/diag/time_rollout.py 65536 full4 $dm 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
