#!/bin/bash
# DIAGNOSTIC: does a second wave per SIMD add throughput? (single-wave kernel
# at 65,536 vs 131,072 envs) and the producer/consumer priority knob.
set -o pipefail
cd "$(dirname "$0")/../.."
B=tools/diag/build
for spec in "pc0 65536" "pc0 131072" "pc0 262144" "pc1 65536" "prio1 65536" "prio2 65536" "pc1 131072"; do
  set -- $spec
  NARDE_LIB=$PWD/$B/libnarde_$1.so timeout -k 10 120 python tools/diag/time_rollout.py $2 2>&1 | grep -v amdgpu.ids || exit 1
done
