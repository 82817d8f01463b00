#!/bin/bash
# DIAGNOSTIC: host round trip of one 20-ply launch (tools/diag/single_launch.py)
# under HIP runtime settings, interleaved twice, one box.
set -o pipefail
cd "$(dirname "$0")/../.."
for rep in 1 2; do
  for setting in "base" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "AMD_DIRECT_DISPATCH=0"; do
    echo -n "$setting "
    if [ "$setting" = base ]; then
      timeout -k 5 90 python tools/diag/single_launch.py ref2 1 20 2>&1 | grep -v amdgpu.ids || exit 1
    else
      env "$setting" timeout -k 5 90 python tools/diag/single_launch.py ref2 1 20 2>&1 | grep -v amdgpu.ids || exit 1
    fi
  done
done
