#!/bin/bash
# DIAGNOSTIC: sustained rates at P plies per launch (default 20: the
# driver's bench shape) for tools/diag/build/libnarde_<tag>.so, both rules.
set -o pipefail
cd "$(dirname "$0")/../.."
P=${P:-20}
for tag in "$@"; do
  for rules in ref2 full4; do
    echo -n "$tag "
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 45 python tools/diag/sustained_rollout.py $P $rules 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
