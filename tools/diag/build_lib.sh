#!/bin/bash
# DIAGNOSTIC: build libnarde.so variants for A/B timing on the GPU box.
#   tools/diag/build_lib.sh <tag> [git-rev] [-D...]
# rev "WT" (default) = the working tree; any other rev = that commit's csrc
# (extracted with git archive).  Output: tools/diag/build/libnarde_<tag>.so
set -euo pipefail
cd "$(dirname "$0")/../.."
tag=$1; rev=${2:-WT}; shift $(( $# >= 2 ? 2 : 1 ))
mkdir -p tools/diag/build
if [ "$rev" = WT ]; then
  src=gym-narde_amd/csrc
else
  tmp=$(mktemp -d)
  git archive "$rev" gym-narde_amd/csrc include | tar -x -C "$tmp"
  src=$tmp/gym-narde_amd/csrc
fi
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared "$@" \
  -o tools/diag/build/libnarde_$tag.so "$src/narde.hip" "$src/dqn_learner.hip"
echo "built tools/diag/build/libnarde_$tag.so ($rev $*)"
