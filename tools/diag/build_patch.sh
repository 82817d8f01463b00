#!/bin/bash
# DIAGNOSTIC: build a libnarde.so variant from the working tree with a
# temporary source patch (python snippet editing the scratch copy):
#   tools/diag/build_patch.sh <tag> '<file>' '<old>' '<new>' [<file> <old> <new> ...]
# Output: tools/diag/build/libnarde_<tag>.so.  The product source is untouched.
set -euo pipefail
cd "$(dirname "$0")/../.."
tag=$1; shift
tmp=$(mktemp -d)
cp -r gym-narde_amd include "$tmp/"
python3 - "$tmp" "$@" <<'PY'
import sys
root, args = sys.argv[1], sys.argv[2:]
for i in range(0, len(args), 3):
    f, old, new = args[i:i + 3]
    p = f"{root}/gym-narde_amd/csrc/{f}"
    s = open(p).read()
    assert old in s, (f, old)
    open(p, "w").write(s.replace(old, new))
PY
mkdir -p tools/diag/build
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared \
  -o tools/diag/build/libnarde_$tag.so "$tmp/gym-narde_amd/csrc/narde.hip" "$tmp/gym-narde_amd/csrc/dqn_learner.hip"
if [ "${ASM:-0}" = 1 ]; then  # the device assembly too (tools/diag/build/libnarde_<tag>.s)
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -S --cuda-device-only \
    -o tools/diag/build/libnarde_$tag.s "$tmp/gym-narde_amd/csrc/narde.hip" 2>/dev/null
fi
rm -rf "$tmp"
echo "built tools/diag/build/libnarde_$tag.so"
