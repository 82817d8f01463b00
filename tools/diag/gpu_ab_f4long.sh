#!/bin/bash
# DIAGNOSTIC: FULL4 sustained 1,000-ply and 100-ply rates of
# tools/diag/build/libnarde_<tag>.so variants, three alternating rounds, one box.
set -o pipefail
for rep in 1 2 3; do
  for tag in "$@"; do
    echo -n "$tag "
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 90 python tools/diag/sustained_rollout.py 1000,100 full4 2>/dev/null \
      | python3 -c "import sys,json; print(' '.join(str(json.loads(l)['ms_per_100_plies']) for l in sys.stdin))" || exit 1
  done
done
