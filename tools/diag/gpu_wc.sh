#!/bin/bash
# DIAGNOSTIC: per-wave lifetimes (wave_clock.py, 20-ply FULL4 launches) and
# sustained 20/40-ply FULL4 rates of tools/diag/build/libnarde_<tag>.so
# variants, one box.   tools/diag/gpu_wc.sh <outdir> <tag>...
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for t in "$@"; do timeout -k 10 120 python tools/diag/wave_clock.py $t 20 > $OUT/$t.jsonl || exit 1; done
for t in "$@"; do
  echo -n "$t "
  NARDE_LIB=$PWD/tools/diag/build/libnarde_$t.so timeout -k 10 90 python tools/diag/sustained_rollout.py 20,40 full4 2>/dev/null \
    | python3 -c "import sys,json; print(' '.join(str(json.loads(l)['ms_per_100_plies']) for l in sys.stdin))" || exit 1
done
