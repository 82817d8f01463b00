#!/bin/bash
# DIAGNOSTIC: PMC FETCH_SIZE / WRITE_SIZE (separate passes) of the FULL4
# rollout for each tools/diag/build/libnarde_<tag>.so (1,000-ply launches).
set -o pipefail
cd "$(dirname "$0")/../.."
ROOT=$PWD
export TMPDIR=/tmp
for tag in "$@"; do
  OUT=$ROOT/gpurun_out/pmcf4_$tag
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && NARDE_LIB=$ROOT/tools/diag/build/libnarde_$tag.so timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv \
       -d "$OUT/$c" -o pmc -- python3 "$ROOT/tools/pmc_target.py" --rules full4 --plies 1000 --launches 2 > "$OUT.$c.log" 2>&1) || exit 1
  done
  python3 tools/pmc_summary.py --fetch "$OUT/FETCH_SIZE" --write "$OUT/WRITE_SIZE" --kernel "k_rollout_full<true>" \
    --bytes-per-ply 118 --plies 1000 --out "$OUT.json" && echo "$tag $(cat $OUT.json)"
done
