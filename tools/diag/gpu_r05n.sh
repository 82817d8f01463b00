#!/bin/bash
# round 5, call N: k_step<true> per-wave cycles by kind of turn, product turn
# and two ablations (tools/diag/build_kclk.sh)
set -o pipefail
OUT=gpurun_out/r05n
mkdir -p $OUT
export TMPDIR=/tmp
for tag in kclk kclk_nolate kclk_noroot; do
  echo "[r05n] $(date +%T) $tag"
  NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 300 python tools/diag/kstep_full_clock.py > $OUT/$tag.json 2> $OUT/$tag.err || exit 1
  cat $OUT/$tag.json
done
echo "[r05n] rc=0"
