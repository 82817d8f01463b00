#!/bin/bash
# round 5, call M: k_step<true> per-wave cycles by kind of turn (kclk build:
# tools/diag/build_patch.sh kclk ... s_memtime around the ply in k_step<true>)
set -o pipefail
OUT=gpurun_out/r05m
mkdir -p $OUT
export TMPDIR=/tmp
echo "[r05m] $(date +%T) kstep clock"
NARDE_LIB=$PWD/tools/diag/build/libnarde_kclk.so timeout -k 10 300 python tools/diag/kstep_full_clock.py > $OUT/kstep_clock.json 2> $OUT/kstep_clock.err
rc=$?
cat $OUT/kstep_clock.json; tail -3 $OUT/kstep_clock.err
echo "[r05m] rc=$rc"
exit $rc
