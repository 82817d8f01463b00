#!/bin/bash
# round 5, call U: the SQ counters this box's rocprofv3 offers (names only)
set -o pipefail
OUT=$PWD/gpurun_out/r05u
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 120 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1
rc=$?
cd - > /dev/null
grep -o "SQ_[A-Z0-9_]*" $OUT/list_avail.txt | sort -u | tr '\n' ' ' | head -c 6000
echo
echo "[r05u] rc=$rc"
exit $rc
