#!/bin/bash
# round 5, call W: what scalar instructions and branches cost one wave
# between its VALU instructions (tools/issue_probe.py --scalar)
set -o pipefail
OUT=gpurun_out/r05w
mkdir -p $OUT
timeout -k 10 120 python3 tools/issue_probe.py --scalar --iters 20000 --out $OUT/scalar.json > $OUT/scalar.log 2>&1
rc=$?
tail -2 $OUT/scalar.log
echo "[r05w] rc=$rc"
exit $rc
