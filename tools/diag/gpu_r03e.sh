#!/bin/bash
# round 3: the full GPU test suite + smoke.
set -o pipefail
OUT=gpurun_out/r03e; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r03e] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -5
[ $rc -eq 0 ] || exit $rc
echo "[r03e] $(date +%T) smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "[r03e] $(date +%T) graph region"
timeout -k 10 150 python tools/diag/graph_region.py 20 > $OUT/graph_region.json 2> $OUT/graph_region.err; rc=$?; tail -3 $OUT/graph_region.err; cat $OUT/graph_region.json; exit $rc
