set -o pipefail
OUT=gpurun_out/r03a; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r03a] $(date +%T) pytest"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "[r03a] $(date +%T) totals diag" \
 && timeout -k 10 180 python tools/diag/totals_region.py 20 > $OUT/totals_region.json 2> $OUT/totals_region.err \
 && cat $OUT/totals_region.json \
 && echo "[r03a] $(date +%T) rocprof default bench with the DQN leg" \
 && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/rocprof_bench -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/rocprof_bench.log 2>&1) \
 && tail -c 600 $OUT/rocprof_bench.log && echo "[r03a] $(date +%T) done"
