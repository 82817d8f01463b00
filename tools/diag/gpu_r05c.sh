#!/bin/bash
# round 5, call C: FULL4 pairwise producer/consumer rollout (k_rollout_pp_full):
# FULL4 GPU tests, sustained A/B (one-wave / barrier pc / pairwise pp), the
# driver-shape FULL4 bench line, the extended issue probe
set -o pipefail
OUT=gpurun_out/r05c
mkdir -p $OUT
export TMPDIR=/tmp
echo "[r05c] $(date +%T) full4 tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_full4.py tests/test_gpu_parity.py -k "full4 or rollout_writes" -x -v --timeout 300 --timeout-method thread > $OUT/full4_tests.log 2>&1 \
  && echo "[r05c] $(date +%T) sustained A/B" \
  && timeout -k 10 500 bash tools/diag/gpu_sus20.sh wave pc pp > $OUT/sus_ab.log 2>&1 \
  && echo "[r05c] $(date +%T) bench full4 driver shape" \
  && timeout -k 10 300 python bench.py --rules full4 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_full4_driver.json 2> $OUT/bench_full4_driver.err \
  && echo "[r05c] $(date +%T) api kernels A/B" \
  && for rep in 1 2; do for tag in ks_base ks_sl ks_nt ks_both; do echo -n "$tag "; NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 120 python tools/api_target.py 2>/dev/null | tail -1 || exit 1; done; done > $OUT/api_ab.log 2>&1 \
  && echo "[r05c] $(date +%T) issue probe" \
  && timeout -k 10 300 python3 tools/issue_probe.py --out $OUT/issue_probe.json > $OUT/issue_probe.log 2>&1 \
  && (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
        --output-format csv -d $GRAFT_REPO_ROOT/$OUT/issue_probe_sq -o sq -- python3 $GRAFT_REPO_ROOT/tools/issue_probe.py --iters 2000 \
        > $GRAFT_REPO_ROOT/$OUT/issue_probe_sq.log 2>&1)
rc=$?
tail -3 $OUT/full4_tests.log; cat $OUT/sus_ab.log; cat $OUT/api_ab.log; tail -c 300 $OUT/bench_full4_driver.json; tail -1 $OUT/issue_probe.log | cut -c1-300
echo "[r05c] rc=$rc"
exit $rc
