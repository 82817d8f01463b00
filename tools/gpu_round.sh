#!/bin/bash
# One round's GPU evidence, in two calls (run on the MI355X box from the repo root):
#   gpurun --timeout 1100 -- bash tools/gpu_round.sh TAG run    # tests, smoke, bench lines, kernel traces
#   gpurun --timeout 1100 -- bash tools/gpu_round.sh TAG pmc    # PMC traffic + SQ issue passes, API kernels
# Every GPU step has its own time limit and the steps are chained with &&,
# so the first failure ends the call.  PMC / SQ passes are separate
# rocprofv3 runs, never combined with tracing domains (MI355X_MICROARCH.md).
set -o pipefail
TAG=${1:-r05}
PHASE=${2:-run}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"

pmc_pair() {  # rules plies kernel bytes_per_ply name
  local rules=$1 plies=$2 kernel=$3 bpp=$4 name=$5 launches=3
  [ "$plies" -lt 100 ] && launches=5
  echo "[gpu_round] $(date +%T) pmc $name" \
  && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/$name/fetch" -o pmc \
        -- python3 "$ROOT/tools/pmc_target.py" --rules "$rules" --plies "$plies" --launches $launches \
        > "$OUT/${name}_fetch.log" 2>&1) \
  && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/$name/write" -o pmc \
        -- python3 "$ROOT/tools/pmc_target.py" --rules "$rules" --plies "$plies" --launches $launches \
        > "$OUT/${name}_write.log" 2>&1) \
  && python3 tools/pmc_summary.py --fetch "$OUT/$name/fetch" --write "$OUT/$name/write" \
        --kernel "$kernel" --bytes-per-ply "$bpp" --plies "$plies" --out "$OUT/$name.json"
}

sq_pass() {  # rules plies kernel name
  local rules=$1 plies=$2 kernel=$3 name=$4 launches=3
  [ "$plies" -lt 100 ] && launches=5
  echo "[gpu_round] $(date +%T) sq $name" \
  && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/$name" -o sq \
        -- python3 "$ROOT/tools/pmc_target.py" --rules "$rules" --plies "$plies" --launches $launches \
        > "$OUT/$name.log" 2>&1) \
  && python3 tools/sq_summary.py --dir "$OUT/$name" --kernel "$kernel" --plies "$plies" --out "$OUT/$name.json"
}

if [ "$PHASE" = run ]; then
  echo "[gpu_round] $(date +%T) pytest -m gpu"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    && echo "pytest rc=0" >> "$OUT/pytest_gpu.log" \
    && echo "[gpu_round] $(date +%T) smoke" \
    && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    && echo "[gpu_round] $(date +%T) bench (driver shape x3)" \
    && for k in 1 2 3; do timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 \
         > "$OUT/bench_driver_$k.json" 2> "$OUT/bench_driver_$k.err" || exit 1; done \
    && echo "[gpu_round] $(date +%T) bench (default)" \
    && timeout -k 10 300 python bench.py > "$OUT/bench_n1.json" 2> "$OUT/bench_n1.err" \
    && echo "[gpu_round] $(date +%T) bench --rules full4 (driver shape, default)" \
    && timeout -k 10 300 python bench.py --rules full4 --steps 20 --warmup 5 --no-cpu-baseline \
         > "$OUT/bench_full4_driver.json" 2> "$OUT/bench_full4_driver.err" \
    && timeout -k 10 300 python bench.py --rules full4 --no-cpu-baseline > "$OUT/bench_full4.json" 2> "$OUT/bench_full4.err" \
    && echo "[gpu_round] $(date +%T) rocprof kernel trace (driver shape)" \
    && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/rocprof_driver" -o bench -- python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
          > "$OUT/rocprof_driver.log" 2>&1) \
    && echo "[gpu_round] $(date +%T) rocprof kernel trace (default bench)" \
    && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/rocprof_bench" -o bench -- python3 "$ROOT/bench.py" --no-cpu-baseline \
          > "$OUT/rocprof_bench.log" 2>&1) \
    && echo "[gpu_round] $(date +%T) done"
  rc=$?
  tail -3 "$OUT/pytest_gpu.log" 2>/dev/null
  cat "$OUT/bench_driver_1.json" 2>/dev/null | tail -1 | cut -c1-400
else
  pmc_pair ref2 20 "k_rollout_pc<true>" 114 pmc_k_rollout_p20 \
    && pmc_pair ref2 1000 "k_rollout_pc<true>" 114 pmc_k_rollout \
    && pmc_pair full4 20 "k_rollout_pp_full<true>" 118 pmc_k_rollout_full_p20 \
    && pmc_pair full4 1000 "k_rollout_pp_full<true>" 118 pmc_k_rollout_full \
    && sq_pass ref2 20 "k_rollout_pc<true>" sq_k_rollout_p20 \
    && sq_pass full4 20 "k_rollout_pp_full<true>" sq_k_rollout_full_p20 \
    && sq_pass ref2 1000 "k_rollout_pc<true>" sq_k_rollout_p1000 \
    && sq_pass full4 1000 "k_rollout_pp_full<true>" sq_k_rollout_full_p1000 \
    && echo "[gpu_round] $(date +%T) DQN driver (configs[3]) traced" \
    && (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/dqn_trace" -o dqn \
          -- python3 "$ROOT/tools/dqn_target.py" 65536 20 > "$OUT/dqn_trace.log" 2>&1) \
    && python3 tools/dqn_breakdown.py "$OUT/dqn_trace" --out "$OUT/dqn_breakdown.json" \
    && echo "[gpu_round] $(date +%T) api kernels (timed, traced)" \
    && timeout -k 10 120 python3 tools/api_target.py > "$OUT/api.json" \
    && (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/api_trace" -o api \
          -- python3 "$ROOT/tools/api_target.py" > "$OUT/api_trace.log" 2>&1) \
    && echo "[gpu_round] $(date +%T) done"
  rc=$?
  cat "$OUT"/pmc_k_rollout*.json "$OUT"/sq_k_rollout*.json 2>/dev/null | grep -o '"traffic_over_algorithmic": [0-9.]*\|"frac_at_profiled_duration": [0-9.]*'
fi
echo "[gpu_round] rc=$rc"
exit $rc
