#!/bin/bash
# One gpurun call's worth of evidence (run on the MI355X box from the repo root):
#   gpurun --timeout 1100 -- bash tools/gpu_round.sh [tag]
# GPU parity tests, smoke, the bench line, the rocprofv3 kernel-trace summary of
# the same bench command (config-4 DQN leg included: the round-2 exception
# under kernel tracing and its fixes are in DESIGN.md section 6; the DQN step
# is also traced on its own below), and two separate PMC passes (FETCH_SIZE, WRITE_SIZE)
# over k_rollout at the bench shape.  Every GPU step has its own time limit
# and the steps are chained with && so the first failure ends the call.
set -o pipefail
TAG=${1:-r01}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[gpu_round] $(date +%T) pytest -m gpu"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  && echo "pytest rc=0" >> "$OUT/pytest_gpu.log" \
  && echo "[gpu_round] $(date +%T) smoke" \
  && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  && echo "[gpu_round] $(date +%T) bench" \
  && timeout -k 10 300 python bench.py > "$OUT/bench_n1.json" 2> "$OUT/bench_n1.err" \
  && echo "[gpu_round] $(date +%T) rocprof kernel trace" \
  && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/rocprof" -o bench -- python3 "$ROOT/bench.py" --no-cpu-baseline \
        > "$OUT/rocprof_bench.log" 2>&1) \
  && echo "[gpu_round] $(date +%T) pmc FETCH_SIZE" \
  && (cd /tmp && timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv \
        -d "$OUT/pmc/fetch" -o pmc -- python3 "$ROOT/tools/pmc_target.py" --plies 1000 --launches 3 > "$OUT/pmc_fetch.log" 2>&1) \
  && echo "[gpu_round] $(date +%T) pmc WRITE_SIZE" \
  && (cd /tmp && timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv \
        -d "$OUT/pmc/write" -o pmc -- python3 "$ROOT/tools/pmc_target.py" --plies 1000 --launches 3 > "$OUT/pmc_write.log" 2>&1) \
  && python3 tools/pmc_summary.py --fetch "$OUT/pmc/fetch" --write "$OUT/pmc/write" --plies 1000 \
        --out "$OUT/pmc_k_rollout.json" \
  && echo "[gpu_round] $(date +%T) pmc FETCH_SIZE full4" \
  && (cd /tmp && timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv \
        -d "$OUT/pmc_full/fetch" -o pmc -- python3 "$ROOT/tools/pmc_target.py" --rules full4 --plies 1000 --launches 3 \
        > "$OUT/pmc_full_fetch.log" 2>&1) \
  && echo "[gpu_round] $(date +%T) pmc WRITE_SIZE full4" \
  && (cd /tmp && timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv \
        -d "$OUT/pmc_full/write" -o pmc -- python3 "$ROOT/tools/pmc_target.py" --rules full4 --plies 1000 --launches 3 \
        > "$OUT/pmc_full_write.log" 2>&1) \
  && python3 tools/pmc_summary.py --fetch "$OUT/pmc_full/fetch" --write "$OUT/pmc_full/write" \
        --kernel "k_rollout_wave<true>" --bytes-per-ply 118 --plies 1000 --out "$OUT/pmc_k_rollout_full.json" \
  && echo "[gpu_round] $(date +%T) bench --rules full4" \
  && timeout -k 10 300 python bench.py --rules full4 --no-cpu-baseline > "$OUT/bench_full4.json" 2> "$OUT/bench_full4.err" \
  && echo "[gpu_round] $(date +%T) rocprof kernel trace full4" \
  && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/rocprof_full4" -o bench -- python3 "$ROOT/bench.py" --rules full4 --no-cpu-baseline \
        > "$OUT/rocprof_full4.log" 2>&1) \
  && echo "[gpu_round] $(date +%T) rocprof kernel trace dqn (config 4, graph replay)" \
  && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/rocprof_dqn" -o dqn -- python3 "$ROOT/tools/dqn_target.py" 65536 20 \
        > "$OUT/rocprof_dqn.log" 2>&1) \
  && echo "[gpu_round] $(date +%T) done"
rc=$?
echo "[gpu_round] rc=$rc"
tail -3 "$OUT/pytest_gpu.log" 2>/dev/null
cat "$OUT/bench_n1.json" "$OUT/bench_full4.json" 2>/dev/null
exit $rc
