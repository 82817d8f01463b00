#!/bin/bash
# The driver's own bench invocation (python bench.py --gpus 1 --steps 20
# --warmup 5: ONE 20-ply launch timed) with its evidence, on the MI355X box
# from the repo root:
#   gpurun --timeout 900 -- bash tools/gpu_driver_shape.sh <tag> [pytest args]
# GPU tests (unless SKIP_TESTS=1), smoke, the bench line at the driver's
# shape, the rocprofv3 kernel-trace summary of that same command, and the two
# PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) over k_rollout_pc at 20
# plies per launch.  Each GPU step has its own time limit; a test FAILURE
# (pytest rc 1) still lets the measurements run, anything worse (a fault, a
# timeout, an abort) ends the call.
set -o pipefail
TAG=${1:?tag}
shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
S=${STEPS:-20}
W=${WARMUP:-5}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  echo "[gpu] $(date +%T) pytest -m gpu $*"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
    > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  echo "pytest rc=$rc" >> "$OUT/pytest_gpu.log"
  tail -4 "$OUT/pytest_gpu.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu] pytest rc=$rc: stop"; exit $rc; fi
  echo "[gpu] $(date +%T) smoke"
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
fi
echo "[gpu] $(date +%T) bench --steps $S --warmup $W"
timeout -k 10 300 python bench.py --gpus 1 --steps $S --warmup $W > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" \
  && echo "[gpu] $(date +%T) rocprof kernel trace (same command)" \
  && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/rocprof_driver" -o bench -- python3 "$ROOT/bench.py" --gpus 1 --steps $S --warmup $W --no-cpu-baseline \
        > "$OUT/rocprof_driver.log" 2>&1) \
  && echo "[gpu] $(date +%T) pmc FETCH_SIZE at $S plies" \
  && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv \
        -d "$OUT/pmc$S/fetch" -o pmc -- python3 "$ROOT/tools/pmc_target.py" --plies $S --launches 5 > "$OUT/pmc_fetch.log" 2>&1) \
  && echo "[gpu] $(date +%T) pmc WRITE_SIZE at $S plies" \
  && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv \
        -d "$OUT/pmc$S/write" -o pmc -- python3 "$ROOT/tools/pmc_target.py" --plies $S --launches 5 > "$OUT/pmc_write.log" 2>&1) \
  && python3 tools/pmc_summary.py --fetch "$OUT/pmc$S/fetch" --write "$OUT/pmc$S/write" --plies $S \
        --out "$OUT/pmc_k_rollout_p$S.json" \
  && echo "[gpu] $(date +%T) done"
rc=$?
echo "[gpu] rc=$rc"
cat "$OUT/bench_driver.json" 2>/dev/null
exit $rc
