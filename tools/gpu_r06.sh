#!/bin/bash
# Round 6's GPU calls (run on the MI355X box from the repo root):
#   gpurun -- bash tools/gpu_r06.sh TAG PHASE
# Every GPU step has its own time limit, the steps are chained with &&.
set -o pipefail
TAG=${1:-r06}
PHASE=${2:-parity}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
case "$PHASE" in
parity)  # the full-batch parity tests and the self-checking bench line
  timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_full4.py -m gpu > "$OUT/pytest.log" 2>&1 \
    && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" \
    && timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
  rc=$?; tail -3 "$OUT/pytest.log"; exit $rc ;;
drv)  # the driver's command, with and without the checker leg, alternating
  for k in 1 2 3; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/drv_chk_$k.json" 2> "$OUT/drv_chk_$k.err" \
      && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-parity-check --no-cpu-baseline \
           > "$OUT/drv_nochk_$k.json" 2> "$OUT/drv_nochk_$k.err" || exit 1
  done ;;
clock)  # per-wave stamps of the driver's timed REF2 launch (tools/diag/build_clock.py, built beforehand)
  for P in 20 1000; do
    timeout -k 10 120 python tools/diag/clock_anatomy.py $P x "$OUT/clock_p$P.npy" > "$OUT/clock_p$P.json" 2> "$OUT/clock_p$P.err" || exit 1
  done ;;
pp)  # FULL4 rollout per-ply clocks by kind of turn (tools/diag/build_ppclock.py, built beforehand)
  timeout -k 10 180 python tools/diag/pp_phase.py > "$OUT/pp_phase.json" 2> "$OUT/pp_phase.err" ;;
dqn)  # the DQN learner's tests, then a graph-replayed trace of the driver (both learner forms)
  timeout -k 10 400 $T tests/test_gpu_dqn.py -m gpu > "$OUT/pytest_dqn.log" 2>&1 \
    && (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/dqn_trace" -o dqn \
          -- python3 "$ROOT/tools/dqn_target.py" 65536 20 > "$ROOT/$OUT/dqn_trace.log" 2>&1) \
    && (cd /tmp && NARDE_ONE_LAUNCH=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/dqn_trace_r5" -o dqn \
          -- python3 "$ROOT/tools/dqn_target.py" 65536 20 > "$ROOT/$OUT/dqn_trace_r5.log" 2>&1) \
    && timeout -k 10 120 python3 tools/dqn_target.py 65536 30 > "$OUT/dqn_time.log" 2>&1 \
    && NARDE_ONE_LAUNCH=0 timeout -k 10 120 python3 tools/dqn_target.py 65536 30 >> "$OUT/dqn_time.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest_dqn.log"; cat "$OUT/dqn_time.log"; exit $rc ;;
ab)  # sustained FULL4 20 / 1,000-ply rollouts of tools/diag/build/libnarde_<tag>.so ($TAGS), 2 rounds
  timeout -k 10 600 bash tools/diag/gpu_sus20.sh $TAGS > "$OUT/sus20.log" 2>&1
  rc=$?; cat "$OUT/sus20.log"; exit $rc ;;
plan)  # the driver's command with the pre-bound timed launch and without it, alternating
  timeout -k 10 300 $T tests/test_gpu_parity.py -m gpu -k "plan or totals_rows" > "$OUT/pytest_plan.log" 2>&1 || exit 1
  for k in 1 2 3 4; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/plan1_$k.json" 2> "$OUT/plan1_$k.err" \
      && NARDE_ROLLOUT_PLAN=0 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
           > "$OUT/plan0_$k.json" 2> "$OUT/plan0_$k.err" || exit 1
  done ;;
single)  # one 20-ply launch after an idle synchronize (the driver's shape), per library in $TAGS, 2 rounds
  for rep in 1 2; do for tag in $TAGS; do
    echo -n "$tag ref2 "
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so NARDE_EVENTS=nofence timeout -k 5 120 python tools/diag/single_launch.py 20 2>/dev/null | tail -1 || exit 1
    [ "${REF2_ONLY:-0}" = 1 ] && continue
    echo -n "$tag full4 "
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so NARDE_EVENTS=nofence timeout -k 5 120 python tools/diag/single_launch.py full4 20 2>/dev/null | tail -1 || exit 1
  done; done > "$OUT/single.log" 2>&1
  rc=$?; cat "$OUT/single.log"; exit $rc ;;
api)  # the API kernels (tools/api_target.py, graph-replayed and eager) per library in $TAGS, 2 rounds, then the tests on the last
  for rep in 1 2; do for tag in $TAGS; do
    echo -n "$tag "
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 120 python tools/api_target.py 2>/dev/null | tail -1 || exit 1
  done; done > "$OUT/api_ab.log" 2>&1 || { cat "$OUT/api_ab.log"; exit 1; }
  for tag in $TAGS; do
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_full4.py tests/test_gpu_facade.py -m gpu > "$OUT/pytest_$tag.log" 2>&1
    echo "$tag tests rc=$? $(tail -1 $OUT/pytest_$tag.log)" >> "$OUT/api_ab.log"
  done
  cat "$OUT/api_ab.log" ;;
sus)  # sustained REF2 and FULL4 rollouts at $PLIES plies per launch per library in $TAGS, 2 rounds
  for rep in 1 2; do for tag in $TAGS; do for rules in ref2 full4; do
    echo -n "$tag $rules "
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 5 120 python tools/diag/sustained_rollout.py ${PLIES:-100,1000} $rules 2>/dev/null | python3 -c "import sys,json; print(' '.join(str(json.loads(l)['plies_per_launch'])+':'+str(json.loads(l)['ms_per_100_plies']) for l in sys.stdin))" || exit 1
  done; done; done > "$OUT/sus.log" 2>&1
  rc=$?; cat "$OUT/sus.log"; exit $rc ;;
libab)  # bench.py's default (1,000-ply) and driver lines per library in $TAGS, alternating, 2 rounds
  for rep in 1 2; do for tag in $TAGS; do
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 300 python bench.py --no-cpu-baseline \
      > "$OUT/def_${tag}_$rep.json" 2> "$OUT/def_${tag}_$rep.err" \
    && NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 \
      --no-cpu-baseline > "$OUT/drv_${tag}_$rep.json" 2> "$OUT/drv_${tag}_$rep.err" || exit 1
  done; done ;;
libdqn)  # the DQN tests on the product, then the driver timed with libnarde_$BASE.so and the product, alternating, then traced
  timeout -k 10 400 $T tests/test_gpu_dqn.py -m gpu > "$OUT/pytest_dqn.log" 2>&1 || { tail -30 "$OUT/pytest_dqn.log"; exit 1; }
  tail -1 "$OUT/pytest_dqn.log"
  for rep in 1 2 3; do
    echo -n "$BASE " >> "$OUT/dqn_time.log"
    NARDE_LIB=$PWD/tools/diag/build/libnarde_$BASE.so timeout -k 10 120 python3 tools/dqn_target.py 65536 30 2>/dev/null >> "$OUT/dqn_time.log" || exit 1
    echo -n "product " >> "$OUT/dqn_time.log"
    timeout -k 10 120 python3 tools/dqn_target.py 65536 30 2>/dev/null >> "$OUT/dqn_time.log" || exit 1
  done
  cat "$OUT/dqn_time.log"
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/dqn_trace" -o dqn \
      -- python3 "$ROOT/tools/dqn_target.py" 65536 20 > "$ROOT/$OUT/dqn_trace.log" 2>&1) \
    && python3 tools/dqn_breakdown.py "$OUT/dqn_trace" --out "$OUT/dqn_breakdown.json" > /dev/null ;;
*) echo "unknown phase $PHASE"; exit 2 ;;
esac
