#!/bin/bash
# round 3: play-set tests, two driver-shape bench lines, SQ issue counters of
# the rollout kernels (FULL4 100 / 20 plies, REF2 20 plies), the REF2 clock
# anatomy at 20 plies.  DIAGNOSTIC.
set -o pipefail
OUT=gpurun_out/r03b; mkdir -p $OUT; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
CNT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"
echo "[r03b] $(date +%T) pytest play set" \
 && timeout -k 10 300 python -u -m pytest tests/test_gpu_play_set.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_play.log 2>&1 \
 && tail -2 $OUT/pytest_play.log \
 && echo "[r03b] $(date +%T) bench x2" \
 && timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench1.json 2> $OUT/bench1.err \
 && timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err \
 && python3 -c "import json;[print(json.load(open(f'$OUT/bench{i}.json'))['value'], json.load(open(f'$OUT/bench{i}.json'))['timed_region_host_us'], json.load(open(f'$OUT/bench{i}.json'))['roofline']['kernel_ms']) for i in (1,2)]" \
 && echo "[r03b] $(date +%T) sq full4 100" \
 && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d $R/$OUT/sq_full4_100 -o sq -- python3 $R/tools/diag/sq_target.py full4 100 > $R/$OUT/sq1.log 2>&1) \
 && python3 tools/diag/sq_summary.py $OUT/sq_full4_100 \
 && echo "[r03b] $(date +%T) sq full4 20" \
 && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d $R/$OUT/sq_full4_20 -o sq -- python3 $R/tools/diag/sq_target.py full4 20 > $R/$OUT/sq2.log 2>&1) \
 && python3 tools/diag/sq_summary.py $OUT/sq_full4_20 \
 && echo "[r03b] $(date +%T) sq ref2 20" \
 && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d $R/$OUT/sq_ref2_20 -o sq -- python3 $R/tools/diag/sq_target.py ref2 20 > $R/$OUT/sq3.log 2>&1) \
 && python3 tools/diag/sq_summary.py $OUT/sq_ref2_20 \
 && echo "[r03b] $(date +%T) clock anatomy" \
 && timeout -k 10 120 python tools/diag/clock_anatomy.py 20 > $OUT/clock20.json 2> $OUT/clock20.err \
 && cat $OUT/clock20.json && echo "[r03b] $(date +%T) done"
