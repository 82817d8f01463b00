#!/bin/bash
# round 5, call D: the issue probe with compare/select pairs; PMC traffic and
# SQ issue passes of the FULL4 pairwise kernel (20 and 1,000 plies); the API
# kernels' trace (graph-replayed and eager)
set -o pipefail
TAG=r05d
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"
pmc_pair() {  # rules plies kernel bytes_per_ply name
  local rules=$1 plies=$2 kernel=$3 bpp=$4 name=$5 launches=3
  [ "$plies" -lt 100 ] && launches=5
  echo "[$TAG] $(date +%T) pmc $name" \
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
  echo "[$TAG] $(date +%T) sq $name" \
  && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/$name" -o sq \
        -- python3 "$ROOT/tools/pmc_target.py" --rules "$rules" --plies "$plies" --launches $launches \
        > "$OUT/$name.log" 2>&1) \
  && python3 tools/sq_summary.py --dir "$OUT/$name" --kernel "$kernel" --plies "$plies" --out "$OUT/$name.json"
}
echo "[$TAG] $(date +%T) pytest -m gpu" \
  && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  && echo "[$TAG] $(date +%T) issue probe" \
  && timeout -k 10 300 python3 tools/issue_probe.py --out $OUT/issue_probe.json > $OUT/issue_probe.log 2>&1 \
  && (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
        --output-format csv -d $OUT/issue_probe_sq -o sq -- python3 $ROOT/tools/issue_probe.py --iters 2000 \
        > $OUT/issue_probe_sq.log 2>&1) \
  && pmc_pair full4 20 "k_rollout_pp_full<true, true>" 118 pmc_k_rollout_full_p20 \
  && pmc_pair full4 1000 "k_rollout_pp_full<true, false>" 118 pmc_k_rollout_full \
  && sq_pass full4 20 "k_rollout_pp_full<true, true>" sq_k_rollout_full_p20 \
  && sq_pass full4 1000 "k_rollout_pp_full<true, false>" sq_k_rollout_full_p1000 \
  && echo "[$TAG] $(date +%T) api kernels (timed, traced)" \
  && timeout -k 10 120 python3 tools/api_target.py > "$OUT/api.json" \
  && (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/api_trace" -o api \
        -- python3 "$ROOT/tools/api_target.py" > "$OUT/api_trace.log" 2>&1)
rc=$?
tail -3 $OUT/pytest_gpu.log; tail -1 $OUT/issue_probe.log | cut -c1-200; cat $OUT/api.json
grep -ho '"traffic_over_algorithmic": [0-9.]*\|"valu_per_env_ply": [0-9.]*\|"frac_at_profiled_duration": [0-9.]*' $OUT/*.json
echo "[$TAG] rc=$rc"
exit $rc
