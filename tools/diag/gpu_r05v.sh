#!/bin/bash
# round 5, call V: where the rollouts' non-VALU time goes -- two SQ passes
# (<= 8 SQ counters each, separate rocprofv3 runs, no tracing) over 20-ply
# FULL4 and REF2 launches
set -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r05v
mkdir -p $OUT
export TMPDIR=/tmp
A="SQ_WAVE_CYCLES SQ_INSTS SQ_INSTS_BRANCH SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_IFETCH"
B="SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_IFETCH_LEVEL"
run() {  # rules kernel pass counters
  echo "[r05v] $(date +%T) $1 $3" \
  && (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $4 --output-format csv -d "$OUT/$1_$3" -o sq \
        -- python3 "$ROOT/tools/pmc_target.py" --rules "$1" --plies 20 --launches 5 > "$OUT/$1_$3.log" 2>&1) \
  && python3 tools/diag/sq_breakdown.py "$OUT/$1_$3" "$2" 20 > "$OUT/$1_$3.json" && cat "$OUT/$1_$3.json"
}
run full4 "k_rollout_pp_full<true, true>" A "$A" \
  && run full4 "k_rollout_pp_full<true, true>" B "$B" \
  && run ref2 "k_rollout_pc<true, true>" A "$A" \
  && run ref2 "k_rollout_pc<true, true>" B "$B"
rc=$?
echo "[r05v] rc=$rc"
exit $rc
