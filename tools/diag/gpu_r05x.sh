#!/bin/bash
# round 5, call X: the FULL4 producer's own instruction count -- SQ pass over
# statistics-only launches (k_rollout_pp_full<false, false>: the consumer
# only draws), 20 and 1,000 plies
set -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r05x
mkdir -p $OUT
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS"
for P in 20 1000; do
  echo "[r05x] $(date +%T) stats-only $P" \
  && (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$OUT/s$P" -o sq \
        -- python3 "$ROOT/tools/pmc_target.py" --rules full4 --plies $P --launches 4 --stats-only > "$OUT/s$P.log" 2>&1) \
  && python3 tools/diag/sq_breakdown.py "$OUT/s$P" "k_rollout_pp_full<false, false>" $P > "$OUT/s$P.json" && cat "$OUT/s$P.json" || exit 1
done
echo "[r05x] rc=0"
