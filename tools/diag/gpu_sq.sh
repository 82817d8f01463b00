#!/bin/bash
# SQ issue counters of the REF2 rollout kernels, both A/B builds. DIAGNOSTIC.
set -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/sq
mkdir -p "$OUT"
export TMPDIR=/tmp
CNT="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"
for v in 0 1; do
  (cd /tmp && NARDE_LIB=$ROOT/tools/diag/build/libnarde_pc$v.so timeout -k 10 240 rocprofv3 --pmc $CNT \
     --output-format csv -d "$OUT/pc$v" -o sq -- python3 "$ROOT/tools/diag/sq_target.py" > "$OUT/pc$v.log" 2>&1) || exit 1
  echo "== pc$v"; python3 tools/diag/sq_summary.py "$OUT/pc$v"
done
