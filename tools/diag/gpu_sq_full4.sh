#!/bin/bash
# SQ issue counters of the FULL4 rollout kernel for each
# tools/diag/build/libnarde_<tag>.so named on the command line. DIAGNOSTIC.
set -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/sqf
mkdir -p "$OUT"
export TMPDIR=/tmp
CNT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"
for v in "$@"; do
  (cd /tmp && NARDE_LIB=$ROOT/tools/diag/build/libnarde_$v.so timeout -s KILL 120 rocprofv3 --pmc $CNT \
     --output-format csv -d "$OUT/$v" -o sq -- python3 "$ROOT/tools/diag/sq_target.py" full4 > "$OUT/$v.log" 2>&1) || exit 1
  echo "== $v"; python3 tools/diag/sq_summary.py "$OUT/$v"
done
