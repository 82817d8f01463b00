#!/bin/bash
# DIAGNOSTIC (round 4, call a): the issue probe, the API kernels warm (timed
# and traced), and SQ passes of the two 20-ply rollout kernels.
set -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r04a
mkdir -p "$OUT"
export TMPDIR=/tmp
CNT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"
timeout -k 10 120 python3 -c "import ctypes; ctypes.CDLL('tools/diag/build/libissue_probe.so').issue_probe_main()" > "$OUT/issue_probe.json" \
 && cat "$OUT/issue_probe.json" \
 && timeout -k 10 120 python3 tools/api_target.py > "$OUT/api.json" && cat "$OUT/api.json" \
 && (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/api_trace" -o api \
        -- python3 "$ROOT/tools/api_target.py" > "$OUT/api_trace.log" 2>&1) \
 && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d "$OUT/sq_ref2" -o sq \
        -- python3 "$ROOT/tools/pmc_target.py" --plies 20 --launches 5 > "$OUT/sq_ref2.log" 2>&1) \
 && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d "$OUT/sq_full4" -o sq \
        -- python3 "$ROOT/tools/pmc_target.py" --rules full4 --plies 20 --launches 5 > "$OUT/sq_full4.log" 2>&1) \
 && python3 tools/sq_summary.py --dir "$OUT/sq_ref2" --kernel "k_rollout_pc<true, true>" --plies 20 --out "$OUT/sq_k_rollout_p20.json" \
 && python3 tools/sq_summary.py --dir "$OUT/sq_full4" --kernel "k_rollout_wave<true>" --plies 20 --out "$OUT/sq_k_rollout_full_p20.json"
rc=$?
find "$OUT/api_trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/api_kernel_stats.csv" \;
echo "rc=$rc"
exit $rc
