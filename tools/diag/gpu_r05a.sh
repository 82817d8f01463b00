#!/bin/bash
# round 5, call A: the parity suite with the oracle's legal words, the smoke,
# the issue probe (cycles, then its SQ counter pass)
set -o pipefail
OUT=gpurun_out/r05
mkdir -p $OUT
export TMPDIR=/tmp
echo "[r05a] $(date +%T) parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 \
  && echo "[r05a] $(date +%T) smoke" \
  && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
  && echo "[r05a] $(date +%T) issue probe" \
  && timeout -k 10 240 python3 tools/issue_probe.py --out $OUT/issue_probe.json > $OUT/issue_probe.log 2>&1 \
  && echo "[r05a] $(date +%T) issue probe SQ pass" \
  && (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
        --output-format csv -d $GRAFT_REPO_ROOT/$OUT/issue_probe_sq -o sq -- python3 $GRAFT_REPO_ROOT/tools/issue_probe.py --iters 2000 \
        > $GRAFT_REPO_ROOT/$OUT/issue_probe_sq.log 2>&1)
rc=$?
tail -3 $OUT/parity.log; tail -2 $OUT/smoke.log; tail -2 $OUT/issue_probe.log
echo "[r05a] rc=$rc"
exit $rc
