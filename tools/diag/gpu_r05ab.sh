#!/bin/bash
# round 5, call AB: FULL4 only -- statistics read at the launch's start
# (pppre) against the product before it (cur), driver-shape lines x8
set -o pipefail
OUT=gpurun_out/r05ab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_full4.py tests/test_gpu_configs.py -k "full4 or totals" -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 \
  && for rep in 1 2 3 4 5 6 7 8; do for tag in cur pppre; do NARDE_LIB=$PWD/tools/diag/build/libnarde_$tag.so timeout -k 10 300 python bench.py --rules full4 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${tag}_$rep.json 2> $OUT/bench_${tag}_$rep.err || exit 1; done; done
rc=$?
tail -2 $OUT/tests.log
python3 - <<PY
import json, glob
for tag in ("cur", "pppre"):
    ks = []
    for f in sorted(glob.glob("$OUT/bench_%s_*.json" % tag)):
        l = [x for x in open(f) if x.startswith("{")][-1]
        ks.append(json.loads(l)["roofline"]["kernel_ms"] * 1e3)
    ks.sort()
    print(tag, "kernel us sorted", [round(k, 1) for k in ks], "median", round(ks[len(ks)//2], 2))
PY
echo "[r05ab] rc=$rc"
exit $rc
