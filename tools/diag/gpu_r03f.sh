#!/bin/bash
# DIAGNOSTIC round-3 call f: REF2 start-up A/B (base vs selfdraw), the
# bench --gpus 1 GPU test, the store roof at 153.6 / 751.3 MB, FULL4 A/B
# (base vs nring: narrow outputs through an LDS ring) with the FULL4 tests
# on nring, and PMC WRITE_SIZE/FETCH_SIZE of both FULL4 builds.
set -o pipefail
mkdir -p gpurun_out/r03f
bash tools/diag/gpu_ab_ref2.sh base selfdraw || exit 1
timeout -k 10 200 python -u -m pytest tests/test_gpu_bench_line.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r03f/pytest_benchline.log 2>&1 || { tail -30 gpurun_out/r03f/pytest_benchline.log; exit 1; }
tail -1 gpurun_out/r03f/pytest_benchline.log
timeout -k 10 120 python tools/diag/store_roof_short.py > gpurun_out/r03f/store_roof_short.json || exit 1
cat gpurun_out/r03f/store_roof_short.json
bash tools/diag/gpu_ab_f4.sh base nring || exit 1
bash tools/diag/gpu_pmc_full4.sh base nring || exit 1
