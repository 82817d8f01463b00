#!/bin/bash
# Copy the judged evidence of one tools/gpu_round.sh call from gpurun_out/<tag>
# into profiles/ (tracked): bench lines, rocprofv3 kernel-stats summaries,
# PMC summaries (+ raw counter CSVs), GPU test log, smoke log.
#   bash tools/collect_profiles.sh <tag> [profiles subdir, default r01]
set -e
TAG=${1:?tag}
DST=profiles/${2:-r01}
SRC=gpurun_out/$TAG
mkdir -p "$DST/pmc" "$DST/pmc_full"
cp "$SRC/bench_n1.json" "$DST/bench_n1.json"
cp "$SRC/bench_full4.json" "$DST/bench_full4.json"
cp "$SRC/pytest_gpu.log" "$DST/pytest_gpu.log"
cp "$SRC/smoke.log" "$DST/smoke.log"
cp "$SRC"/rocprof/*kernel_stats.csv "$DST/rocprof_kernel_stats_bench.csv"
cp "$SRC"/rocprof_full4/*kernel_stats.csv "$DST/rocprof_kernel_stats_full4.csv"
cp "$SRC"/rocprof_dqn/*kernel_stats.csv "$DST/rocprof_kernel_stats_dqn.csv"
cp "$(find "$SRC/pmc/fetch" -name '*counter_collection.csv' | head -1)" "$DST/pmc/fetch_size_counter_collection.csv"
cp "$(find "$SRC/pmc/write" -name '*counter_collection.csv' | head -1)" "$DST/pmc/write_size_counter_collection.csv"
cp "$(find "$SRC/pmc_full/fetch" -name '*counter_collection.csv' | head -1)" "$DST/pmc_full/fetch_size_counter_collection.csv"
cp "$(find "$SRC/pmc_full/write" -name '*counter_collection.csv' | head -1)" "$DST/pmc_full/write_size_counter_collection.csv"
cp "$SRC/pmc_k_rollout.json" profiles/pmc_k_rollout.json
cp "$SRC/pmc_k_rollout_full.json" profiles/pmc_k_rollout_full.json
echo "collected $SRC -> $DST"
