#!/bin/bash
# DIAGNOSTIC (on the GPU box, from the repo root; writes scratch copies of
# bench.py there): what runs last before the driver-shape timed launch.
#   A = bench.py: the region's three untimed calls, then the --warmup launches
#   B = the --warmup launches first, then the three untimed calls
#   C = B plus one plain 20-ply launch (no markers) after the untimed calls
# Alternating runs of `--gpus 1 --steps 20 --warmup 5` (secondary legs off).
#   gpurun --timeout 600 -- bash tools/diag/gpu_ab_order.sh [variants] [reps]
set -o pipefail
VARIANTS=${1:-"bench bench_b bench_c"}
REPS=${2:-6}
python3 - <<'PY' || exit 1
s = open("bench.py").read()
a = """    for _ in range(3):
        calls[0]()
        if len(calls) > 1:
            calls[-1]()
    eng.sync()
    ramp_n += 3 if len(calls) == 1 else 6

    run_plies(args.warmup)
"""
assert a in s
b = a.replace("    run_plies(args.warmup)\n", "")
b = "    run_plies(args.warmup)\n" + b
c = b.replace("            calls[-1]()\n    eng.sync()", "            calls[-1]()\n    full_launch()\n    eng.sync()")
open("bench_b.py", "w").write(s.replace(a, b))
open("bench_c.py", "w").write(s.replace(a, c))
PY
mkdir -p gpurun_out/ab_order
for rep in $(seq 1 "$REPS"); do
  for v in $VARIANTS; do
    timeout -k 10 120 python "$v.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --dqn-steps 0 \
      --api-steps 0 --other-launches 0 --fused-launches 0 > "gpurun_out/ab_order/$v.$rep.json" 2>/dev/null || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_order/$v.$rep.json').read().strip().splitlines()[-1]);print('$v',$rep,'%.4g'%d['value'],d['roofline']['kernel_ms'],d['timed_region_host_us'])"
  done
done
