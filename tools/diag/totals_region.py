#!/usr/bin/env python3
"""DIAGNOSTIC: what reading the episode totals costs inside the driver's
timed region (bench.py --steps 20 --warmup 5: device ramped, GPU idle, ONE
20-ply launch between two synchronizes).  Median over 40 trials of the wall
time from the launch call to the end of torch.cuda.synchronize(), for:
  launch        the 20-ply launch (+ its two timing markers) only
  totals        ... then VecNardeEnv.totals(out) + gather_total_rows (bench.py)
  totals_bound  ... then the pre-bound totals launcher (one ctypes call)
  fused         the 20-ply launch writing the totals rows itself (if the
                library has narde_rollout_timed_totals)
argv: plies (default 20)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde import distributed as D  # noqa: E402
from gym_narde.vector import TimingEvent, VecNardeEnv  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    env = VecNardeEnv(65536, device="cuda:0", seed=0)
    big = env.rollout_buffers(1000)
    ramp = env.rollout_launcher(1000, big)
    for _ in range(120):
        ramp()
    torch.cuda.synchronize()
    e0, e1 = TimingEvent("cuda:0"), TimingEvent("cuda:0")
    b = env.rollout_buffers(P)
    L = env.rollout_launcher(P, b, events=(e0, e1))
    rows = torch.empty((64, 3), dtype=torch.int64, device="cuda:0")
    T = env.totals_launcher(rows)
    variants = {
        "launch": lambda: None,
        "totals": lambda: D.gather_total_rows(env.totals(out=rows)),
        "totals_bound": T,
    }
    res = {k: [] for k in variants}
    spans = {k: [] for k in variants}
    for _ in range(40):
        for name, after in variants.items():
            for _ in range(3):
                ramp()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            L()
            after()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) * 1e6)
            spans[name].append(e0.elapsed_ms(e1) * 1e3)
    out = {"plies": P}
    for k, v in res.items():
        v.sort()
        s = sorted(spans[k])
        out[k] = {"wall_us": round(v[len(v) // 2], 2), "span_us": round(s[len(s) // 2], 2),
                  "wall_p10_p90": [round(v[len(v) // 10], 1), round(v[9 * len(v) // 10], 1)]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
