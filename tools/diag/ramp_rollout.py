#!/usr/bin/env python3
"""DIAGNOSTIC: per-launch time of back-to-back k_rollout_pc launches over
~3 s from a cold start, in groups of 20 launches (HIP events), to see how
long the device takes to reach its sustained rate."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    n, P, G = 65536, 100, 20
    env = VecNardeEnv(n, device="cuda:0", seed=0)
    bufs = env.rollout_buffers(P)
    env.rollout(P, bufs)
    torch.cuda.synchronize()
    time.sleep(1.0)  # let the device idle
    ev = []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 3.0:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(G):
            env.rollout(P, bufs)
        e.record()
        ev.append((s, e, time.perf_counter() - t0))
        if len(ev) % 25 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    series = [(round(t, 4), round(s.elapsed_time(e) / G, 4)) for s, e, t in ev]
    pick = series[:30] + series[30::25]
    print(json.dumps({"launch_ms_by_group": pick, "groups": len(series)}))


if __name__ == "__main__":
    main()
