#!/usr/bin/env python3
"""DIAGNOSTIC: sustained k_rollout rate per plies-per-launch.  For each P in
argv[1] (comma list, default 100,1000): ~0.5 s of back-to-back launches
(untimed), then ~1 s timed with two events around the whole run; prints ms
per 100 plies.  argv[2] = rules (ref2|full4), argv[3] = dice mode
(all36|nodoubles)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def run_for(fn, seconds):
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < seconds:
        fn()
        k += 1
        if k % 20 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return k


def main():
    Ps = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "100,1000").split(",")]
    rules = sys.argv[2] if len(sys.argv) > 2 else "ref2"
    dice_mode = sys.argv[3] if len(sys.argv) > 3 else "all36"
    n = 65536
    env = VecNardeEnv(n, device="cuda:0", seed=0, rules=rules, dice_mode=dice_mode)
    for P in Ps:
        bufs = env.rollout_buffers(P)
        fn = lambda: env.rollout(P, bufs)  # noqa: E731
        run_for(fn, 0.5)
        L = max(3, int(1.0 / (P * 1.5e-6 * (5 if rules == "full4" else 1))))
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(L):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e)
        per100 = ms / (L * P / 100)
        print(json.dumps({"rules": rules, "dice": dice_mode, "plies_per_launch": P, "launches": L,
                          "ms_per_100_plies": round(per100, 4),
                          "TBps": round(n * (114 * 100 + 64 * 100 / P) / (per100 * 1e-3) / 1e12, 3)}), flush=True)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
