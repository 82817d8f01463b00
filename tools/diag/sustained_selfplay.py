#!/usr/bin/env python3
"""DIAGNOSTIC: sustained stats-only rollout (selfplay) rate: argv[1] = plies
per launch, a comma list (default 1000), argv[2] = rules (ref2|full4).  ~0.5 s untimed,
then ~1 s timed between two events; prints ms per 100 plies."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    Ps = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1000").split(",")]
    rules = sys.argv[2] if len(sys.argv) > 2 else "full4"
    env = VecNardeEnv(65536, device="cuda:0", seed=0, rules=rules)
    for P in Ps:
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5:
            env.selfplay(P)
            torch.cuda.synchronize()
        L = max(3, int(1.0 / (P * 1.5e-6 * (5 if rules == "full4" else 1))))
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(L):
            env.selfplay(P)
        e.record()
        torch.cuda.synchronize()
        print(json.dumps({"rules": rules, "stats_only": True, "plies_per_launch": P, "launches": L,
                          "ms_per_100_plies": round(s.elapsed_time(e) / (L * P / 100), 4)}), flush=True)


if __name__ == "__main__":
    main()
