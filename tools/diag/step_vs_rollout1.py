#!/usr/bin/env python3
"""DIAGNOSTIC (round 5): the REF2 self-play API step (k_step<false>, one wave
per 64 envs) against a 1-ply launch of the producer/consumer rollout
(k_rollout_pc<true>, rule and consumer waves, the same outputs) --
VERDICT r04 asked for k_step split across two waves per SIMD as k_rollout_pc
does.  Device time per call, graph-replayed (tools/api_target.py graphed),
B = 65,536.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from api_target import graphed  # noqa: E402
from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    n = 65536
    out = {"envs": n}
    for rep in range(3):
        env = VecNardeEnv(n, device="cuda:0", seed=0)
        for _ in range(100):
            env.step()
        bufs = env.rollout_buffers(1)
        one = lambda: env.rollout(1, bufs)  # noqa: E731  (the stream current at each call: graph capture)
        for _ in range(100):
            one()
        torch.cuda.synchronize()
        out.setdefault("k_step_us", []).append(round(graphed(env.step, 600), 2))
        out.setdefault("rollout1_us", []).append(round(graphed(one, 600), 2))
        env.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
