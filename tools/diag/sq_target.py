#!/usr/bin/env python3
"""rocprofv3 --pmc target for SQ issue counters: 3 k_rollout launches with
outputs, then 3 stats-only, at the bench shape, for the libnarde.so named by
$NARDE_LIB (default: the in-tree build).  argv: rules (ref2 / full4), plies
per launch (default 100).  DIAGNOSTIC."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    rules = sys.argv[1] if len(sys.argv) > 1 else "ref2"
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    env = VecNardeEnv(65536, device="cuda:0", seed=0, rules=rules)
    bufs = env.rollout_buffers(P)
    for _ in range(3):
        env.rollout(P, bufs)
    for _ in range(3):
        env.selfplay(P)
    torch.cuda.synchronize()
    env.close()


if __name__ == "__main__":
    main()
