#!/usr/bin/env python3
"""rocprofv3 --pmc target: k_rollout_pc<true> / k_rollout_pp_full<true> at the bench shape.

Runs `--launches` launches of `--plies` plies over `--envs` envs with every
per-ply output written (exactly bench.py's timed kernel), after one warm-up
launch.  Profile it in separate passes, one counter group per pass:
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT/fetch -o pmc -- python3 tools/pmc_target.py
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d OUT/write -o pmc -- python3 tools/pmc_target.py
then summarise with tools/pmc_summary.py.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))

import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--plies", type=int, default=1000)
    ap.add_argument("--launches", type=int, default=3)
    ap.add_argument("--rules", choices=("ref2", "full4"), default="ref2")
    ap.add_argument("--stats-only", action="store_true",
                    help="the statistics-only launches (selfplay: k_rollout_*<false>, no per-ply output)")
    a = ap.parse_args()
    env = VecNardeEnv(a.envs, device="cuda:0", seed=0, rules=a.rules)
    bufs = None if a.stats_only else env.rollout_buffers(a.plies)
    for _ in range(a.launches + 1):
        if a.stats_only:
            env.selfplay(a.plies)
        else:
            env.rollout(a.plies, bufs)
    torch.cuda.synchronize()
    env.close()


if __name__ == "__main__":
    main()
