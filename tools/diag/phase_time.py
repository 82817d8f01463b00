#!/usr/bin/env python3
"""DIAGNOSTIC (round 4): one 20-ply FULL4 rollout launch timed at a given
game phase.  All envs start together, so after `skip` untimed plies (one
stats-only launch) the population sits at one phase of its games: early
(0), mid (40), late (65-85: the home-board blocks).  Per phase: the median
of 7 repetitions (fresh handle each time, same seed), us per launch, for
the library named by $NARDE_LIB."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    skips = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,40,60,70,80").split(",")]
    out = {"lib": os.path.basename(os.environ.get("NARDE_LIB", "libnarde.so"))}
    for skip in skips:
        ts = []
        for rep in range(7):
            env = VecNardeEnv(65536, device="cuda:0", seed=0, rules="full4")
            bufs = env.rollout_buffers(20)
            if skip:
                env.selfplay(skip)
            env.rollout(20, bufs)  # warm the launch path (this advances the phase by 20 plies)
            torch.cuda.synchronize()
            env.close()
            env = VecNardeEnv(65536, device="cuda:0", seed=0, rules="full4")
            if skip:
                env.selfplay(skip)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            env.rollout(20, bufs)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) * 1e3)
            env.close()
            del bufs
        out[f"plies_{skip}_{skip + 20}"] = round(statistics.median(ts), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
