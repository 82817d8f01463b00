#!/usr/bin/env python3
"""DIAGNOSTIC (round 4): where the single-ply REF2 k_step's ~6 us go.  The
same launch (narde_step, device dice, random-legal policy, auto-reset) with
every output, with only the obs rows, with only the narrow outputs, with
none (the record update alone), and a 1-ply stats-only rollout; 300 warm
launches each, HIP events around the run, us per launch.  $NARDE_LIB picks
the library."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde import _lib  # noqa: E402
from gym_narde.vector import VecNardeEnv  # noqa: E402


def timed(fn, warm=100, reps=300):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) * 1e3 / reps, 2)


def main():
    n = 65536
    env = VecNardeEnv(n, device="cuda:0", seed=0)
    h = env.handle.h
    st = env._s()
    obs, rew, term, trunc, leg, act = env._step_out
    f = env._step_fn
    cases = {
        "all": (obs, rew, term, trunc, leg, act),
        "obs_only": (obs, None, None, None, None, None),
        "narrow_only": (None, rew, term, trunc, leg, act),
        "none": (None, None, None, None, None, None),
    }
    out = {}
    for name, ptrs in cases.items():
        out[name] = timed(lambda: f(h, None, None, *ptrs, 1, st))
    out["selfplay_1ply_stats_only"] = timed(lambda: env.selfplay(1))
    bufs = env.rollout_buffers(1)
    out["rollout_1ply_all"] = timed(lambda: env.rollout(1, bufs))
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
