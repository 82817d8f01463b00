#!/usr/bin/env python3
"""Time k_rollout (outputs on/off) for the libnarde.so named by $NARDE_LIB.
Optional argv[1] = number of envs (default 65,536)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    rules = sys.argv[2] if len(sys.argv) > 2 else "ref2"
    dice_mode = sys.argv[3] if len(sys.argv) > 3 else "all36"
    P, reps = 100, 30
    env = VecNardeEnv(n, device="cuda:0", seed=0, rules=rules, dice_mode=dice_mode)
    bufs = env.rollout_buffers(P)
    env.selfplay(300)
    out = {"lib": os.path.basename(os.environ.get("NARDE_LIB", "libnarde.so")), "envs": n,
           "rules": rules, "dice": dice_mode,
           "rollout_ms": round(timed(lambda: env.rollout(P, bufs), reps), 4),
           "selfplay_ms": round(timed(lambda: env.selfplay(P), reps), 4)}
    out["rollout_steps_per_s"] = round(n * P / (out["rollout_ms"] * 1e-3))
    out["selfplay_steps_per_s"] = round(n * P / (out["selfplay_ms"] * 1e-3))
    out["rollout_TBps"] = round(n * (114 * P + 64) / (out["rollout_ms"] * 1e-3) / 1e12, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
