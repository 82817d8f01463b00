#!/usr/bin/env python3
"""DIAGNOSTIC: k_step (one ply per launch) time, REF2 and FULL4, for the
libnarde.so named by $NARDE_LIB: 500 launches after 200 warm ones, HIP
events around the run."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402

out = {"lib": os.path.basename(os.environ.get("NARDE_LIB", "libnarde.so"))}
for rules in ("ref2", "full4"):
    env = VecNardeEnv(65536, device="cuda:0", seed=0, rules=rules)
    for _ in range(200):
        env.step()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(500):
        env.step()
    e.record()
    torch.cuda.synchronize()
    out[rules + "_step_us"] = round(s.elapsed_time(e) / 500 * 1e3, 2)
    env.close()
print(json.dumps(out))
