#!/usr/bin/env python3
"""DIAGNOSTIC: sustained stats-only self-play (k_rollout_pc<false>, no
per-ply outputs) rate at 1,000 plies per launch for $NARDE_LIB."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402

env = VecNardeEnv(65536, device="cuda:0", seed=0)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    env.selfplay(1000)
    torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(200):
    env.selfplay(1000)
e.record()
torch.cuda.synchronize()
print(json.dumps({"lib": os.path.basename(os.environ.get("NARDE_LIB", "")),
                  "selfplay_ms_per_100_plies": round(s.elapsed_time(e) / 200 / 10, 4)}))
