"""DIAGNOSTIC: host-side cost of VecNardeEnv.step (eager API, B envs)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402

for B in (65536, 1024):
    env = VecNardeEnv(B, device="cuda:0", seed=0)
    acts = torch.zeros((B, 2), dtype=torch.int16, device="cuda:0")
    for label, fn in (("policy", lambda: env.step()), ("actions", lambda: env.step(acts))):
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        n = 2000
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        print(f"B={B} {label}: {(time.perf_counter() - t0) / n * 1e6:.2f} us per step() call")
