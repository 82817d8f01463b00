#!/usr/bin/env python3
"""DIAGNOSTIC: narde_observe at B = 65,536: the 198-float observation and the
int32[24] one, microseconds per call (events around 50 calls)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402

env = VecNardeEnv(65536, device="cuda:0", seed=0)
env.selfplay(100)
out = torch.empty((65536, 198), dtype=torch.float32, device="cuda:0")
for kind in ("tesauro198", "observe"):
    fn = (lambda: env.tesauro198(out=out)) if kind == "tesauro198" else env.observe
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(50):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / 50
    nbytes = 65536 * (198 * 4 if kind == "tesauro198" else 96) + 65536 * 32
    print(f"{kind}: {us:.2f} us per call, {nbytes / (us * 1e-6) / 1e12:.2f} TB/s")
