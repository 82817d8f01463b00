#!/usr/bin/env python3
"""DIAGNOSTIC: the store roof at the driver's bench shape.  The 20-ply REF2
launch writes 153.6 MB; this times ONE torch fill_ of the same bytes (16-B
vector stores, no reads) after the same device ramp as single_launch.py,
GPU idle, median over 30 trials of the event span and of the host round
trip (fill + synchronize).  Also the 100-ply (751.3 MB) size.  The floor
for the 20-ply dispatch that VERDICT r02 asked to bring to <= 30 us."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    env = VecNardeEnv(65536, device="cuda:0", seed=0)
    big = env.rollout_buffers(1000)
    ramp = env.rollout_launcher(1000, big)
    for _ in range(120):
        ramp()
    torch.cuda.synchronize()
    out = {}
    for name, nbytes in (("20_plies", 153_616_384), ("100_plies", 751_304_704)):
        x = torch.empty(nbytes // 4, dtype=torch.int32, device="cuda:0")
        x.fill_(0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        spans, trips = [], []
        for i in range(30):
            for _ in range(3):
                ramp()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            x.fill_(i)
            e1.record()
            torch.cuda.synchronize()
            trips.append((time.perf_counter() - t0) * 1e6)
            spans.append(e0.elapsed_time(e1) * 1e3)
        spans.sort()
        trips.sort()
        out[name] = {"bytes": nbytes, "span_med_us": round(spans[15], 2), "span_p10": round(spans[3], 2),
                     "trip_med_us": round(trips[15], 1), "TBps_span": round(nbytes / (spans[15] * 1e-6) / 1e12, 3)}
        del x
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
