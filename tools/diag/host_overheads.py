#!/usr/bin/env python3
"""DIAGNOSTIC: what the bench's timed region costs besides the kernel, at the
driver's shape (one 20-ply k_rollout_pc launch over 65,536 envs).

Prints per-call host costs (event record, idle synchronize, ctypes launch)
and round trips of a single launch with different completion waits, plus
the event-timed duration of single launches of 5 / 20 / 100 / 1,000 plies
after a device ramp.  NARDE_SPIN=1 sets hipDeviceScheduleSpin on the device
before torch creates its context (a spinning host wait instead of a
yielding one)."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))

if os.environ.get("NARDE_SPIN") == "1":
    hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(ctypes.c_uint(1)))

import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def us(t):
    return round(t * 1e6, 2)


def main():
    env = VecNardeEnv(65536, device="cuda:0", seed=0)
    big = env.rollout_buffers(1000)
    ramp = env.rollout_launcher(1000, big)
    for _ in range(150):
        ramp()
    torch.cuda.synchronize()
    out = {}
    n = 2000
    ev = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    for _ in range(n):
        ev.record()
    torch.cuda.synchronize()
    out["event_record_us"] = us((time.perf_counter() - t0) / n)
    t0 = time.perf_counter()
    for _ in range(n):
        torch.cuda.synchronize()
    out["idle_synchronize_us"] = us((time.perf_counter() - t0) / n)
    q = torch.cuda.Event()
    q.record()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        q.query()
    out["event_query_us"] = us((time.perf_counter() - t0) / n)

    bufs = env.rollout_buffers(20)
    L = env.rollout_launcher(20, bufs)
    for _ in range(50):
        ramp()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        L()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    out["launch_call_us"] = us((t1 - t0) / 200)

    def trip(kind, reps=60):
        vals = []
        for _ in range(reps):
            for _ in range(3):
                ramp()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            if kind == "bare":
                L()
                torch.cuda.synchronize()
            elif kind == "events":
                e0.record()
                L()
                e1.record()
                torch.cuda.synchronize()
            elif kind == "events_spin":
                e0.record()
                L()
                e1.record()
                while not e1.query():
                    pass
                torch.cuda.synchronize()
            vals.append(time.perf_counter() - t0)
        vals.sort()
        return us(vals[len(vals) // 2])

    for k in ("bare", "events", "events_spin"):
        out[f"round_trip_{k}_median_us"] = trip(k)

    for P in (5, 20, 100, 1000):
        b = big if P == 1000 else env.rollout_buffers(P)
        LP = env.rollout_launcher(P, b)
        d = []
        for _ in range(30):
            for _ in range(3):
                ramp()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            LP()
            e1.record()
            torch.cuda.synchronize()
            d.append(e0.elapsed_time(e1))
        d.sort()
        out[f"launch_{P}_plies_event_median_us"] = round(d[len(d) // 2] * 1e3, 2)
        # back to back (the gaps between launches hidden)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            LP()
        e1.record()
        torch.cuda.synchronize()
        out[f"launch_{P}_plies_b2b_us"] = round(e0.elapsed_time(e1) * 1e3 / 20, 2)
    print(out)


if __name__ == "__main__":
    main()
