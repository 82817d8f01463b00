#!/usr/bin/env python3
"""DIAGNOSTIC: the host side of the driver's timed region (bench.py --steps
20 --warmup 5: device ramped, GPU idle, ONE 20-ply launch between two
synchronizes).  Median over 40 trials of the wall time from the launch call
to the end of the wait, for several ways of waiting:
  sync      launch (+ events), torch.cuda.synchronize()       (bench.py today)
  evsync    launch (+ events), hipEventSynchronize(stop event), then torch.cuda.synchronize()
  stsync    launch (+ events), hipStreamSynchronize(stream), then torch.cuda.synchronize()
  query     launch (+ events), spin on hipEventQuery(stop event), then torch.cuda.synchronize()
and the same without the two timing events (bare_*).  $HIP_SPIN=1 first
sets hipDeviceScheduleSpin.  argv: plies (default 20)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import TimingEvent, VecNardeEnv  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    hip = ctypes.CDLL("libamdhip64.so.7")
    out = {"plies": P}
    if os.environ.get("HIP_SPIN") == "1":
        out["set_flags"] = hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
    env = VecNardeEnv(65536, device="cuda:0", seed=0)
    big = env.rollout_buffers(1000)
    ramp = env.rollout_launcher(1000, big)
    for _ in range(120):
        ramp()
    torch.cuda.synchronize()
    e0, e1 = TimingEvent("cuda:0"), TimingEvent("cuda:0")
    b = env.rollout_buffers(P)
    L = env.rollout_launcher(P, b, events=(e0, e1))
    Lb = env.rollout_launcher(P, b)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    stop = ctypes.c_void_p(e1.handle)

    def w_sync():
        pass

    def w_evsync():
        hip.hipEventSynchronize(stop)

    def w_stsync():
        hip.hipStreamSynchronize(stream)

    def w_query():
        while hip.hipEventQuery(stop) != 0:
            pass

    waits = {"sync": w_sync, "evsync": w_evsync, "stsync": w_stsync, "query": w_query}
    res = {k: [] for k in waits}
    res.update({"bare_" + k: [] for k in ("sync", "stsync")})
    spans = []
    for _ in range(40):
        for name, w in waits.items():
            for _ in range(3):
                ramp()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            L()
            w()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) * 1e6)
            spans.append(e0.elapsed_ms(e1) * 1e3)
        for name in ("sync", "stsync"):
            for _ in range(3):
                ramp()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            Lb()
            waits[name]()
            torch.cuda.synchronize()
            res["bare_" + name].append((time.perf_counter() - t0) * 1e6)
    for k, v in res.items():
        v.sort()
        out[k] = round(v[len(v) // 2], 2)
    spans.sort()
    out["span_us"] = round(spans[len(spans) // 2], 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
