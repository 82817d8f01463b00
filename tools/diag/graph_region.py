#!/usr/bin/env python3
"""DIAGNOSTIC: the driver-shape timed region (one 20-ply launch between two
synchronizes, device ramped) with the launch and its two timing markers
made by one ctypes call (narde_rollout_timed, bench.py today) against the
same three operations captured once into a HIP graph and replayed
(torch.cuda.CUDAGraph around the same ctypes call: an event-record node,
the kernel node, an event-record node).  Median wall time of the region
over 40 alternating trials, and the event span of each."""
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
    env = VecNardeEnv(65536, device="cuda:0", seed=0)
    big = env.rollout_buffers(1000)
    ramp = env.rollout_launcher(1000, big)
    for _ in range(120):
        ramp()
    torch.cuda.synchronize()
    b = env.rollout_buffers(P)
    e0, e1 = TimingEvent("cuda:0"), TimingEvent("cuda:0")
    direct = env.rollout_launcher(P, b, events=(e0, e1))
    g0, g1 = TimingEvent("cuda:0"), TimingEvent("cuda:0")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        cap = env.rollout_launcher(P, b, events=(g0, g1))  # binds the capture stream
        cap()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            cap()
    torch.cuda.current_stream().wait_stream(s)
    graph.replay()
    torch.cuda.synchronize()
    res = {"direct": [], "graph": []}
    spans = {"direct": [], "graph": []}
    for _ in range(40):
        for name, fn, evs in (("direct", direct, (e0, e1)), ("graph", graph.replay, (g0, g1))):
            for _ in range(3):
                ramp()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) * 1e6)
            spans[name].append(evs[0].elapsed_ms(evs[1]) * 1e3)
    out = {"plies": P}
    for k in res:
        r, sp = sorted(res[k]), sorted(spans[k])
        out[k] = {"region_med_us": round(r[20], 1), "p10_p90": [round(r[4], 1), round(r[36], 1)],
                  "span_med_us": round(sp[20], 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
