#!/usr/bin/env python3
"""DIAGNOSTIC: where the time of ONE k_rollout_pc launch goes (after a device
ramp, GPU idle, as in bench.py at the driver's shape).  Needs
tools/diag/build/libnarde_clock.so (build_clock.py).  argv: plies (default
20) [stats] -- 'stats' launches the stats-only kernel.  Prints, relative to
the earliest wave entry (wall_clock64 ticks at 100 MHz = 10 ns), the
percentiles over producer and consumer waves of every stamp, and the event
span of the launch."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB = os.path.join(ROOT, "tools", "diag", "build", "libnarde_clock.so")
os.environ["NARDE_LIB"] = LIB
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    stats = len(sys.argv) > 2 and sys.argv[2] == "stats"
    lib = ctypes.CDLL(LIB)
    env = VecNardeEnv(65536, device="cuda:0", seed=0)
    big = env.rollout_buffers(1000)
    ramp = env.rollout_launcher(1000, big)
    b = env.rollout_buffers(P)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    e1.record()
    rows = torch.empty(((65536 + 255) // 256, 3), dtype=torch.int64, device="cuda:0")
    L = env.rollout_launcher(P, b, events=(e0, e1), totals=rows)  # the bench's timed launch
    res = []
    trials = []
    for trial in range(5):
        for _ in range(120 if trial == 0 else 3):
            ramp()
        torch.cuda.synchronize()
        if stats:
            e0.record()
            env.selfplay(P)
            e1.record()
        else:
            L()
        torch.cuda.synchronize()
        ts = np.zeros((4096, 64), dtype=np.int64)
        assert lib.narde_diag_ts(ts.ctypes.data_as(ctypes.c_void_p)) == 0
        ts = ts[:2048]
        t0 = ts[:, 0].min()
        rel = np.where(ts > 0, (ts - t0) * 0.01, np.nan)  # us
        prod = np.array([w % 8 < 4 for w in range(2048)])
        nb = 2 + (P - 3 + 3) // 4 if P > 3 else (1 if P <= 1 else 2)
        out = {"plies": P, "stats_only": stats, "event_span_us": round(e0.elapsed_time(e1) * 1e3, 2),
               "in_kernel_span_us": round(float(np.nanmax(rel[:, 63])), 2)}
        cols = {"entry": 0, "loaded_or_drawn": 1, "start_barrier": 2}
        for k in range(min(nb, 56)):
            cols[f"block{k}"] = 3 + k
        cols.update({"last_emit": 59, "record_stored": 60, "stats_loaded": 61, "totals": 62, "end": 63})
        for name, c in cols.items():
            for who, m in (("prod", prod), ("cons", ~prod)):
                v = rel[m, c]
                v = v[~np.isnan(v)]
                if len(v):
                    out[f"{name}.{who}"] = [round(float(np.percentile(v, q)), 2) for q in (0, 50, 100)]
        ts0 = ts[:, 0]
        ts0 = ts0[ts0 > 0]
        trials.append(rel)
        res.append(out)
    print(json.dumps(res[-1], indent=0))
    if len(sys.argv) > 3:
        np.save(sys.argv[3], np.stack(trials))
    print(json.dumps({"event_span_us": [r["event_span_us"] for r in res],
                      "in_kernel_span_us": [r["in_kernel_span_us"] for r in res]}))


if __name__ == "__main__":
    main()
