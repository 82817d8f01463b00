#!/usr/bin/env python3
"""DIAGNOSTIC: per-wave lifetimes of short FULL4 rollout launches (the bench's
other_rules leg at the driver's 20 plies: back-to-back launches).  argv:
tag (wclock -> k_rollout_wave, wclock_full -> k_rollout_full), plies
(default 20).  Needs tools/diag/build/libnarde_<tag>.so (build_wave_clock.py).
Prints, per launch, the event span and the percentiles over waves of the end
of each wave's ply loop, relative to the first wave's entry (us)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
tag = sys.argv[1] if len(sys.argv) > 1 else "wclock"
LIB = os.path.join(ROOT, "tools", "diag", "build", f"libnarde_{tag}.so")
os.environ["NARDE_LIB"] = LIB
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    lib = ctypes.CDLL(LIB)
    env = VecNardeEnv(65536, device="cuda:0", seed=0, rules="full4")
    b = env.rollout_buffers(P)
    for _ in range(300):  # ~40 ms of back-to-back launches: clocks up
        env.rollout(P, b)
    torch.cuda.synchronize()
    full = "full" in tag
    nw = 2048 if full else 1024
    passes = hasattr(lib, "narde_diag_passes")
    for trial in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        env.rollout(P, b)
        torch.cuda.synchronize()
        if passes:
            assert lib.narde_diag_passes(None, 1) == 0
        e0.record()
        env.rollout(P, b)
        e1.record()
        torch.cuda.synchronize()
        ts = np.zeros((4096, 2), dtype=np.int64)
        assert lib.narde_diag_wts(ts.ctypes.data_as(ctypes.c_void_p)) == 0
        ts = ts[:nw]
        t0 = ts[:, 0].min()
        rel = (ts - t0) * 0.01  # wall_clock64 = 100 MHz
        rule = np.array([(w % 8) < 4 for w in range(nw)]) if full else np.ones(nw, bool)
        end = rel[rule, 1]
        life = (ts[rule, 1] - ts[rule, 0]) * 0.01
        q = lambda a, x: round(float(np.percentile(a, x)), 2)  # noqa: E731
        out = {"tag": tag, "plies": P, "event_span_us": round(e0.elapsed_time(e1) * 1e3, 2),
               "entry_spread_us": q(rel[:, 0], 100),
               "end_us": {"p10": q(end, 10), "p50": q(end, 50), "p90": q(end, 90), "p99": q(end, 99),
                          "max": q(end, 100), "mean": round(float(end.mean()), 2)},
               "life_mean_us": round(float(life.mean()), 2)}
        if full:
            out["helper_end_max_us"] = q(rel[~rule, 1], 100)
        if passes:  # owner-passes per wave (depth / pair) against the wave's end
            pc = np.zeros((4096, 2), dtype=np.uint32)
            assert lib.narde_diag_passes(pc.ctypes.data_as(ctypes.c_void_p), 0) == 0
            pc = pc[:nw].astype(np.float64)
            ends = rel[:, 1]
            X = np.column_stack([np.ones(nw), pc[:, 0], pc[:, 1]])
            coef, *_ = np.linalg.lstsq(X, ends, rcond=None)
            out["passes"] = {"depth_mean": round(float(pc[:, 0].mean()), 2), "depth_max": int(pc[:, 0].max()),
                             "pair_mean": round(float(pc[:, 1].mean()), 2), "pair_max": int(pc[:, 1].max()),
                             "fit_us": [round(float(c), 3) for c in coef],
                             "slowest_wave_passes": pc[int(np.argmax(ends))].astype(int).tolist()}
        # which workgroups hold the slowest waves (per-CU placement is not known)
        out["slowest_waves"] = [int(x) for x in np.argsort(-rel[:, 1])[:5]]
        print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
