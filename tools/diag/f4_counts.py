#!/usr/bin/env python3
"""DIAGNOSTIC: per-rule-wave loop counters of k_rollout_full (build with
tools/diag/build_f4count.py): passes per ply, passes spent waiting for the
helper, lanes playing per pass, parks per lane and ply -- for one 1,000-ply
launch after a warm-up.  argv: plies per launch (1000)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB = os.path.join(ROOT, "tools", "diag", "build", "libnarde_f4count.so")
os.environ["NARDE_LIB"] = LIB
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    lib = ctypes.CDLL(LIB)
    env = VecNardeEnv(65536, device="cuda:0", seed=0, rules="full4")
    b = env.rollout_buffers(P)
    for _ in range(3):
        env.rollout(P, b)
    torch.cuda.synchronize()
    c = np.zeros((4096, 4), np.uint64)
    assert lib.narde_diag_f4(c.ctypes.data_as(ctypes.c_void_p)) == 0
    c = c[:1024].astype(np.float64)
    passes, waits, lanes, parks = c[:, 0], c[:, 1], c[:, 2], c[:, 3]
    h = np.zeros((4096, 4), np.uint64)
    assert lib.narde_diag_f4h(h.ctypes.data_as(ctypes.c_void_p)) == 0
    h = h[:1024].astype(np.float64)
    helper = {"helper_passes_per_ply": round(float(h[:, 0].mean() / P), 4),
              "lanes_per_helper_pass": round(float(h[:, 1].sum() / max(1.0, h[:, 0].sum())), 2),
              "helper_busy_frac_of_rule_loop": round(float(h[:, 2].sum() / h[:, 3].sum()), 4),
              "rule_loop_us_per_ply": round(float(h[:, 3].mean() / P / 100.0), 4)}  # wall_clock64: 100 MHz
    out = {"plies": P, **helper,
           "passes_per_ply": [round(float(x), 4) for x in np.percentile(passes / P, [0, 50, 100])],
           "wait_passes_per_ply": round(float(waits.mean() / P), 4),
           "lanes_per_pass": round(float(lanes.sum() / passes.sum()), 2),
           "parks_per_lane_ply": round(float(parks.sum() / (1024 * 64 * P)), 5),
           "parks_per_wave_ply": round(float(parks.sum() / (1024 * P)), 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
