#!/usr/bin/env python3
"""DIAGNOSTIC: in-kernel clock of k_rollout_pc (MI355X_MICROARCH.md, DVFS
give-back item 6).  $NARDE_LIB must be a -DNARDE_DIAG_CLOCK=1 build.  Runs
~2 s of back-to-back launches, then reads the last launch's per-workgroup
(s_memtime, s_memrealtime) stamps: clock = d(memtime) / d(realtime) x 100 MHz.
argv[1] = 'rollout' (outputs on) or 'selfplay' (stats only)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde import _lib  # noqa: E402
from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "rollout"
    n, P = 65536, 100
    env = VecNardeEnv(n, device="cuda:0", seed=0)
    bufs = env.rollout_buffers(P)
    fn = (lambda: env.rollout(P, bufs)) if mode == "rollout" else (lambda: env.selfplay(P))
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < 2.0:
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        k += 50
    wall_ms = (time.perf_counter() - t0) * 1e3 / k
    lib = ctypes.CDLL(os.environ["NARDE_LIB"])
    buf = np.zeros((4096, 4), dtype=np.uint64)
    rc = lib.narde_diag_clock(buf.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0, rc
    wg = n // 256
    b = buf[:wg].astype(np.float64)
    dclk, drt = b[:, 1] - b[:, 0], b[:, 3] - b[:, 2]
    ghz = dclk / drt * 0.1
    print(json.dumps({"lib": os.path.basename(os.environ["NARDE_LIB"]), "mode": mode,
                      "launch_ms_wall": round(wall_ms, 4),
                      "wg_ms_median": round(float(np.median(drt)) / 1e5, 4),
                      "clock_GHz_median": round(float(np.median(ghz)), 3),
                      "clock_GHz_p10_p90": [round(float(np.percentile(ghz, 10)), 3),
                                            round(float(np.percentile(ghz, 90)), 3)],
                      "cycles_median": int(np.median(dclk))}))


if __name__ == "__main__":
    main()
