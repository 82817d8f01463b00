#!/usr/bin/env python3
"""Run the stamped diagnostic build of the rollout ply and print per-phase
cycle shares (DIAGNOSTIC; see diag.hip)."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PHASES = ["rng+dice", "list1", "policy1+move1", "list2+policy2+move2", "end+flip+reset", "obs store",
          "record store"]


def main():
    so = os.path.join(HERE, "build", "libdiag.so")
    if not os.path.exists(so) or any(a.startswith("--build") for a in sys.argv):
        os.makedirs(os.path.dirname(so), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                               "-fPIC", "-shared", "-o", so, os.path.join(HERE, "diag.hip")])
    if "--build-only" in sys.argv:
        return
    lib = ctypes.CDLL(so)
    lib.diag_run.restype = ctypes.c_float
    n, plies = 65536, 100
    waves = n // 64
    cyc = np.zeros((waves, len(PHASES)), np.uint64)
    ms = lib.diag_run(n, 300, plies, cyc.ctypes.data_as(ctypes.c_void_p))
    tot = cyc.sum(0).astype(np.float64)
    share = tot / tot.sum()
    per_ply = tot / waves / plies
    print(json.dumps({"kernel_ms": round(ms, 4), "cycles_per_ply_per_wave": round(float(per_ply.sum()), 1),
                      "phases": {p: {"share": round(float(s), 4), "cycles_per_ply": round(float(c), 1)}
                                 for p, s, c in zip(PHASES, share, per_ply)}}, indent=1))


if __name__ == "__main__":
    main()
