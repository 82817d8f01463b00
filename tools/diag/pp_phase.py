#!/usr/bin/env python3
"""DIAGNOSTIC: where a 20-ply FULL4 launch (k_rollout_pp_full<true>,
B = 65,536) spends its time, by ply and by kind of turn, from
tools/diag/build/libnarde_ppclock.so (build_ppclock.py).  Two series of five
20-ply launches: 'sync' -- every game from the start position in lockstep
(bench.py's other_rules leg: one ~100-ply game cycle), 'steady' -- after 300
plies of statistics-only self-play.  Per launch: the event span, the
producer waves' summed ply time (median / max over the 1,024 waves), and
what the slowest wave met; per ply: the share of waves of each kind and
their mean ply time; per kind of wave: the mean s_memtime ticks of the ply's
segments (0 block test, 1 turn_c0_free, 2 the turn, 3 / 4 / 5 the bound
turn's pair-bound C_0 / doubles-bound C_0 / sub-moves, 6 the close).
Prints one JSON object."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB = os.path.join(ROOT, "tools", "diag", "build", "libnarde_ppclock.so")
os.environ["NARDE_LIB"] = LIB
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402

MAXP = 160
KINDS = {"free": lambda k: (k & 3) == 0, "two_bound_only": lambda k: (k & 3) == 2,
         "dbl_bound": lambda k: (k & 1) == 1}


def series(lib, env, P, launches):
    b = env.rollout_buffers(P)
    out = []
    for _ in range(launches):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        env.rollout(P, b)
        e1.record()
        torch.cuda.synchronize()
        a = np.zeros((1024, MAXP, 12), np.int64)
        assert lib.narde_diag_pp(a.ctypes.data_as(ctypes.c_void_p)) == 0
        a = a[:, :P]
        dur = (a[:, :, 1] - a[:, :, 0]) * 0.01  # us
        kind = a[:, :, 2]
        srch = a[:, :, 3]
        seg = a[:, :, 4:12].astype(np.float64)  # s_memtime ticks per segment
        tot = dur.sum(1)
        segs = {}
        for name, f in list(KINDS.items()) + [("searching", lambda k: None)]:
            m = (srch > 0) if name == "searching" else f(kind)
            if m.any():
                segs[name] = {"share": round(float(m.mean()), 4), "ply_us": round(float(dur[m].mean()), 3),
                              "ticks": [round(float(x), 1) for x in seg[m].mean(0)[:7]]}
        slow = int(np.argmax(tot))
        per_ply = []
        for p in range(P):
            row = {"ply": int(env.ply - P + p)}
            for name, f in KINDS.items():
                m = f(kind[:, p])
                row[name] = [round(float(m.mean()), 4), round(float(dur[m, p].mean()), 3) if m.any() else None]
            m = srch[:, p] > 0
            row["searching"] = [round(float(m.mean()), 4), round(float(dur[m, p].mean()), 3) if m.any() else None]
            row["median_us"] = round(float(np.median(dur[:, p])), 3)
            row["max_us"] = round(float(dur[:, p].max()), 3)
            per_ply.append(row)
        out.append({
            "first_ply": int(env.ply - P),
            "event_span_us": round(e0.elapsed_time(e1) * 1e3, 2),
            "wave_sum_us": [round(float(np.percentile(tot, q)), 2) for q in (0, 50, 99, 100)],
            "slowest_wave": {"sum_us": round(float(tot[slow]), 2),
                             "plies_searching": int((srch[slow] > 0).sum()),
                             "plies_dbl_bound": int(((kind[slow] & 1) == 1).sum()),
                             "plies_two_bound": int(((kind[slow] & 2) == 2).sum())},
            "median_wave": {"plies_searching": float(np.median((srch > 0).sum(1))),
                            "plies_dbl_bound": float(np.median(((kind & 1) == 1).sum(1)))},
            "corr_sum_vs_searching_plies": round(float(np.corrcoef(tot, (srch > 0).sum(1))[0, 1]), 3),
            "segments_by_kind": segs,
            "per_ply": per_ply,
        })
    return out


def main():
    lib = ctypes.CDLL(LIB)
    ramp_env = VecNardeEnv(65536, device="cuda:0", seed=1, rules="full4")
    rb = ramp_env.rollout_buffers(1000)
    for _ in range(40):
        ramp_env.rollout(1000, rb)
    torch.cuda.synchronize()
    del rb
    ramp_env.close()
    res = {}
    env = VecNardeEnv(65536, device="cuda:0", seed=0, rules="full4")
    res["sync"] = series(lib, env, 20, 5)
    env.close()
    env = VecNardeEnv(65536, device="cuda:0", seed=11, rules="full4")
    env.selfplay(300)
    res["steady"] = series(lib, env, 20, 5)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
