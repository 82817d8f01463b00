#!/usr/bin/env python3
"""DIAGNOSTIC (round 5): where k_step<true>'s time goes -- per-wave cycles
of one FULL4 ply against the kinds of turn the wave holds.  Needs the
`kclk` build (tools/diag/gpu_r05m.sh: k_step<true> with s_memtime around
the ply; lanes 0-3 of each wave overwrite their reward with the wave's
cycles and its counts of block-bound doubles / block-bound two-dice /
searching doubles lanes -- wrong rewards, diagnostic only).  Prints one
JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    n, warm, steps = 65536, 300, 200
    env = VecNardeEnv(n, device="cuda:0", seed=0, rules="full4")
    for _ in range(warm):
        env.step()
    torch.cuda.synchronize()
    rows = []
    for _ in range(steps):
        env.step()
        rows.append(env.reward.view(-1, 64)[:, :4].clone())
    torch.cuda.synchronize()
    r = torch.stack(rows).cpu().numpy().astype("int64")  # [steps, waves, 4]
    cyc, nbd, nb2, nsr = r[..., 0], r[..., 1], r[..., 2], r[..., 3]
    import numpy as np
    out = {"steps": steps, "waves": int(cyc.shape[1])}
    out["median_wave_cycles"] = float(np.median(cyc))
    out["mean_max_wave_cycles"] = float(cyc.max(axis=1).mean())
    kinds = {}
    for name, m in (("free", (nbd == 0) & (nb2 == 0)), ("two_dice_bound_only", (nbd == 0) & (nb2 > 0)),
                    ("dbl_bound_no_search", (nbd > 0) & (nsr == 0)), ("search_1", nsr == 1),
                    ("search_2", nsr == 2), ("search_3plus", nsr >= 3)):
        if m.any():
            kinds[name] = {"share": round(float(m.mean()), 5), "mean": round(float(cyc[m].mean())),
                           "p99": round(float(np.percentile(cyc[m], 99))), "max": int(cyc[m].max())}
    out["by_kind"] = kinds
    am = cyc.argmax(axis=1)
    mx = [(int(cyc[s, w]), int(nbd[s, w]), int(nb2[s, w]), int(nsr[s, w])) for s, w in enumerate(am)]
    out["slowest_wave_kinds"] = {
        "search>=1": sum(1 for m in mx if m[3] >= 1), "dbl_bound_no_search": sum(1 for m in mx if m[1] and not m[3]),
        "two_dice_only": sum(1 for m in mx if not m[1] and m[2]), "free": sum(1 for m in mx if not m[1] and not m[2])}
    out["slowest_examples"] = sorted(mx, reverse=True)[:10]
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
