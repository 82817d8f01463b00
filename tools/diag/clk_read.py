#!/usr/bin/env python3
"""DIAGNOSTIC (round 4): per-wave cycle accounting of one FULL4 rollout
launch from the s_memtime-instrumented build (tools/diag/build/
libnarde_clk.so, made by a build_patch.sh patch of ply_policy_full /
k_rollout_wave): each wave's lanes 0-2 leave their cycle buckets in the
stats plane.  Buckets per wave (sum over the launch's plies): draw + block
set, turn by kind (free, block-bound two dice, block-bound doubles), close,
stores; plus counts of kind-1/2 plies, the whole loop's span and its start.
argv[1] = plies per launch (default 20), argv[2] = self-play plies first."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    pre = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    n = 65536
    env = VecNardeEnv(n, device="cuda:0", seed=0, rules="full4")
    env.selfplay(pre)
    bufs = env.rollout_buffers(P)
    env.rollout(P, bufs)
    env.rollout(P, bufs)
    torch.cuda.synchronize()
    st = env.stats().cpu().numpy().astype(np.int64).reshape(n // 64, 64, 3) & 0xFFFFFFFF
    a = np.concatenate([st[:, 0, :], st[:, 1, :], st[:, 2, :2]], axis=1)
    span = st[:, 2, 2]
    start = st[:, 3, 0] | (st[:, 3, 1] << 32)
    names = ["draw_bs", "turn_free", "turn_b2", "turn_bd", "close", "store"]
    out = {"plies": P, "waves": int(a.shape[0])}
    for k, nm in enumerate(names):
        out[nm + "_mean"] = round(float(a[:, k].mean()) / P, 1)
    out["b2_plies_mean"] = round(float(a[:, 6].mean()), 2)
    out["bd_plies_mean"] = round(float(a[:, 7].mean()), 2)
    tot = a[:, :6].sum(1)
    out["sum_buckets_per_ply_mean"] = round(float(tot.mean()) / P, 1)
    out["span_per_ply_mean"] = round(float(span.mean()) / P, 1)
    out["span_p50_p90_p99_max"] = [int(np.percentile(span, q)) for q in (50, 90, 99, 100)]
    out["start_skew_p50_p99_max"] = [int(np.percentile(start - start.min(), q)) for q in (50, 99, 100)]
    out["end_skew_max"] = int((start + span).max() - (start + span).min())
    # what the slowest waves spend
    idx = np.argsort(span)[-16:]
    out["slowest16_mean"] = {nm: round(float(a[idx, k].mean()) / P, 1) for k, nm in enumerate(names)}
    out["slowest16_b2_bd_plies"] = [round(float(a[idx, 6].mean()), 2), round(float(a[idx, 7].mean()), 2)]
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
