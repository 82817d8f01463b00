#!/usr/bin/env python3
"""DIAGNOSTIC: where k_rollout_full and per-ply k_step<full> part (the
launch-boundary test of tests/test_gpu_full4.py, with details)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    n, seed = 2048, 31337
    a = VecNardeEnv(n, device="cuda:0", rules="full4", seed=seed)
    b = VecNardeEnv(n, device="cuda:0", rules="full4", seed=seed)
    bufs = a.rollout_buffers(70)
    got = {k: [] for k in bufs}
    for plies in (1, 29, 70):
        a.rollout(plies, bufs)
        torch.cuda.synchronize()
        for k, v in bufs.items():
            got[k].append(v[:plies].cpu().numpy().copy())
    got = {k: np.concatenate(v) for k, v in got.items()}
    ref = {k: [] for k in ("obs", "legal", "actions", "reward")}
    for p in range(100):
        obs, rew, term, trunc, info = b.step()
        torch.cuda.synchronize()
        ref["obs"].append(obs.cpu().numpy().copy())
        ref["legal"].append(info["legal"].cpu().numpy().copy())
        ref["actions"].append(info["played"].cpu().numpy().copy())
        ref["reward"].append(rew.cpu().numpy().copy())
    ref = {k: np.stack(v) for k, v in ref.items()}
    for k in ref:
        g = got[k].reshape(100, n, -1)
        r = ref[k].reshape(100, n, -1)
        bad = np.nonzero((g != r).any(axis=2))
        print(k, "mismatching (ply, env) pairs:", len(bad[0]))
        if len(bad[0]):
            first = sorted(zip(bad[0].tolist(), bad[1].tolist()))[:8]
            print("  first:", first)
    g = got["obs"].reshape(100, n, -1)
    r = ref["obs"].reshape(100, n, -1)
    bad = np.nonzero((g != r).any(axis=2))
    if len(bad[0]):
        p0 = int(bad[0].min())
        envs = sorted(set(bad[1][bad[0] == p0].tolist()))[:4]
        for e in envs:
            print(f"env {e} (wave {e // 64}, lane {e % 64}) first bad ply {p0}")
            for p in range(max(0, p0 - 3), min(100, p0 + 2)):
                gl = got["legal"].reshape(100, n)[p, e]
                rl = ref["legal"].reshape(100, n)[p, e]
                ga = got["actions"].reshape(100, n, -1)[p, e]
                ra = ref["actions"].reshape(100, n, -1)[p, e]
                print(f"  ply {p}: legal got {int(gl) & (2**64 - 1):016x} ref {int(rl) & (2**64 - 1):016x}"
                      f" played got {ga.tobytes().hex()} ref {ra.tobytes().hex()}")
                print("     obs got", g[p, e].tolist())
                print("     obs ref", r[p, e].tolist())


if __name__ == "__main__":
    main()
