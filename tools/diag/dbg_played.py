#!/usr/bin/env python3
"""DIAGNOSTIC (round 4): the played words of one FULL4 ply, rollout (1-ply
k_rollout_wave) vs k_step<true>, for the libnarde.so named by $NARDE_LIB:
how many envs differ and a sample of them (played, legal word, M)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402

for n, seed in ((2125, 31337), (65536, 5)):
    a = VecNardeEnv(n, device="cuda:0", seed=seed, rules="full4")
    b = VecNardeEnv(n, device="cuda:0", seed=seed, rules="full4")
    bufs = a.rollout_buffers(1)
    for ply in range(3):
        a.rollout(1, bufs)
        _, _, _, _, info = b.step()
        torch.cuda.synchronize()
        pa = bufs["actions"][0].cpu().numpy().view(np.uint64)
        pb = info["played"].cpu().numpy().view(np.uint64)
        lg = bufs["legal"][0].cpu().numpy().view(np.uint64)
        bad = np.nonzero(pa != pb)[0]
        M = (lg >> np.uint64(56)) & np.uint64(7)
        dbl = ((lg >> np.uint64(48)) & np.uint64(15)) == ((lg >> np.uint64(52)) & np.uint64(15))
        print(f"n={n} ply={ply}: {len(bad)} of {n} differ; M of those {np.bincount(M[bad].astype(int), minlength=5)}, "
              f"doubles {int(dbl[bad].sum())}; lanes%64 {sorted(set((bad % 64).tolist()))[:12]}")
        for i in bad[:6]:
            print(f"   env {i}: rollout {int(pa[i]):#018x} step {int(pb[i]):#018x} legal {int(lg[i]):#018x}")
    a.close()
    b.close()
