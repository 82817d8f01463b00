#!/usr/bin/env python3
"""Latency of the scalar drop-in facade (host buffers -> PCIe -> kernels ->
PCIe -> host, synchronous), i.e. the PCIe-inclusive rate of DESIGN.md §6.
Plays seeded random-legal games through gym_narde.envs.NardeEnv."""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))

import numpy as np  # noqa: E402

from gym_narde.envs import NardeEnv  # noqa: E402


def main(steps=3000):
    rng = random.Random(0)
    env = NardeEnv()
    env.reset(seed=0)
    t_gvm = t_step = 0.0
    n_gvm = 0
    for _ in range(50):  # warm-up
        env.game.get_valid_moves([3, 5], env.current_player)
    for k in range(steps):
        st = np.random.get_state()
        dice = [np.random.randint(1, 7), np.random.randint(1, 7)]
        np.random.set_state(st)
        t0 = time.perf_counter()
        valid = env.game.get_valid_moves(dice, env.current_player)
        t_gvm += time.perf_counter() - t0
        n_gvm += 1
        m = valid[rng.randrange(len(valid))] if valid else (0, 0)
        code = m[0] * 24 + (0 if m[1] == "off" else m[1])
        t0 = time.perf_counter()
        _, _, term, _, _ = env.step((code, 0))
        t_step += time.perf_counter() - t0
        if term:
            env.reset()
    print(json.dumps({"facade_step_us": round(t_step / steps * 1e6, 2),
                      "facade_get_valid_moves_us": round(t_gvm / n_gvm * 1e6, 2),
                      "facade_steps_per_s": round(steps / t_step, 1)}))


if __name__ == "__main__":
    main()
