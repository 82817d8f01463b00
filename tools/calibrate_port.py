#!/usr/bin/env python3
"""Calibrate the CPU baseline port (oracle/narde_port.py) against the real
reference NardeEnv, in THIS container only (the reference never travels).

Both run random-legal self-play on one core with injected dice:
  * reference: NardeEnv.step timed alone; the policy (which needs the two
    get_valid_moves lists ahead of the step) runs outside the timer;
  * port: PortEnv.step with the policy inside the step (it draws from the
    step's own lists: one randrange + encode per move, ~1% of a step).
Prints steps/s of each and the port/reference ratio (quoted in DESIGN.md).
"""
import copy
import os
import random
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))

import capture_golden as cg  # noqa: E402
import narde_port  # noqa: E402


def time_reference(NardeEnv, seconds, seed=0):
    rng = random.Random(seed)
    np.random.seed(seed)
    env = NardeEnv()
    env.reset(seed=seed)
    steps, spent, n = 0, 0.0, 0
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        st = np.random.get_state()
        dice = [int(np.random.randint(1, 7)), int(np.random.randint(1, 7))]
        np.random.set_state(st)
        a = cg.random_legal_action(copy.deepcopy(env.game), dice, env.current_player, rng)
        t0 = time.perf_counter()
        _, _, done, _, _ = env.step(a)
        n += 1
        if done or n >= 1000:
            env.reset()
            n = 0
        spent += time.perf_counter() - t0
        steps += 1
    return steps / spent


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    _, NardeEnv = cg.load_reference()
    ref = time_reference(NardeEnv, seconds)
    s, w, _ = narde_port.selfplay_port(64, seconds=seconds, seed=0)
    port = s / w
    print(f"reference NardeEnv.step: {ref:,.0f} steps/s/core")
    print(f"port PortEnv.step:       {port:,.0f} steps/s/core")
    print(f"port/reference ratio:    {port / ref:.3f}")


if __name__ == "__main__":
    main()
