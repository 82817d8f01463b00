#!/usr/bin/env python3
"""Record evaluate_model.py's loop (tests/callers.py restatement) on the
imported reference env -> tests/golden/callers.npz (THIS container only;
test infrastructure).  The GPU test replays the same loop on the drop-in
facade and must reproduce every step."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import callers  # noqa: E402
import capture_golden as CG  # noqa: E402

GAMES, NP_SEED, PY_SEED, MODEL_SEED = 6, 2025, 7, 1234


class Wrapped:
    """What gym.make('gym_narde:narde-v0') hands the caller: a wrapper whose
    .unwrapped is the NardeEnv (the throw-away gymnasium stub has no
    wrappers; TimeLimit's truncation is applied by callers.play)."""

    def __init__(self, env):
        env.unwrapped = env  # gymnasium.Env.unwrapped of an unwrapped env
        self.unwrapped = env

    def reset(self, *a, **k):
        return self.unwrapped.reset(*a, **k)

    def step(self, action):
        return self.unwrapped.step(action)


def main():
    _, NardeEnv = CG.load_reference()
    model = callers.build_model(MODEL_SEED)
    rec = callers.play(lambda: Wrapped(NardeEnv()), model, GAMES, NP_SEED, PY_SEED)
    rec["meta"] = np.array([GAMES, NP_SEED, PY_SEED, MODEL_SEED], np.int64)
    rec["fingerprint"] = np.array(callers.fingerprint(model))
    p = os.path.join(HERE, "..", "tests", "golden", "callers.npz")
    np.savez_compressed(p, **rec)
    print(f"wrote {p}: {len(rec['action'])} steps, {GAMES} games, "
          f"{int(rec['done'].sum())} ends, AI moves {(rec['player'] != 0).sum()}")


if __name__ == "__main__":
    main()
