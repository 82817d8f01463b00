#!/usr/bin/env python3
"""Record the reference's caller loops (tests/callers.py restatements) on the
imported reference env (THIS container only; test infrastructure):

  tests/golden/callers.npz  evaluate_model.py's loop, the AI being the
                            reference's trained checkpoint
                            saved_models/narde_model_final.pt (loaded with
                            torch.load(weights_only=True)), its decisions
                            recorded; + play_against_ai.py's game loop with a
                            scripted keyboard and the rendered text
  tests/golden/trainer.npz  train_deepq_pytorch.py:855-1081's env-facing
                            calls with its exploring agent

The GPU tests replay the same loops on the drop-in facade and must
reproduce every step (tests/test_gpu_callers.py).
The checkpoint itself is not a fixture and never travels."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import callers  # noqa: E402
import capture_golden as CG  # noqa: E402

CHECKPOINT = "/root/reference/saved_models/narde_model_final.pt"
GAMES, NP_SEED, PY_SEED = 6, 2025, 7
HUMAN_NP_SEED, HUMAN_KEY_SEED = 31, 5
TRAIN_EPISODES, TRAIN_NP_SEED, TRAIN_PY_SEED = 12, 4242, 99


class Wrapped:
    """What gym.make('gym_narde:narde-v0') hands the caller: a wrapper whose
    .unwrapped is the NardeEnv (the throw-away gymnasium stub has no
    wrappers; TimeLimit's truncation is applied by the loops)."""

    def __init__(self, env):
        env.unwrapped = env  # gymnasium.Env.unwrapped of an unwrapped env
        self.unwrapped = env

    def reset(self, *a, **k):
        return self.unwrapped.reset(*a, **k)

    def step(self, action):
        return self.unwrapped.step(action)

    def render(self):
        return self.unwrapped.render()


def main():
    _, NardeEnv = CG.load_reference()
    model = callers.load_model(CHECKPOINT)
    out = {}
    ai = callers.ModelAI(model)
    rec = callers.play(lambda: Wrapped(NardeEnv()), ai, GAMES, NP_SEED, PY_SEED)
    out.update(rec)
    out.update(ai.record("ai"))
    out["meta"] = np.array([GAMES, NP_SEED, PY_SEED], np.int64)
    out["fingerprint"] = np.array(callers.fingerprint(model))
    ai_h = callers.ModelAI(model)
    hum = callers.play_human(lambda **k: Wrapped(NardeEnv(**k)), ai_h, HUMAN_NP_SEED, HUMAN_KEY_SEED)
    out.update({f"human_{k}": v for k, v in hum.items()})
    out.update(ai_h.record("human_ai"))
    out["human_meta"] = np.array([HUMAN_NP_SEED, HUMAN_KEY_SEED], np.int64)
    p = os.path.join(HERE, "..", "tests", "golden", "callers.npz")
    np.savez_compressed(p, **out)
    print(f"wrote {p}: evaluate {len(rec['action'])} steps / {GAMES} games / {len(ai.actions)} AI "
          f"decisions; play_against_ai {len(hum['action'])} steps, {len(ai_h.actions)} AI decisions, "
          f"{len(hum['text'])} bytes of text")
    tr = callers.train_loop(lambda: Wrapped(NardeEnv()), TRAIN_EPISODES, TRAIN_NP_SEED, TRAIN_PY_SEED)
    tr["meta"] = np.array([TRAIN_EPISODES, TRAIN_NP_SEED, TRAIN_PY_SEED], np.int64)
    p = os.path.join(HERE, "..", "tests", "golden", "trainer.npz")
    np.savez_compressed(p, **tr)
    print(f"wrote {p}: {len(tr['action'])} steps, {int(tr['done'].sum())} episode ends, "
          f"{int((tr['nvalid'] == 0).sum())} no-move steps ({len(tr['blocks'])} block checks), "
          f"{len(tr['combos'])} act() combinations, shaped rewards in "
          f"[{tr['shaped'].min():.1f}, {tr['shaped'].max():.1f}]")


if __name__ == "__main__":
    main()
