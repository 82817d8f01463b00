#!/usr/bin/env python3
"""Record DQNAgent.act's GREEDY branch (train_deepq_pytorch.py:411-560) on the
imported reference (THIS container only; test infrastructure).

For the first steps of tests/golden/trainer.npz where act() runs, the
reference's own DQNAgent.act is called with epsilon 0 on the step's
pre-state and agent dice, its network replaced by a stub that returns fixed
Q-values: Q1 = default_rng(100000 + i).standard_normal(576) for move 1, and
for move 2 given move 1 the row base2 + tab[move1] with base2 =
default_rng(200000 + i).standard_normal(576), tab =
default_rng(7).standard_normal((576, 576)) (float32).  The chosen
(move1, move2) is recorded in tests/golden/act_greedy.npz; the tests rebuild
the same Q-values from the seeds and must pick the same codes through the
build's candidate masks (narde_act_masks) -- the reference's candidate sets
(valid_first_moves' keys, then valid_first_moves[move1], pre-move lists).
Usage: python tools/capture_act_greedy.py [--steps 2500]"""
import argparse
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import capture_golden as CG  # noqa: E402

TRAINER = "/root/reference/train_deepq_pytorch.py"


def q_values(i, tab):
    q1 = np.random.default_rng(100000 + i).standard_normal(576).astype(np.float32)
    b2 = np.random.default_rng(200000 + i).standard_normal(576).astype(np.float32)
    return q1, b2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2500)
    ap.add_argument("--out", default=os.path.join(HERE, "..", "tests", "golden", "act_greedy.npz"))
    args = ap.parse_args()
    _, NardeEnv = CG.load_reference()
    import torch

    # the trainer module makes an env at import (train_deepq_pytorch.py:182):
    # the throw-away gymnasium stub gets a make() returning the reference env
    gymnasium = sys.modules["gymnasium"]

    def make(*a, **k):
        e = NardeEnv()
        e.unwrapped = e
        return e

    gymnasium.make = make
    spec = importlib.util.spec_from_file_location("ref_trainer", TRAINER)
    tr = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tr)
    t = np.load(os.path.join(HERE, "..", "tests", "golden", "trainer.npz"), allow_pickle=False)
    tab = np.random.default_rng(7).standard_normal((576, 576)).astype(np.float32)

    class StubQ(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.q1 = self.b2 = None

        def forward(self, x, move1=None):
            if move1 is None:
                return torch.from_numpy(self.q1)[None]
            return torch.from_numpy(self.b2 + tab[int(move1.reshape(-1)[0])])[None]

    agent = tr.DQNAgent(state_size=24, action_size=576 * 576, use_decomposed_network=True,
                        use_prioritized_replay=True)
    agent.device = torch.device("cpu")
    agent.model = StubQ()
    agent.epsilon = 0.0  # np.random.rand() <= 0.0: the greedy branch
    env = NardeEnv()
    env.unwrapped = env
    steps, acts = [], []
    rows = np.nonzero(t["nvalid"] > 0)[0][:args.steps]
    for i in rows:
        g = env.game
        g.board = t["pre_board"][i].astype(np.int32).copy()
        g.borne_off_white, g.borne_off_black = int(t["pre_off"][i, 0]), int(t["pre_off"][i, 1])
        g.first_turn_white, g.first_turn_black = bool(t["pre_ft"][i, 0]), bool(t["pre_ft"][i, 1])
        env.current_player = int(t["player"][i])
        dice = [int(t["dice"][i, 0]), int(t["dice"][i, 1])]
        valid = g.get_valid_moves(dice, env.current_player)  # as the trainer loop does (:867)
        agent.model.q1, agent.model.b2 = q_values(int(i), tab)
        state = g.get_perspective_board(env.current_player)
        a = agent.act(state=state, valid_moves=valid, env=env, dice=dice, current_player=env.current_player,
                      training=True)
        steps.append(int(i))
        acts.append((int(a[0]), int(a[1])))
    np.savez_compressed(args.out, step=np.asarray(steps, np.int32), action=np.asarray(acts, np.int16),
                        meta=np.array([100000, 200000, 7], np.int64))
    print(f"wrote {args.out}: {len(steps)} greedy act() decisions")


if __name__ == "__main__":
    main()
