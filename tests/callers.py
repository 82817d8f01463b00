"""Restatement of the reference's caller loop evaluate_model.py (agents
:17-134, evaluate loop :136-196), parametrised by the env factory, so the
SAME loop runs on the imported reference (tools/capture_callers.py, in the
build container) and on the drop-in facade (tests/test_gpu_callers.py, on the
GPU box).  Test infrastructure only.

Kept from the reference: the RandomAgent draws (random.choice twice,
:26-28), the AIAgent's use of env.unwrapped.game.get_perspective_board /
get_valid_moves and its decomposed argmax (:61-127), the agents rolling their
own dice with np.random.randint while env.step rolls again (:169-176), the
winner read from env.unwrapped.current_player (:181-183), and TimeLimit 1000
(gym_narde/__init__.py:3-7).  The network is DecomposedDQN's architecture
(train_deepq_pytorch.py:184-222) with seeded random weights on the CPU: the
reference checkpoint is not a fixture and never travels.
"""
import random

import numpy as np
import torch
import torch.nn as nn

WHITE, BLACK = 1, -1


class Net(nn.Module):
    """train_deepq_pytorch.py:184-231 (one-hot concat kept, as the reference)."""

    def __init__(self, state_size=24, moves=576):
        super().__init__()
        self.moves = moves
        self.feature_network = nn.Sequential(nn.Linear(state_size, 256), nn.ReLU(),
                                             nn.Linear(256, 256), nn.ReLU())
        self.move1_head = nn.Linear(256, moves)
        self.move2_head = nn.Linear(256 + moves, moves)

    def forward(self, x, selected_move1=None):
        f = self.feature_network(x)
        q1 = self.move1_head(f)
        if selected_move1 is None:
            return q1
        oh = torch.zeros(x.size(0), self.moves)
        oh.scatter_(1, selected_move1.unsqueeze(1), 1)
        return self.move2_head(torch.cat((f, oh), dim=1))


def build_model(seed=1234):
    torch.manual_seed(seed)
    m = Net()
    m.eval()
    return m


def fingerprint(model):
    with torch.no_grad():
        return float(sum(p.double().sum() for p in model.parameters()))


def code(m):
    f, t = m
    return f * 24 + (0 if t == "off" else t)


def random_action(env, color, dice, rng):  # evaluate_model.py:22-39
    valid = env.game.get_valid_moves(dice, color)
    if len(valid) == 0:
        return (0, 0)
    m1 = rng.choice(valid)
    m2 = rng.choice(valid) if len(valid) > 1 else m1
    return (code(m1), code(m2))


def ai_action(env, color, dice, model):  # evaluate_model.py:61-127
    state = env.unwrapped.game.get_perspective_board(color)
    x = torch.FloatTensor(np.asarray(state)).unsqueeze(0)
    valid = env.unwrapped.game.get_valid_moves(dice, color)
    if len(valid) == 0:
        return (0, 0)
    first = {}
    for m1 in valid:
        first[code(m1) if m1[1] != "off" else m1[0] * 24] = [0]
    with torch.no_grad():
        q1 = model(x)
        keys = list(first.keys())
        v = q1.squeeze(0).index_select(0, torch.tensor(keys))
        best1 = keys[int(torch.argmax(v).item())]
        c2 = first[best1]
        q2 = model(x, torch.tensor([best1]))
        v2 = q2.squeeze(0).index_select(0, torch.tensor(c2))
        best2 = c2[int(torch.argmax(v2).item())]
    return (best1, best2)


def play(make_env, model, games, np_seed, py_seed, max_steps=1000):
    """evaluate_model.py:136-196 with recording.  Returns per-step arrays."""
    np.random.seed(np_seed)
    rng = random.Random(py_seed)
    rec = {k: [] for k in ("game", "ai_color", "dice", "action", "obs", "reward", "done", "player")}
    env = make_env()
    for g in range(games):
        ai_color = WHITE if np.random.rand() > 0.5 else BLACK
        obs, _ = env.reset()
        cur = env.unwrapped.current_player
        steps = 0
        while True:
            steps += 1
            dice = [np.random.randint(1, 7), np.random.randint(1, 7)]
            if cur == ai_color:
                action = ai_action(env.unwrapped, cur, dice, model)
            else:
                action = random_action(env.unwrapped, cur, dice, rng)
            obs, reward, term, trunc, _ = env.step(action)
            trunc = trunc or steps >= max_steps
            rec["game"].append(g)
            rec["ai_color"].append(ai_color)
            rec["dice"].append(dice)
            rec["action"].append(action)
            rec["obs"].append(np.asarray(obs, dtype=np.int8))
            rec["reward"].append(int(reward))
            rec["done"].append(int(bool(term) or bool(trunc)))
            rec["player"].append(int(env.unwrapped.current_player))
            if term or trunc:
                break
            cur = env.unwrapped.current_player
    out = {k: np.asarray(v) for k, v in rec.items()}
    out["dice"] = out["dice"].astype(np.uint8)
    out["action"] = out["action"].astype(np.int16)
    out["obs"] = np.stack(rec["obs"]).astype(np.int8)
    return out
