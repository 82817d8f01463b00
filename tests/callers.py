"""Restatements of the reference's three caller loops, parametrised by the env
factory, so the SAME loop runs on the imported reference
(tools/capture_callers.py, in the build container) and on the drop-in facade
(tests/test_gpu_callers.py, on the GPU box).  Test infrastructure only.

  play         evaluate_model.py:136-196 -- the AI (the trained checkpoint
               saved_models/narde_model_final.pt, :41-134) against the random
               agent (:17-39)
  play_human   play_against_ai.py:179-237 -- the AI against HumanPlayer
               (:110-177) with a scripted keyboard, env.render() captured
  train_loop   train_deepq_pytorch.py:855-1081 -- every env-facing call of
               the trainer's episode loop with its agent exploring (epsilon 1,
               the trainer's starting value): act()'s combination lists from
               get_valid_moves(temp_dice) (:411-515), the step, the borne-off
               reward shaping (:892-912), and the no-move diagnostics reading
               first_turn_* (:1048) and _violates_block_rule on mutated board
               copies (:1066-1076)

Kept from the reference: the agents rolling their own dice with
np.random.randint while env.step rolls again, the RandomAgent's
random.choice draws, the AI's decomposed argmax over the perspective board,
the winner read from env.unwrapped.current_player, TimeLimit 1000
(gym_narde/__init__.py:3-7).

The checkpoint is loaded only in the capture (torch.load weights_only=True,
this container); it never travels.  The AI is a callable: ModelAI runs the
network and records each decision (the perspective board and move list it
saw, the action it chose); ReplayAI, on the GPU box, asserts that the
facade shows it the same board and list and plays the recorded action.  So
the facade is driven through exactly the trajectory the trained policy
took on the reference.
"""
import contextlib
import io
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


def load_model(path):
    """The reference checkpoint (a DecomposedDQN state_dict saved on MPS)."""
    m = Net()
    m.load_state_dict(torch.load(path, weights_only=True, map_location="cpu"))
    m.eval()
    return m


def fingerprint(model):
    with torch.no_grad():
        return float(sum(p.double().sum() for p in model.parameters()))


def code(m):
    f, t = m
    return f * 24 + (0 if t == "off" else t)


def enc_list(moves):
    out = np.full((64, 2), -1, np.int8)
    for i, (f, t) in enumerate(moves):
        out[i] = (f, 24 if t == "off" else t)
    return out


def random_action(env, color, dice, rng):  # evaluate_model.py:22-39
    valid = env.game.get_valid_moves(dice, color)
    if len(valid) == 0:
        return (0, 0)
    m1 = rng.choice(valid)
    m2 = rng.choice(valid) if len(valid) > 1 else m1
    return (code(m1), code(m2))


class ModelAI:
    """AIAgent.choose_best_action (evaluate_model.py:61-127, identical in
    play_against_ai.py:36-108) with the network; records every decision."""

    def __init__(self, model):
        self.model = model
        self.boards, self.lists, self.counts, self.actions = [], [], [], []

    def __call__(self, env, color, dice):
        state = env.unwrapped.game.get_perspective_board(color)
        x = torch.FloatTensor(np.asarray(state)).unsqueeze(0)
        valid = env.unwrapped.game.get_valid_moves(dice, color)
        self.boards.append(np.asarray(state, np.int8))
        self.lists.append(enc_list(valid))
        self.counts.append(len(valid))
        if len(valid) == 0:
            action = (0, 0)
        else:
            first = {}
            for m1 in valid:
                first[code(m1) if m1[1] != "off" else m1[0] * 24] = [0]
            with torch.no_grad():
                q1 = self.model(x)
                keys = list(first.keys())
                v = q1.squeeze(0).index_select(0, torch.tensor(keys))
                best1 = keys[int(torch.argmax(v).item())]
                c2 = first[best1]
                q2 = self.model(x, torch.tensor([best1]))
                v2 = q2.squeeze(0).index_select(0, torch.tensor(c2))
                best2 = c2[int(torch.argmax(v2).item())]
            action = (best1, best2)
        self.actions.append(action)
        return action

    def record(self, prefix):
        return {f"{prefix}_board": np.asarray(self.boards, np.int8).reshape(-1, 24),
                f"{prefix}_list": np.asarray(self.lists, np.int8).reshape(-1, 64, 2),
                f"{prefix}_count": np.asarray(self.counts, np.int16),
                f"{prefix}_action": np.asarray(self.actions, np.int16).reshape(-1, 2)}


class ReplayAI:
    """The recorded AI: checks that the env shows the board and move list the
    trained policy saw on the reference, then plays its recorded action."""

    def __init__(self, d, prefix):
        self.board, self.list = d[f"{prefix}_board"], d[f"{prefix}_list"]
        self.count, self.action = d[f"{prefix}_count"], d[f"{prefix}_action"]
        self.k = 0

    def __call__(self, env, color, dice):
        k = self.k
        state = env.unwrapped.game.get_perspective_board(color)
        valid = env.unwrapped.game.get_valid_moves(dice, color)
        assert np.array_equal(np.asarray(state, np.int8), self.board[k]), f"AI decision {k}: board"
        assert len(valid) == self.count[k] and np.array_equal(enc_list(valid), self.list[k]), \
            f"AI decision {k}: move list"
        self.k += 1
        return tuple(int(x) for x in self.action[k])


def play(make_env, ai, games, np_seed, py_seed, max_steps=1000):
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
                action = ai(env, cur, dice)
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


def human_action(env, color, dice, keys):  # play_against_ai.py:114-177, keyboard scripted
    """HumanPlayer.choose_best_action with `keys` (an iterator of the
    strings input() would return) instead of the keyboard; its prints go to
    the captured stdout like the rest of the game."""
    print(f"\nYour turn ({color})")
    env.render()
    print(f"Dice rolls: {dice}")
    valid = env.unwrapped.game.get_valid_moves(dice, color)
    if len(valid) == 0:
        print("No valid moves. Skipping turn.")
        return (0, 0)
    for i, (f, t) in enumerate(valid):
        print(f"{i + 1}. From point {f + 1} to point {'off' if t == 'off' else t + 1}")
    while True:
        choice = next(keys)
        if not choice:
            move1 = valid[0]
            break
        try:
            idx = int(choice) - 1
        except ValueError:
            move1 = valid[0]
            break
        if idx == -1:
            return (0, 0)
        if 0 <= idx < len(valid):
            move1 = valid[idx]
            break
    move2 = valid[0]
    return (code(move1), code(move2))


def _keys(seed):
    """What a player types: mostly a listed move, sometimes Enter, an
    out-of-range number, a word, or 0 (skip)."""
    rng = random.Random(seed)
    while True:
        r = rng.random()
        if r < 0.05:
            yield ""
        elif r < 0.08:
            yield "0"
        elif r < 0.11:
            yield "99"
        elif r < 0.13:
            yield "move"
        else:
            yield str(rng.randint(1, 6))


def play_human(make_env, ai, np_seed, key_seed, max_steps=1000):
    """play_against_ai.py:179-237 (one game) with recording; the full text
    the game prints (both agents' output and every env.render()) is kept."""
    np.random.seed(np_seed)
    keys = _keys(key_seed)
    buf = io.StringIO()
    rec = {k: [] for k in ("dice", "action", "obs", "reward", "done", "player")}
    with contextlib.redirect_stdout(buf):
        env = make_env(render_mode="human")
        human_color = WHITE if np.random.rand() > 0.5 else BLACK
        ai_color = BLACK if human_color == WHITE else WHITE
        obs, _ = env.reset()
        cur = env.unwrapped.current_player
        for _ in range(max_steps):
            dice = [np.random.randint(1, 7), np.random.randint(1, 7)]
            print(f"Dice rolled: {dice}")
            if cur == ai_color:
                action = ai(env, cur, dice)
            else:
                action = human_action(env, cur, dice, keys)
            obs, reward, term, trunc, _ = env.step(action)
            env.render()
            rec["dice"].append(dice)
            rec["action"].append(action)
            rec["obs"].append(np.asarray(obs, np.int8))
            rec["reward"].append(int(reward))
            rec["done"].append(int(bool(term) or bool(trunc)))
            rec["player"].append(int(env.unwrapped.current_player))
            if term or trunc:
                print(f"Game over! Winner: {env.unwrapped.current_player}")
                break
            cur = env.unwrapped.current_player
    out = {k: np.asarray(v) for k, v in rec.items()}
    out["dice"] = out["dice"].astype(np.uint8)
    out["action"] = out["action"].astype(np.int16)
    out["obs"] = np.stack(rec["obs"]).astype(np.int8)
    out["human_color"] = np.array(human_color, np.int8)
    out["text"] = np.frombuffer(buf.getvalue().encode(), np.uint8)
    return out


def act_explore(env, valid_moves, dice, current_player, rng):
    """DQNAgent.act (train_deepq_pytorch.py:411-515) on its exploration
    branch (epsilon = 1.0, the trainer's starting value): every first move's
    remaining dice and their get_valid_moves list, then np.random.rand() <=
    epsilon and random.choice over the combinations.  Returns the action and
    the combination list."""
    combos = []
    for move1 in valid_moves:
        f1, t1 = move1
        c1 = f1 * 24 if t1 == "off" else f1 * 24 + t1
        temp = list(dice)
        if t1 == "off":
            dist = f1 + 1
            match = next((d for d in temp if d >= dist), None)
            if match is None and temp:
                match = max(temp)
        else:
            dist = abs(f1 - t1)
            match = next((d for d in temp if d == dist), None)
            if match is None and temp:
                match = temp[0]
        if match is not None and match in temp:
            temp.remove(match)
        remaining = env.unwrapped.game.get_valid_moves(temp, current_player) if temp else []
        if not remaining:
            combos.append((c1, 0))
        else:
            for f2, t2 in remaining:
                combos.append((c1, f2 * 24 if t2 == "off" else f2 * 24 + t2))
    if not combos:
        return (0, 0), combos
    assert np.random.rand() <= 1.0  # the draw the reference makes (:514)
    return rng.choice(combos), combos


def _rotate(board):  # gym_narde/envs/narde.py:16-17, as train_deepq_pytorch imports it
    return np.concatenate((-board[12:], -board[:12])).astype(np.int32)


def no_move_diagnostics(env, next_state, dice):
    """train_deepq_pytorch.py:1013-1076 (the verbose no-move branch): the
    first_turn_* read and _violates_block_rule on every mutated board copy.
    Returns (first_turn read or -1, block-rule results)."""
    cp = env.unwrapped.current_player
    own = [i for i, v in enumerate(next_state) if (v > 0 if cp == 1 else v < 0)]
    all_moves = [(p, p - d) for p in own for d in dice if 0 <= p - d < 24]
    head = 23 if cp == 1 else 11
    ft = -1
    if head in own:
        ft = int(bool(env.unwrapped.game.first_turn_white if cp == 1 else env.unwrapped.game.first_turn_black))
    test_board = np.array(next_state).copy() if cp == 1 else _rotate(np.array(next_state))
    blocks = []
    for f, t in all_moves:
        b = test_board.copy()
        b[f] -= 1
        b[t] += 1
        blocks.append(int(bool(env.unwrapped.game._violates_block_rule(b))))
    return ft, blocks


def _peek_dice():
    """The two draws env.step is about to make (narde_env.py:29)."""
    st = np.random.get_state()
    d = [np.random.randint(1, 7), np.random.randint(1, 7)]
    np.random.set_state(st)
    return d


def train_loop(make_env, episodes, np_seed, py_seed, max_steps=1000):
    """train_deepq_pytorch.py:855-1081's env-facing calls, recorded per step.
    pre_* is the game state before env.step, env_dice the step's own roll
    (peeked from the RNG state), shaped the reward after the shaping
    (float64, as the reference), seen_* the borne-off trackers after it."""
    np.random.seed(np_seed)
    rng = random.Random(py_seed)
    env = make_env()
    keys = ("episode", "dice", "env_dice", "player", "nvalid", "action", "obs", "reward", "shaped",
            "done", "truncated", "seen_w", "seen_b", "pre_board", "pre_off", "pre_ft", "ft_read")
    rec = {k: [] for k in keys}
    combos_flat, combos_len, blocks_flat, blocks_len = [], [], [], []
    for e in range(episodes):
        state, _ = env.reset()
        total_white_off = 0
        total_black_off = 0
        for step in range(max_steps):
            dice = [np.random.randint(1, 7), np.random.randint(1, 7)]
            cp = env.unwrapped.current_player
            valid = env.unwrapped.game.get_valid_moves(dice, cp)
            g = env.unwrapped.game
            rec["pre_board"].append(np.asarray(g.board, np.int8).copy())
            rec["pre_off"].append((g.borne_off_white, g.borne_off_black))
            rec["pre_ft"].append((int(bool(g.first_turn_white)), int(bool(g.first_turn_black))))
            combos = []
            if len(valid) == 0:
                action = (0, 0)
                rec["env_dice"].append(_peek_dice())
                next_state, reward, done, trunc, _ = env.step(action)
                env_reward = reward
                trunc = trunc or step + 1 >= max_steps
                done = done or trunc
            else:
                action, combos = act_explore(env, valid, dice, cp, rng)
                rec["env_dice"].append(_peek_dice())
                next_state, reward, done, trunc, _ = env.step(action)
                env_reward = reward
                trunc = trunc or step + 1 >= max_steps
                done = done or trunc
                if env.unwrapped.current_player == 1:
                    borne_off_before = total_white_off
                    total_white_off = env.unwrapped.game.borne_off_white
                    newly = total_white_off - borne_off_before
                    if newly > 0:
                        reward += 1.0 * newly
                    reward += 0.1 * total_white_off
                elif env.unwrapped.current_player == -1:
                    borne_off_before = total_black_off
                    total_black_off = env.unwrapped.game.borne_off_black
                    newly = total_black_off - borne_off_before
                    if newly > 0:
                        reward += 1.0 * newly
                    reward += 0.1 * total_black_off
            ft_read, blocks = -1, []
            if len(valid) == 0:
                ft_read, blocks = no_move_diagnostics(env, next_state, dice)
            rec["episode"].append(e)
            rec["dice"].append(dice)
            rec["player"].append(cp)
            rec["nvalid"].append(len(valid))
            rec["action"].append(action)
            rec["obs"].append(np.asarray(next_state, np.int8))
            rec["reward"].append(int(env_reward))
            rec["shaped"].append(float(reward))
            rec["done"].append(int(bool(done)))
            rec["truncated"].append(int(bool(trunc)))
            rec["seen_w"].append(total_white_off)
            rec["seen_b"].append(total_black_off)
            rec["ft_read"].append(ft_read)
            combos_flat.extend(combos)
            combos_len.append(len(combos))
            blocks_flat.extend(blocks)
            blocks_len.append(len(blocks))
            if done:
                break
    out = {k: np.asarray(v) for k, v in rec.items()}
    for k, dt in (("dice", np.uint8), ("env_dice", np.uint8), ("action", np.int16), ("obs", np.int8),
                  ("pre_board", np.int8), ("pre_off", np.uint8), ("pre_ft", np.uint8), ("player", np.int8),
                  ("nvalid", np.int16), ("shaped", np.float64), ("seen_w", np.int8), ("seen_b", np.int8),
                  ("ft_read", np.int8), ("done", np.uint8), ("truncated", np.uint8), ("episode", np.int16)):
        out[k] = out[k].astype(dt)
    out["combos"] = np.asarray(combos_flat, np.int16).reshape(-1, 2)
    out["combos_len"] = np.asarray(combos_len, np.int32)
    out["blocks"] = np.asarray(blocks_flat, np.uint8)
    out["blocks_len"] = np.asarray(blocks_len, np.int32)
    return out
