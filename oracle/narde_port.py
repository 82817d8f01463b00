"""Pure-Python restatement of the reference env (the CPU baseline "port").

TEST / BASELINE INFRASTRUCTURE ONLY -- imported by tests/ and bench.py's
cpu_baseline leg, never by the product.  It keeps the reference's per-env
Python/numpy loop structure (one object per env, int32 numpy board, list of
(from, to) tuples with 'off') so its speed stands in for the reference's on
the GPU box, where the reference itself cannot go.  Checked against the
golden vectors in tests/test_oracle_golden.py.

Follows /root/reference/gym_narde/envs/narde.py:16-192 and
/root/reference/gym_narde/envs/narde_env.py:27-141.
"""
import random

import numpy as np


def rotate_board(board):  # narde.py:16-17
    return np.concatenate((-board[12:], -board[:12])).astype(np.int32)


class PortNarde:
    def __init__(self):  # narde.py:21-29
        self.board = np.zeros(24, dtype=np.int32)
        self.board[23] = 15
        self.board[11] = -15
        self.borne_off_white = 0
        self.borne_off_black = 0
        self.first_turn_white = True
        self.first_turn_black = True

    def get_perspective_board(self, current_player):  # narde.py:31-34
        if current_player == 1:
            return self.board.copy()
        return rotate_board(self.board)

    def execute_rotated_move(self, move, current_player):  # narde.py:36-56
        if current_player != 1:
            f, t = move
            move = ((f + 12) % 24, "off") if t == "off" else ((f + 12) % 24, (t + 12) % 24)
        self._execute_move(move)
        if current_player == 1:
            self.first_turn_white = False
        else:
            self.first_turn_black = False

    def get_valid_moves(self, roll, current_player=1):  # narde.py:58-92
        roll = sorted(roll, reverse=True)
        board = self.board if current_player == 1 else rotate_board(self.board)
        moves = []
        for die in roll:
            for pos in range(24):
                if board[pos] <= 0:
                    continue
                new_pos = pos - die
                if 0 <= new_pos < 24:
                    if board[new_pos] >= 0:
                        moves.append((pos, new_pos))
                elif new_pos < 0:
                    if np.sum(np.maximum(board[6:], 0)) == 0 and die >= pos + 1:
                        moves.append((pos, "off"))
        filtered = []
        for move in moves:
            bc = board.copy()
            bc[move[0]] -= 1
            if move[1] != "off":
                bc[move[1]] += 1
            if not self._violates_block_rule(bc):
                filtered.append(move)
        first_turn = self.first_turn_white if current_player == 1 else self.first_turn_black
        max_head = 2 if first_turn and sorted(roll) in [[3, 3], [4, 4], [6, 6]] else 1
        allowed, n = [], 0
        for move in filtered:  # narde.py:127-137
            if move[0] == 23:
                if n < max_head:
                    allowed.append(move)
                    n += 1
            else:
                allowed.append(move)
        return allowed

    def _execute_move(self, move):  # narde.py:108-125
        f, t = move
        if t == "off":
            if self.board[f] > 0:
                self.board[f] -= 1
                self.borne_off_white += 1
            else:
                self.board[f] += 1
                self.borne_off_black += 1
        else:
            if self.board[f] > 0:
                self.board[f] -= 1
                self.board[t] += 1
            else:
                self.board[f] += 1
                self.board[t] -= 1

    @staticmethod
    def _violates_block_rule(board):  # narde.py:139-184
        i = 0
        while i < 24:
            if board[i] > 0:
                start = i
                j = i + 1
                while j < 24 and board[j] > 0:
                    j += 1
                if j - start >= 6:
                    ahead = False
                    for k in range(0, start):
                        if board[k] < 0:
                            ahead = True
                            break
                    if not ahead:
                        return True
                i = j
            else:
                i += 1
        return False


def _decode(code):  # narde_env.py:238-254
    f, t = code // 24, code % 24
    return (f, "off") if (t == 0 and 0 <= f <= 5) else (f, t)


def _encode(m):
    return m[0] * 24 + (0 if m[1] == "off" else m[1])


class PortEnv:
    """NardeEnv (narde_env.py:7-141) with injectable dice and an optional
    in-step random legal policy (picks from the step's own lists)."""

    def __init__(self):
        self.game = PortNarde()
        self.current_player = 1

    def reset_with(self, white_roll, black_roll):  # narde_env.py:105-120
        self.game = PortNarde()
        self.current_player = 1 if white_roll > black_roll else -1
        return self.game.get_perspective_board(self.current_player)

    def _check_game_ended(self):  # narde_env.py:134-141
        g = self.game
        if self.current_player == 1 and g.borne_off_white == 15:
            return True, 1 if g.borne_off_black > 0 else 2
        if self.current_player == -1 and g.borne_off_black == 15:
            return True, 1 if g.borne_off_white > 0 else 2
        return False, 0

    def step(self, dice, action=None, rng=None):  # narde_env.py:27-103
        g = self.game
        valid = g.get_valid_moves(dice, self.current_player)
        if len(valid) == 0:
            done, reward = self._check_game_ended()
            if not done:
                self.current_player *= -1
            return g.get_perspective_board(self.current_player), reward, done
        elif len(valid) == 1:
            g.execute_rotated_move(valid[0], self.current_player)
        else:
            if action is None:
                c1 = _encode(valid[rng.randrange(len(valid))])
            else:
                c1 = action[0]
            m1 = _decode(c1)
            if m1 in valid:
                g.execute_rotated_move(m1, self.current_player)
                dist = m1[0] + 1 if m1[1] == "off" else abs(m1[0] - m1[1])
                temp = list(dice)
                if dist in temp:
                    temp.remove(dist)
                elif temp:
                    temp.pop(0)
                if temp:
                    nv = g.get_valid_moves(temp, self.current_player)
                    if action is None:
                        c2 = _encode(nv[rng.randrange(len(nv))]) if nv else 0
                    else:
                        c2 = action[1]
                    m2 = _decode(c2)
                    if m2 in nv:
                        g.execute_rotated_move(m2, self.current_player)
        done, reward = self._check_game_ended()
        if not done:
            self.current_player *= -1
        return g.get_perspective_board(self.current_player), reward, done


def selfplay_port(n_envs, seconds=None, plies=None, seed=0, max_steps=1000):
    """Random-legal self-play over n_envs PortEnv objects, ply-major like the
    GPU lockstep.  Stops after `plies` plies or once `seconds` elapsed (checked
    per ply).  Returns (env_steps, wall_seconds, episodes)."""
    import time

    rng = random.Random(seed)
    nprng = np.random.RandomState(seed)
    envs = [PortEnv() for _ in range(n_envs)]
    elapsed = [0] * n_envs
    for e in envs:
        while True:
            w, b = nprng.randint(1, 7), nprng.randint(1, 7)
            if w != b:
                break
        e.reset_with(w, b)
    steps = episodes = 0
    t0 = time.perf_counter()
    p = 0
    while True:
        if plies is not None and p >= plies:
            break
        if seconds is not None and time.perf_counter() - t0 >= seconds:
            break
        for i, e in enumerate(envs):
            dice = [int(nprng.randint(1, 7)), int(nprng.randint(1, 7))]
            _, _, done = e.step(dice, None, rng)
            elapsed[i] += 1
            steps += 1
            if done or elapsed[i] >= max_steps:
                episodes += 1
                elapsed[i] = 0
                while True:
                    w, b = nprng.randint(1, 7), nprng.randint(1, 7)
                    if w != b:
                        break
                e.reset_with(w, b)
        p += 1
    return steps, time.perf_counter() - t0, episodes
