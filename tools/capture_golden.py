#!/usr/bin/env python3
"""Capture golden vectors from the reference gym-narde (THIS container only).

Test infrastructure, not product code.  The reference never leaves this
container: this script imports it from /root/reference, drives it with
injected dice, and writes plain-data fixtures (numpy .npz, allow_pickle=False)
under tests/golden/.  The fixtures are what travels; the tests read only them.

gymnasium is not installed here, so the reference's `import gymnasium` is
satisfied by a throw-away stub written to a temp dir (Env/spaces/register
only -- the reference uses nothing else from it).  The stub is never committed
or imported by product code.

Reference entry points exercised (paths relative to /root/reference):
  gym_narde/envs/narde.py:58-92    Narde.get_valid_moves  (legal.npz)
  gym_narde/envs/narde.py:139-184  Narde._violates_block_rule (block.npz)
  gym_narde/envs/narde.py:36-56    Narde.execute_rotated_move (apply.npz)
  gym_narde/envs/narde_env.py:27-103  NardeEnv.step (steps.npz)
  gym_narde/envs/narde_env.py:105-120 NardeEnv.reset (resets.npz)
  full seeded episodes through reset/step (episodes.npz)

Usage:  python tools/capture_golden.py [--out tests/golden] [--scale 1.0]
"""
import argparse
import copy
import os
import random
import sys
import tempfile

import numpy as np

REF = "/root/reference"
OFF = 24          # fixture encoding of the reference's 'off' destination
MAXM = 64         # list capacity in fixtures (4-die rolls give <= 60)

_STUB_INIT = """
class Env:
    metadata = {}
    def __init__(self, *a, **k):
        pass
from . import spaces
"""
_STUB_SPACES = """
class Box:
    def __init__(self, low=None, high=None, shape=None, dtype=None):
        self.low, self.high, self.shape, self.dtype = low, high, shape, dtype
class Discrete:
    def __init__(self, n):
        self.n = n
class Tuple:
    def __init__(self, spaces):
        self.spaces = tuple(spaces)
"""
_STUB_REG = """
def register(**kwargs):
    pass
"""


def load_reference():
    tmp = tempfile.mkdtemp(prefix="gymstub_")
    pkg = os.path.join(tmp, "gymnasium")
    os.makedirs(os.path.join(pkg, "envs"))
    with open(os.path.join(pkg, "__init__.py"), "w") as f:
        f.write(_STUB_INIT)
    with open(os.path.join(pkg, "spaces.py"), "w") as f:
        f.write(_STUB_SPACES)
    with open(os.path.join(pkg, "envs", "__init__.py"), "w") as f:
        f.write("")
    with open(os.path.join(pkg, "envs", "registration.py"), "w") as f:
        f.write(_STUB_REG)
    sys.path.insert(0, tmp)
    sys.path.insert(1, REF)
    sys.dont_write_bytecode = True
    from gym_narde.envs import narde as narde_mod
    from gym_narde.envs.narde_env import NardeEnv
    return narde_mod, NardeEnv


class DiceInjector:
    """Replace np.random.randint so the reference consumes chosen values."""

    def __init__(self):
        self.queue = []
        self._orig = np.random.randint

    def __enter__(self):
        def fake(lo, hi=None, *a, **k):
            assert self.queue, "reference drew more dice than injected"
            return self.queue.pop(0)
        np.random.randint = fake
        return self

    def __exit__(self, *exc):
        np.random.randint = self._orig


def enc_moves(moves):
    out = np.full((MAXM, 2), -1, dtype=np.int8)
    for i, (f, t) in enumerate(moves):
        out[i, 0] = f
        out[i, 1] = OFF if t == "off" else t
    return out, len(moves)


def move_code(m):
    f, t = m
    return f * 24 + (0 if t == "off" else t)


def snapshot(game):
    return (game.board.astype(np.int8).copy(), int(game.borne_off_white),
            int(game.borne_off_black), bool(game.first_turn_white),
            bool(game.first_turn_black))


def set_game(game, board, offw, offb, ftw, ftb):
    game.board = np.asarray(board, dtype=np.int32).copy()
    game.borne_off_white = int(offw)
    game.borne_off_black = int(offb)
    game.first_turn_white = bool(ftw)
    game.first_turn_black = bool(ftb)


def remaining_after(dice, m):
    """narde_env.py:63-83 die bookkeeping (used only to drive the policy)."""
    dist = m[0] + 1 if m[1] == "off" else abs(m[0] - m[1])
    tmp = list(dice)
    if dist in tmp:
        tmp.remove(dist)
    elif tmp:
        tmp.pop(0)
    return tmp


def random_legal_action(game, dice, player, rng):
    """Random legal policy: move1 uniform over the list
    (duplicates weighted), move2 uniform over the post-move1 list."""
    valid = game.get_valid_moves(dice, player)
    if not valid:
        return (0, 0)
    m1 = valid[rng.randrange(len(valid))]
    g2 = copy.deepcopy(game)
    g2.execute_rotated_move(m1, player)
    rem = remaining_after(dice, m1)
    v2 = g2.get_valid_moves(rem, player) if rem else []
    m2 = v2[rng.randrange(len(v2))] if v2 else None
    return (move_code(m1), move_code(m2) if m2 is not None else 0)


def selfplay_states(NardeEnv, n_states, seed):
    """Reachable pre-step states from seeded reference self-play."""
    rng = random.Random(seed)
    np.random.seed(seed)
    env = NardeEnv()
    env.reset(seed=seed)
    states = []
    steps = 0
    while len(states) < n_states:
        g = env.game
        states.append(snapshot(g) + (env.current_player,))
        st = np.random.get_state()
        dice = [int(np.random.randint(1, 7)), int(np.random.randint(1, 7))]
        np.random.set_state(st)
        a = random_legal_action(g, dice, env.current_player, rng)
        _, _, done, _, _ = env.step(a)
        steps += 1
        if done or steps >= 1000:
            env.reset()
            steps = 0
    return states


def synthetic_state(rng):
    """Random non-reachable-but-valid-shaped board: 15 per colour split
    between board points and off, no mixed points, optional 6-runs."""
    board = np.zeros(24, dtype=np.int32)
    free = list(range(24))
    rng.shuffle(free)
    offw = rng.choice([0, 0, 0, rng.randrange(0, 15)])
    offb = rng.choice([0, 0, 0, rng.randrange(0, 15)])
    mode = rng.randrange(4)
    # white
    if mode == 0:  # contiguous run(s) -> block-rule coverage
        start = rng.randrange(0, 19)
        ln = rng.randrange(4, 8)
        pts = [p for p in range(start, min(24, start + ln))]
    elif mode == 1:  # all in home -> bear-off coverage
        pts = rng.sample(range(0, 6), rng.randrange(1, 7))
    else:
        pts = free[: rng.randrange(1, 10)]
    nw = 15 - offw
    for i in range(nw):
        board[pts[i % len(pts)]] += 1
    # black (avoid white points)
    cand = [p for p in range(24) if board[p] == 0]
    if mode == 1 and rng.random() < 0.5:
        # black in its own home (abs 12..17) so its bear-off is live too
        cand2 = [p for p in range(12, 18) if board[p] == 0]
        if cand2:
            cand = cand2
    if rng.random() < 0.3:
        s = rng.choice(cand)
        bpts = [p for p in range(s, min(24, s + rng.randrange(3, 8))) if board[p] == 0]
    else:
        bpts = rng.sample(cand, min(len(cand), rng.randrange(1, 9)))
    if not bpts:
        bpts = [cand[0]]
    nb = 15 - offb
    for i in range(nb):
        board[bpts[i % len(bpts)]] -= 1
    ftw = rng.random() < 0.3
    ftb = rng.random() < 0.3
    player = rng.choice([1, -1])
    return (board.astype(np.int8), offw, offb, ftw, ftb, player)


def endgame_state(rng):
    """Mover close to bearing off its last checkers (termination/mars
    coverage, narde_env.py:134-141)."""
    board = np.zeros(24, dtype=np.int32)
    player = rng.choice([1, -1])
    left = rng.randrange(1, 4)
    # mover perspective home is 0..5; absolute = p (white) or p+12 (black)
    for _ in range(left):
        p = rng.randrange(0, 6)
        board[p if player == 1 else p + 12] += 1
    opp_off = rng.choice([0, 0, rng.randrange(0, 15)])
    cand = [p for p in range(24) if board[p] == 0]
    pts = rng.sample(cand, rng.randrange(1, 6))
    for i in range(15 - opp_off):
        board[pts[i % len(pts)]] -= 1
    if player == -1:
        board = -board
    offw = 15 - int(board[board > 0].sum())
    offb = 15 - int(-board[board < 0].sum())
    return (board.astype(np.int8), offw, offb, False, rng.random() < 0.2, player)


def random_roll(rng):
    r = rng.random()
    if r < 0.7:
        return [rng.randint(1, 6), rng.randint(1, 6)]
    if r < 0.8:
        return [rng.randint(1, 6)]
    if r < 0.9:
        d = rng.randint(1, 6)
        return [d] * 4
    d = rng.randint(1, 6)
    return [d] * 3


KAT_LEGAL = [
    # (board dict, black dict, ftw, ftb, roll, player) -- SURVEY Appendix B
    ("start", None, True, True, [5, 3], 1),
    ("start", None, True, True, [3, 5], 1),
    ("start", None, True, True, [6, 6], 1),
    ("start", None, True, True, [4, 4], 1),
    ("start", None, True, True, [3, 3], 1),
    ("start", None, True, True, [5, 5], 1),
    ("start", None, True, True, [1, 2], 1),
    ("start", None, True, True, [5, 5, 5, 5], 1),
    ("start", None, True, True, [5, 3], -1),
    ("start", None, True, True, [6, 6], -1),
    ("start", None, True, True, [4, 4], -1),
    ({0: 1, 2: 12, 3: 2}, {11: -15}, False, True, [3, 1], 1),
    ({0: 1, 2: 12, 3: 2}, {11: -15}, False, True, [6, 5], 1),
    ({0: 1, 1: 1, 2: 1, 3: 1, 4: 1, 6: 2, 23: 8}, {12: -15}, False, False, [1, 3], 1),
]


def kat_state(spec):
    bd, bl, ftw, ftb, roll, player = spec
    board = np.zeros(24, dtype=np.int32)
    if bd == "start":
        board[23] = 15
        board[11] = -15
    else:
        for k, v in bd.items():
            board[k] = v
        for k, v in bl.items():
            board[k] = v
    offw = 15 - int(board[board > 0].sum())
    offb = 15 - int(-board[board < 0].sum())
    return (board.astype(np.int8), offw, offb, ftw, ftb, player), roll


def capture_legal(narde_mod, NardeEnv, scale, rng):
    n_reach = int(30000 * scale)
    n_synth = int(30000 * scale)
    states = selfplay_states(NardeEnv, n_reach // 2, seed=11)
    cases = []
    for s in states:
        cases.append((s, [rng.randint(1, 6), rng.randint(1, 6)]))
        cases.append((s, random_roll(rng)))
    for _ in range(n_synth):
        cases.append((synthetic_state(rng), random_roll(rng)))
    kat = [kat_state(k) for k in KAT_LEGAL]
    cases = kat + cases
    N = len(cases)
    out = dict(
        board=np.zeros((N, 24), np.int8), off=np.zeros((N, 2), np.uint8),
        first_turn=np.zeros((N, 2), np.uint8), player=np.zeros(N, np.int8),
        roll=np.zeros((N, 4), np.uint8), nroll=np.zeros(N, np.uint8),
        moves=np.zeros((N, MAXM, 2), np.int8), count=np.zeros(N, np.int16),
        n_kat=np.int32(len(kat)))
    g = narde_mod.Narde()
    for i, ((board, offw, offb, ftw, ftb, player), roll) in enumerate(cases):
        set_game(g, board, offw, offb, ftw, ftb)
        mv = g.get_valid_moves(list(roll), player)
        out["board"][i] = board
        out["off"][i] = (offw, offb)
        out["first_turn"][i] = (ftw, ftb)
        out["player"][i] = player
        out["roll"][i, : len(roll)] = roll
        out["nroll"][i] = len(roll)
        out["moves"][i], out["count"][i] = enc_moves(mv)
    return out


def capture_block(narde_mod, scale, rng):
    """_violates_block_rule on raw perspective boards (the trainer calls it
    directly: train_deepq_pytorch.py:1075)."""
    N = int(20000 * scale)
    boards = np.zeros((N, 24), np.int8)
    res = np.zeros(N, np.uint8)
    g = narde_mod.Narde()
    for i in range(N):
        b = np.zeros(24, np.int32)
        if rng.random() < 0.6:
            s = rng.randrange(0, 24)
            for p in range(s, min(24, s + rng.randrange(4, 10))):
                b[p] = rng.randint(1, 3)
        for _ in range(rng.randrange(0, 8)):
            b[rng.randrange(24)] = rng.choice([-2, -1, 0, 1, 2])
        boards[i] = b
        res[i] = bool(g._violates_block_rule(b))
    return dict(board=boards, violates=res)


def capture_apply(narde_mod, scale, rng):
    """execute_rotated_move on reachable-ish states: every listed move."""
    N = int(8000 * scale)
    rows = []
    g = narde_mod.Narde()
    while len(rows) < N:
        st = synthetic_state(rng)
        board, offw, offb, ftw, ftb, player = st
        set_game(g, board, offw, offb, ftw, ftb)
        mv = g.get_valid_moves([rng.randint(1, 6), rng.randint(1, 6)], player)
        if not mv:
            continue
        m = mv[rng.randrange(len(mv))]
        g.execute_rotated_move(m, player)
        rows.append((st, m, snapshot(g)))
    out = dict(board=np.zeros((N, 24), np.int8), off=np.zeros((N, 2), np.uint8),
               first_turn=np.zeros((N, 2), np.uint8), player=np.zeros(N, np.int8),
               move=np.zeros((N, 2), np.int8),
               post_board=np.zeros((N, 24), np.int8), post_off=np.zeros((N, 2), np.uint8),
               post_first_turn=np.zeros((N, 2), np.uint8))
    for i, (st, m, post) in enumerate(rows):
        board, offw, offb, ftw, ftb, player = st
        out["board"][i] = board
        out["off"][i] = (offw, offb)
        out["first_turn"][i] = (ftw, ftb)
        out["player"][i] = player
        out["move"][i] = (m[0], OFF if m[1] == "off" else m[1])
        out["post_board"][i] = post[0]
        out["post_off"][i] = (post[1], post[2])
        out["post_first_turn"][i] = (post[3], post[4])
    return out


def capture_steps(narde_mod, NardeEnv, scale, rng):
    n_reach = int(25000 * scale)
    n_synth = int(15000 * scale)
    states = selfplay_states(NardeEnv, n_reach, seed=23)
    states += [synthetic_state(rng) for _ in range(n_synth)]
    states += [endgame_state(rng) for _ in range(int(4000 * scale))]
    # hand-built quirk states
    quirk = []
    b = np.zeros(24, np.int8); b[0] = 1; b[1] = 3; b[3] = 3; b[11] = -15
    quirk += [((b, 8, 0, False, True, 1), [2, 6], (72, 72)),
              ((b, 8, 0, False, True, 1), [6, 2], (72, 72))]
    b = np.zeros(24, np.int8); b[23] = 14; b[17] = 1; b[11] = -15
    quirk += [((b, 0, 0, False, False, 1), [6, 5], (23 * 24 + 17, 23 * 24 + 18))]
    b = np.zeros(24, np.int8); b[0] = 2; b[4] = 3; b[11] = -15
    quirk += [((b, 10, 0, False, True, 1), [5, 1], (4 * 24, 0))]
    env = NardeEnv()
    N = len(states) + len(quirk)
    out = dict(
        board=np.zeros((N, 24), np.int8), off=np.zeros((N, 2), np.uint8),
        first_turn=np.zeros((N, 2), np.uint8), player=np.zeros(N, np.int8),
        dice=np.zeros((N, 2), np.uint8), action=np.zeros((N, 2), np.int16),
        post_board=np.zeros((N, 24), np.int8), post_off=np.zeros((N, 2), np.uint8),
        post_first_turn=np.zeros((N, 2), np.uint8), post_player=np.zeros(N, np.int8),
        obs=np.zeros((N, 24), np.int8), reward=np.zeros(N, np.int8),
        terminated=np.zeros(N, np.uint8), truncated=np.zeros(N, np.uint8),
        ncalls=np.zeros(N, np.uint8),
        list1=np.full((N, MAXM, 2), -1, np.int8), count1=np.zeros(N, np.int16),
        list2=np.full((N, MAXM, 2), -1, np.int8), count2=np.full(N, -1, np.int16),
        roll2=np.zeros(N, np.uint8))
    jobs = [(s, None, None) for s in states] + quirk
    for i, (st, dice, action) in enumerate(jobs):
        board, offw, offb, ftw, ftb, player = st
        env.game = narde_mod.Narde()
        set_game(env.game, board, offw, offb, ftw, ftb)
        env.current_player = player
        if dice is None:
            dice = [rng.randint(1, 6), rng.randint(1, 6)]
        if action is None:
            r = rng.random()
            gcopy = copy.deepcopy(env.game)
            if r < 0.5:
                action = random_legal_action(gcopy, dice, player, rng)
            elif r < 0.7:
                v = gcopy.get_valid_moves(dice, player)
                a1 = move_code(v[rng.randrange(len(v))]) if v else rng.randrange(576)
                action = (a1, rng.randrange(576))
            elif r < 0.85:
                action = (rng.randrange(576), rng.randrange(576))
            else:
                action = (rng.randrange(0, 6) * 24, rng.choice([0, rng.randrange(0, 6) * 24]))
        calls = []
        orig = env.game.get_valid_moves

        def spy(roll, current_player=1, _orig=orig):
            res = _orig(roll, current_player)
            calls.append((list(roll), list(res)))
            return res
        env.game.get_valid_moves = spy
        with DiceInjector() as inj:
            inj.queue = list(dice)
            obs, reward, term, trunc, _ = env.step(tuple(int(x) for x in action))
            assert not inj.queue
        post = snapshot(env.game)
        out["board"][i] = board
        out["off"][i] = (offw, offb)
        out["first_turn"][i] = (ftw, ftb)
        out["player"][i] = player
        out["dice"][i] = dice
        out["action"][i] = action
        out["post_board"][i] = post[0]
        out["post_off"][i] = (post[1], post[2])
        out["post_first_turn"][i] = (post[3], post[4])
        out["post_player"][i] = env.current_player
        out["obs"][i] = np.asarray(obs, np.int32).astype(np.int8)
        out["reward"][i] = reward
        out["terminated"][i] = bool(term)
        out["truncated"][i] = bool(trunc)
        out["ncalls"][i] = len(calls)
        out["list1"][i], out["count1"][i] = enc_moves(calls[0][1])
        if len(calls) > 1:
            assert len(calls[1][0]) == 1
            out["list2"][i], out["count2"][i] = enc_moves(calls[1][1])
            out["roll2"][i] = calls[1][0][0]
    return out


def capture_episodes(NardeEnv, n_episodes):
    """Whole seeded episodes through the reference's own numpy RNG:
    reset(seed=s) then a seeded random legal policy that peeks the dice."""
    seeds, lengths = [], []
    dice_l, act_l, obs_l, rew_l, term_l, player_l = [], [], [], [], [], []
    reset_obs, reset_player = [], []
    for s in range(n_episodes):
        rng = random.Random(1000 + s)
        env = NardeEnv()
        obs, _ = env.reset(seed=s)
        reset_obs.append(np.asarray(obs, np.int8))
        reset_player.append(env.current_player)
        n = 0
        while True:
            st = np.random.get_state()
            dice = [int(np.random.randint(1, 7)), int(np.random.randint(1, 7))]
            np.random.set_state(st)
            a = random_legal_action(copy.deepcopy(env.game), dice, env.current_player, rng)
            obs, r, term, trunc, _ = env.step(a)
            dice_l.append(dice)
            act_l.append(a)
            obs_l.append(np.asarray(obs, np.int8))
            rew_l.append(r)
            term_l.append(bool(term))
            player_l.append(env.current_player)
            n += 1
            if term or n >= 1000:
                break
        seeds.append(s)
        lengths.append(n)
    return dict(seed=np.array(seeds, np.int32), length=np.array(lengths, np.int32),
                dice=np.array(dice_l, np.uint8), action=np.array(act_l, np.int16),
                obs=np.array(obs_l, np.int8), reward=np.array(rew_l, np.int8),
                terminated=np.array(term_l, np.uint8), player=np.array(player_l, np.int8),
                reset_obs=np.array(reset_obs, np.int8),
                reset_player=np.array(reset_player, np.int8))


def capture_resets(NardeEnv, n):
    """reset(seed) draw pattern: first player + the next legacy-RNG draw,
    which pins how many values reset consumed (narde_env.py:111-115)."""
    player, nxt = [], []
    for s in range(n):
        env = NardeEnv()
        env.reset(seed=s)
        player.append(env.current_player)
        nxt.append(int(np.random.randint(0, 2 ** 31 - 1)))
    return dict(seed=np.arange(n, dtype=np.int32), player=np.array(player, np.int8),
                next_draw=np.array(nxt, np.int64))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "tests", "golden"))
    ap.add_argument("--scale", type=float, default=1.0)
    args = ap.parse_args()
    narde_mod, NardeEnv = load_reference()
    rng = random.Random(20250523)
    os.makedirs(args.out, exist_ok=True)

    def save(name, d):
        p = os.path.join(args.out, name)
        np.savez_compressed(p, **d)
        print(f"wrote {p} ({os.path.getsize(p) / 1e6:.2f} MB)")

    save("legal.npz", capture_legal(narde_mod, NardeEnv, args.scale, rng))
    save("block.npz", capture_block(narde_mod, args.scale, rng))
    save("apply.npz", capture_apply(narde_mod, args.scale, rng))
    save("steps.npz", capture_steps(narde_mod, NardeEnv, args.scale, rng))
    save("episodes.npz", capture_episodes(NardeEnv, int(40 * args.scale)))
    save("resets.npz", capture_resets(NardeEnv, 256))


if __name__ == "__main__":
    main()
