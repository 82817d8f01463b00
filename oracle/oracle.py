"""ctypes/numpy front-end for the C oracle (oracle/narde_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package (gym-narde_amd/).

All arrays are numpy, C-contiguous; states are the build's absolute int8
layout (board int8[24], off uint8[2] = (white, black), first_turn uint8[2] =
(white, black), player int8 = +1/-1).  Moves use to = 24 for 'off'.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# NARDE_ORACLE_LIB: an alternative build of the same source (tools/sanitize.sh)
LIB_PATH = os.environ.get("NARDE_ORACLE_LIB", os.path.join(HERE, "build", "libnarde_oracle.so"))
MAXM = 64
OFF = 24

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def legal_moves(board, ft, player, roll, nroll):
    """Narde.get_valid_moves over a batch -> (moves int8[n,64,2], count int16[n])."""
    board = _c(board, np.int8)
    n = board.shape[0]
    ft = _c(ft, np.uint8)
    player = _c(player, np.int8)
    roll = _c(roll, np.uint8)
    nroll = _c(nroll, np.uint8)
    moves = np.empty((n, MAXM, 2), np.int8)
    count = np.empty(n, np.int16)
    off = np.zeros((n, 2), np.uint8)
    lib().or_legal_batch(ctypes.c_int64(n), _p(board), _p(off), _p(ft), _p(player), _p(roll),
                         _p(nroll), _p(moves), _p(count))
    return moves, count


def violates_block_rule(board):
    board = _c(board, np.int8)
    out = np.empty(board.shape[0], np.uint8)
    lib().or_block_batch(ctypes.c_int64(board.shape[0]), _p(board), _p(out))
    return out


def apply_move(board, off, ft, player, move):
    board = _c(board, np.int8).copy()
    off = _c(off, np.uint8).copy()
    ft = _c(ft, np.uint8).copy()
    player = _c(player, np.int8)
    move = _c(move, np.int8)
    lib().or_apply_batch(ctypes.c_int64(board.shape[0]), _p(board), _p(off), _p(ft), _p(player), _p(move))
    return board, off, ft


def step(board, off, ft, player, dice, action, with_lists=True):
    """NardeEnv.step with injected dice; returns a dict of post-state + outputs."""
    board = _c(board, np.int8).copy()
    off = _c(off, np.uint8).copy()
    ft = _c(ft, np.uint8).copy()
    player = _c(player, np.int8).copy()
    dice = _c(dice, np.uint8)
    action = _c(action, np.int16)
    n = board.shape[0]
    obs = np.empty((n, 24), np.int8)
    reward = np.empty(n, np.int8)
    term = np.empty(n, np.uint8)
    if with_lists:
        list1 = np.empty((n, MAXM, 2), np.int8)
        list2 = np.empty((n, MAXM, 2), np.int8)
        count1 = np.empty(n, np.int16)
        count2 = np.empty(n, np.int16)
        roll2 = np.empty(n, np.uint8)
    else:
        list1 = list2 = count1 = count2 = roll2 = None
    legal1 = np.empty(n, np.uint64)
    lib().or_step_batch(ctypes.c_int64(n), _p(board), _p(off), _p(ft), _p(player), _p(dice),
                        _p(action), _p(obs), _p(reward), _p(term), _p(list1), _p(count1),
                        _p(list2), _p(count2), _p(roll2), _p(legal1))
    return dict(board=board, off=off, first_turn=ft, player=player, obs=obs, reward=reward,
                terminated=term, list1=list1, count1=count1, list2=list2, count2=count2,
                roll2=roll2, legal1=legal1)


def full4_turn(board, off, ft, player, dice, words):
    """FULL4 turns with given dice and pick words.
    Returns post-turn state (no flip) + max_dice, cmask [n,4,2] (C_k source
    masks of the higher / lower die), played [n,4,2] (from, die), reward, done."""
    board = _c(board, np.int8).copy()
    off = _c(off, np.uint8).copy()
    ft = _c(ft, np.uint8).copy()
    player = _c(player, np.int8)
    n = board.shape[0]
    M = np.empty(n, np.int8)
    cm = np.empty((n, 4, 2), np.uint32)
    played = np.empty((n, 4, 2), np.int8)
    reward = np.empty(n, np.int8)
    done = np.empty(n, np.uint8)
    lib().or_full4_batch(ctypes.c_int64(n), _p(board), _p(off), _p(ft), _p(player),
                         _p(_c(dice, np.uint8)), _p(_c(words, np.uint32)), _p(M), _p(cm),
                         _p(played), _p(reward), _p(done))
    return dict(board=board, off=off, first_turn=ft, max_dice=M, cmask=cm, played=played,
                reward=reward, done=done)


def expand_compact(words):
    """Compact two-dice legal words (u64[N]) -> (moves int8[N,64,2] padded with
    -1, count int16[N]) in the reference's list order: the higher die's
    entries, then the lower die's, ascending source, to = from - die or 24
    ('off').  Vectorised (numpy); the inverse of or_compact2."""
    w = np.ascontiguousarray(words, dtype=np.uint64).reshape(-1)
    n = w.shape[0]
    pos = np.arange(24, dtype=np.uint64)
    Lh = ((w[:, None] >> pos) & np.uint64(1)).astype(bool)
    Ll = ((w[:, None] >> (pos + np.uint64(24))) & np.uint64(1)).astype(bool)
    dh = ((w >> np.uint64(48)) & np.uint64(0xF)).astype(np.int16)
    dl = ((w >> np.uint64(52)) & np.uint64(0xF)).astype(np.int16)
    bits = np.concatenate([Lh, Ll], axis=1)                      # [N, 48] group-major
    src = np.tile(np.arange(24, dtype=np.int16), 2)[None, :]      # [1, 48]
    die = np.concatenate([np.repeat(dh[:, None], 24, 1), np.repeat(dl[:, None], 24, 1)], 1)
    dst = src - die
    dst = np.where(dst < 0, OFF, dst)
    order = np.argsort(~bits, axis=1, kind="stable")             # set bits first, in order
    cnt = bits.sum(1).astype(np.int16)
    rows = np.arange(n)[:, None]
    f = np.broadcast_to(src, (n, 48))[rows, order]
    t = dst[rows, order]
    keep = np.arange(48)[None, :] < cnt[:, None]
    moves = np.full((n, MAXM, 2), -1, np.int8)
    moves[:, :48, 0] = np.where(keep, f, -1)
    moves[:, :48, 1] = np.where(keep, t, -1)
    return moves, cnt


def tesauro198(board, off, player):
    board = _c(board, np.int8)
    n = board.shape[0]
    out = np.empty((n, 198), np.float32)
    lib().or_tesauro198_batch(ctypes.c_int64(n), _p(board), _p(_c(off, np.uint8)),
                              _p(_c(player, np.int8)), _p(out))
    return out


def philox(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().or_philox4x32_10(c, k, o)
    return tuple(o)


class SelfPlay:
    """Batched self-play state for the restated random-legal driver."""

    def __init__(self, n, seed=0, env0=0, dice_mode=0, max_steps=1000):
        self.n, self.seed, self.env0 = n, seed, env0
        self.dice_mode, self.max_steps = dice_mode, max_steps
        self.board = np.zeros((n, 24), np.int8)
        self.off = np.zeros((n, 2), np.uint8)
        self.ft = np.zeros((n, 2), np.uint8)
        self.player = np.zeros(n, np.int8)
        self.elapsed = np.zeros(n, np.uint16)
        self.stats = np.zeros((n, 3), np.int32)
        self.t = 0

    def reset(self, epoch=0):
        lib().or_reset_batch(ctypes.c_int64(self.n), ctypes.c_int64(self.env0),
                             ctypes.c_uint64(self.seed), ctypes.c_uint32(epoch),
                             _p(self.board), _p(self.off), _p(self.ft), _p(self.player),
                             _p(self.elapsed))
        self.stats[:] = 0

    def load(self, board, off, ft, player, elapsed, stats, t):
        """Take over a device handle's state at lockstep ply t (get_state(),
        stats() and ply of VecNardeEnv): run() then replays the plies the
        handle plays from there (oracle/replay.py)."""
        n = self.n
        self.board = np.array(board, dtype=np.int8).reshape(n, 24)
        self.off = np.array(off, dtype=np.uint8).reshape(n, 2)
        self.ft = np.array(ft, dtype=np.uint8).reshape(n, 2)
        self.player = np.array(player, dtype=np.int8).reshape(n)
        self.elapsed = np.array(elapsed).astype(np.uint16).reshape(n)
        self.stats = np.array(stats, dtype=np.int32).reshape(n, 3)
        self.t = int(t)

    def run(self, plies, record=True):
        n = self.n
        if record:
            obs = np.empty((plies, n, 24), np.int8)
            reward = np.empty((plies, n), np.int8)
            term = np.empty((plies, n), np.uint8)
            trunc = np.empty((plies, n), np.uint8)
            dice = np.empty((plies, n, 2), np.uint8)
            action = np.empty((plies, n, 2), np.int16)
            count1 = np.empty((plies, n), np.int16)
            legal = np.empty((plies, n), np.uint64)
        else:
            obs = reward = term = trunc = dice = action = count1 = legal = None
        lib().or_selfplay(ctypes.c_int64(n), ctypes.c_int64(self.env0), ctypes.c_uint64(self.seed),
                          ctypes.c_uint32(self.t), ctypes.c_int(plies), ctypes.c_int(self.dice_mode),
                          ctypes.c_int(self.max_steps), _p(self.board), _p(self.off), _p(self.ft),
                          _p(self.player), _p(self.elapsed), _p(self.stats), _p(obs), _p(reward),
                          _p(term), _p(trunc), _p(dice), _p(action), _p(count1), _p(legal))
        self.t += plies
        if record:
            # legal: list #1 of each ply in the build's compact form, built by
            # the oracle from its own list (or_compact2)
            return dict(obs=obs, reward=reward, terminated=term, truncated=trunc, dice=dice,
                        action=action, count1=count1, legal=legal)
        return None


    def run_full(self, plies, record=True):
        """FULL4 self-play, same state as run()."""
        n = self.n
        if record:
            obs = np.empty((plies, n, 24), np.int8)
            reward = np.empty((plies, n), np.int8)
            term = np.empty((plies, n), np.uint8)
            trunc = np.empty((plies, n), np.uint8)
            dice = np.empty((plies, n, 2), np.uint8)
            legal = np.empty((plies, n), np.uint64)
            played = np.empty((plies, n), np.uint64)
        else:
            obs = reward = term = trunc = dice = legal = played = None
        lib().or_selfplay_full(ctypes.c_int64(n), ctypes.c_int64(self.env0),
                               ctypes.c_uint64(self.seed), ctypes.c_uint32(self.t),
                               ctypes.c_int(plies), ctypes.c_int(self.dice_mode),
                               ctypes.c_int(self.max_steps), _p(self.board), _p(self.off),
                               _p(self.ft), _p(self.player), _p(self.elapsed), _p(self.stats),
                               _p(obs), _p(reward), _p(term), _p(trunc), _p(dice), _p(legal),
                               _p(played))
        self.t += plies
        if record:
            return dict(obs=obs, reward=reward, terminated=term, truncated=trunc, dice=dice,
                        legal=legal, played=played)
        return None
