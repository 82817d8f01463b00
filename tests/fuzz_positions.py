"""Random positions for differential tests (test_gpu_fuzz.py,
test_full4_cpu.py): run-heavy boards where the block rule decides and
bear-off endgames, placed for a random mover.  Test helper, not a test."""
import numpy as np
from test_oracle_golden import _prime_boards


def endgame_boards(n, seed):
    """Mover (positive, perspective) mostly home with some checkers off,
    a few stragglers outside; opponent on 1-3 points the mover leaves free."""
    rng = np.random.default_rng(seed)
    boards = np.zeros((n, 24), np.int8)
    off = np.zeros((n, 2), np.uint8)
    for i in range(n):
        k = int(rng.integers(0, 14))
        for _ in range(15 - k):
            p = int(rng.integers(0, 6)) if rng.random() < 0.85 else int(rng.integers(6, 14))
            boards[i, p] += 1
        free = np.nonzero(boards[i] == 0)[0]
        pts = rng.choice(free, size=min(int(rng.integers(1, 4)), len(free)), replace=False)
        opp = 15
        for j, p in enumerate(pts):
            c = opp if j == len(pts) - 1 else int(rng.integers(1, opp - (len(pts) - 1 - j) + 1))
            boards[i, p] = -c
            opp -= c
        off[i, 0] = k
    return boards, off


def random_positions(n, seed):
    """Half run-heavy, half endgame perspective positions, each placed on
    the absolute board for a random mover: white as is, black rotated
    (get_perspective_board(-1) = rotate_board, narde.py:16-17,31-34).
    Returns (board, off, first_turn, player, rng)."""
    rng = np.random.default_rng(seed)
    h = n // 2
    pb = _prime_boards(h, seed + 1)
    eb, eoff = endgame_boards(n - h, seed + 2)
    persp = np.concatenate([pb, eb])
    off = np.concatenate([np.zeros((h, 2), np.uint8), eoff])
    player = np.where(rng.random(n) < 0.5, 1, -1).astype(np.int8)
    board = persp.copy()
    blk = player == -1
    board[blk] = -np.roll(persp[blk], 12, axis=1)
    off[blk] = off[blk][:, ::-1]
    ft = rng.integers(0, 2, (n, 2)).astype(np.uint8)
    return board, np.ascontiguousarray(off), ft, player, rng
