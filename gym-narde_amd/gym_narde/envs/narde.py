"""Scalar `Narde` game object -- drop-in for gym_narde.envs.narde.

Same names, argument meaning and return values as the reference
(/root/reference/gym_narde/envs/narde.py); every rule evaluation
(get_valid_moves, the block rule, move execution) runs in the HIP kernels of
libnarde.so through the host entry points (narde_host_*).  The game state
lives in host numpy attributes exactly like the reference's (`board` is a live
int32[24] array callers may mutate), and is shipped to the device on each
call.  Moves are (from, to) tuples with to == 'off' for bearing off.

Positions must be legal Narde positions: each point in [-15, 15] and at most
15 checkers (on board + off) per colour; anything else raises ValueError
(the reference's int32 board would silently accept them).
"""
import numpy as np

from .. import _lib

OFF = _lib.OFF
_HEAD_ROLLS = ((3, 3), (4, 4), (6, 6))


def rotate_board(board):
    """narde.py:16-17 -- the other player's perspective of a board."""
    return np.concatenate((-board[12:], -board[:12])).astype(np.int32)


def _state_arrays(game, player):
    board = np.ascontiguousarray(np.asarray(game.board), dtype=np.int64)
    if board.shape != (24,) or np.abs(board).max(initial=0) > 15:
        raise ValueError("board must be 24 points with counts in [-15, 15]")
    off = np.array([game.borne_off_white, game.borne_off_black], dtype=np.int64)
    if (off < 0).any() or (off > 15).any():
        raise ValueError("borne-off counters must be in [0, 15]")
    b8 = board.astype(np.int8).reshape(1, 24)
    return (b8, off.astype(np.uint8).reshape(1, 2),
            np.array([[bool(game.first_turn_white), bool(game.first_turn_black)]], np.uint8),
            np.array([1 if player == 1 else -1], np.int8))


def _decode_list(moves, count):
    out = []
    for k in range(int(count)):
        f, t = int(moves[k, 0]), int(moves[k, 1])
        out.append((f, "off" if t == OFF else t))
    return out


class Narde:
    """Narde rules (narde.py:20-192) with the evaluation on the GPU."""

    def __init__(self):
        self.board = np.zeros(24, dtype=np.int32)
        self.board[23] = 15
        self.board[11] = -15
        self.borne_off_white = 0
        self.borne_off_black = 0
        self.first_turn_white = True
        self.first_turn_black = True

    # narde.py:31-34
    def get_perspective_board(self, current_player):
        if current_player == 1:
            return self.board.copy()
        return rotate_board(self.board)

    # narde.py:58-92
    def get_valid_moves(self, roll, current_player=1):
        roll = [int(d) for d in roll]
        if len(roll) > 4:
            raise ValueError("at most 4 dice per roll")
        if any(d < 1 or d > 6 for d in roll):
            # the reference would scan with such a die; no legal roll has one
            raise ValueError("dice must be in 1..6")
        player = 1 if current_player == 1 else -1
        board, off, ft, pl = _state_arrays(self, player)
        dice4 = np.zeros((1, 4), np.uint8)
        dice4[0, :len(roll)] = roll
        count = np.zeros(1, np.int16)
        moves = np.zeros((1, _lib.MAX_MOVES, 2), np.int8)
        h = _lib.host_handle()
        h.call("narde_host_legal_moves", 1, _lib.ptr(board), _lib.ptr(off), _lib.ptr(ft),
               _lib.ptr(pl), _lib.ptr(dice4), _lib.ptr(count), _lib.ptr(moves))
        return _decode_list(moves[0], count[0])

    # narde.py:94-106 (kept for API parity; applied inside get_valid_moves)
    def _validate_head_moves(self, moves, roll, first_turn):
        max_head = 2 if first_turn and tuple(sorted(roll)) in _HEAD_ROLLS else 1
        return self._filter_head_moves(moves, 23, max_head)

    # narde.py:127-137
    def _filter_head_moves(self, moves, head_pos, max_head_moves):
        allowed, n = [], 0
        for move in moves:
            if move[0] == head_pos:
                if n < max_head_moves:
                    allowed.append(move)
                    n += 1
            else:
                allowed.append(move)
        return allowed

    # narde.py:36-56 (+ _execute_move :108-125)
    def execute_rotated_move(self, move, current_player):
        player = 1 if current_player == 1 else -1
        f, t = move
        mv = np.array([[int(f), OFF if t == "off" else int(t)]], np.int8)
        board, off, ft, pl = _state_arrays(self, player)
        h = _lib.host_handle()
        h.call("narde_host_apply_moves", 1, _lib.ptr(board), _lib.ptr(off), _lib.ptr(ft),
               _lib.ptr(pl), _lib.ptr(mv))
        self._load(board[0], off[0], ft[0])

    def _execute_move(self, move):
        """narde.py:108-125: absolute coordinates, colour from the source sign."""
        f, _ = move
        player = 1 if self.board[f] > 0 else -1
        if player == -1:
            t = move[1]
            move = ((f - 12) % 24, t if t == "off" else (t - 12) % 24)
        ft = (self.first_turn_white, self.first_turn_black)
        self.execute_rotated_move(move, player)
        self.first_turn_white, self.first_turn_black = ft

    def _load(self, board, off, ft):
        self.board[:] = board.astype(np.int32)
        self.borne_off_white = int(off[0])
        self.borne_off_black = int(off[1])
        self.first_turn_white = bool(ft[0])
        self.first_turn_black = bool(ft[1])

    # narde.py:139-184
    def _violates_block_rule(self, board):
        b = np.clip(np.asarray(board), -127, 127).astype(np.int8).reshape(1, 24)
        out = np.zeros(1, np.uint8)
        _lib.host_handle().call("narde_host_violates_block_rule", 1, _lib.ptr(b), _lib.ptr(out))
        return bool(out[0])

    # narde.py:186-192
    def validate_move(self, move, roll, current_player=1):
        return move in self.get_valid_moves(roll, current_player)

    def get_valid_plays(self, roll, current_player=1):
        """The plays NardeEnv.step (narde_env.py:27-103) carries out for this
        two-dice roll, as a set of move tuples: (m1, m2) for each m1 of
        get_valid_moves(roll) and each m2 of get_valid_moves(rest) after m1,
        where rest is the roll less m1's distance (else its first die, the
        step's pop(0)); (m1,) when no second move follows m1, and the only
        play when list #1 has one move (the step then plays it alone:
        narde_env.py:41-43); set() when no move is legal.  (The step also
        takes partial actions -- an illegal move-2 code plays m1 alone, an
        illegal move-1 code nothing; those are not listed.)  The README's
        get_valid_actions (README.md:156-165) names such a set; the reference
        code never builds one.  Three batched GPU calls: list #1, every m1
        applied to a copy of the position, every list #2."""
        roll = [int(d) for d in roll]
        if len(roll) != 2 or any(d < 1 or d > 6 for d in roll):
            raise ValueError("a roll of two dice in 1..6")
        player = 1 if current_player == 1 else -1
        listed = self.get_valid_moves(roll, player)
        if len(listed) <= 1:
            return {tuple(listed)} if listed else set()
        first = list(dict.fromkeys(listed))  # distinct, list order
        n = len(first)
        board, off, ft, pl = _state_arrays(self, player)
        board, off, ft, pl = (np.repeat(a, n, axis=0) for a in (board, off, ft, pl))
        mv = np.array([[f, OFF if t == "off" else t] for f, t in first], np.int8)
        h = _lib.host_handle()
        h.call("narde_host_apply_moves", n, _lib.ptr(board), _lib.ptr(off), _lib.ptr(ft), _lib.ptr(pl), _lib.ptr(mv))
        dice4 = np.zeros((n, 4), np.uint8)
        for k, (f, t) in enumerate(first):
            dist = f + 1 if t == "off" else abs(f - t)  # narde_env.py:63-70
            rest = list(roll)
            if dist in rest:
                rest.remove(dist)
            else:
                rest.pop(0)
            dice4[k, 0] = rest[0]
        count = np.zeros(n, np.int16)
        moves = np.zeros((n, _lib.MAX_MOVES, 2), np.int8)
        h.call("narde_host_legal_moves", n, _lib.ptr(board), _lib.ptr(off), _lib.ptr(ft), _lib.ptr(pl),
               _lib.ptr(dice4), _lib.ptr(count), _lib.ptr(moves))
        plays = set()
        for k, m1 in enumerate(first):
            second = _decode_list(moves[k], count[k])
            if second:
                plays.update((m1, m2) for m2 in second)
            else:
                plays.add((m1,))
        return plays
