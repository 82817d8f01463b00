"""Host-side logic of the facade that needs no GPU."""
import numpy as np
import pytest
from conftest import golden

import gym_narde
from gym_narde import _compat
from gym_narde.envs.narde import Narde, rotate_board
from gym_narde.vector import decode_compact


def test_rotate_board_matches_reference_definition():
    b = np.arange(-12, 12, dtype=np.int32)
    r = rotate_board(b)
    assert r.dtype == np.int32
    assert np.array_equal(r, np.concatenate((-b[12:], -b[:12])))
    assert np.array_equal(rotate_board(r), b)


def test_start_position_and_perspective():
    g = Narde()
    assert g.board[23] == 15 and g.board[11] == -15 and g.board.dtype == np.int32
    assert np.array_equal(g.get_perspective_board(-1), g.board)  # start is symmetric
    assert g.first_turn_white and g.first_turn_black


def test_head_filter_helpers():
    g = Narde()
    mv = [(23, 17), (23, 17), (5, 0)]
    assert g._validate_head_moves(mv, [6, 6], True) == mv
    assert g._validate_head_moves(mv, [6, 6], False) == [(23, 17), (5, 0)]
    assert g._filter_head_moves(mv, 23, 1) == [(23, 17), (5, 0)]


def test_decode_compact_roundtrip():
    L_hi = (1 << 0) | (1 << 2) | (1 << 23)
    L_lo = (1 << 3)
    c = L_hi | (L_lo << 24) | (6 << 48) | (1 << 52)
    assert decode_compact(np.uint64(c)) == [(0, "off"), (2, "off"), (23, 17), (3, 2)]
    assert decode_compact(np.array([c, 0], np.uint64))[1] == []


def test_timelimit_semantics():
    class Dummy:
        def reset(self, **k):
            return 0, {}

        def step(self, a):
            return 0, 0, False, False, {}

        @property
        def unwrapped(self):
            return self

    env = _compat.TimeLimit(Dummy(), 3)
    env.reset()
    assert [env.step(0)[3] for _ in range(3)] == [False, False, True]


def test_make_and_spaces():
    env = gym_narde.make("gym_narde:narde-v0")
    assert env.unwrapped.observation_space.shape == (24,)
    a = env.unwrapped.action_space.sample()
    assert len(a) == 2 and all(0 <= x < 576 for x in a)
    with pytest.raises(ValueError):
        gym_narde.make("narde-pixel-v0")


def test_invalid_position_rejected_before_any_gpu_call():
    g = Narde()
    g.board[0] = 16
    with pytest.raises(ValueError):
        g.get_valid_moves([1, 2])


def test_golden_fixtures_are_plain_data():
    for name in ("legal.npz", "steps.npz", "episodes.npz", "resets.npz", "block.npz", "apply.npz",
                 "full4.npz", "callers.npz", "trainer.npz"):
        d = golden(name)
        assert all(isinstance(v, np.ndarray) and v.dtype != object for v in d.values())
