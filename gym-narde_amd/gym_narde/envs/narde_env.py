"""Scalar `NardeEnv` -- drop-in for gym_narde.envs.narde_env.NardeEnv.

Mirrors /root/reference/gym_narde/envs/narde_env.py: the same reset/step
signature and return tuples, `current_player`, `game`, spaces and render.
Dice come from numpy's global legacy RNG exactly as in the reference
(reset: pairs until unequal, narde_env.py:111-115; step: two draws,
narde_env.py:29), so a seeded episode reproduces the reference's episode
move for move.  The step itself (both legal-move generations, action decode,
die bookkeeping, moves, end check, flip, observation) runs in the HIP kernel
k_step through narde_host_step.
"""
import numpy as np

from .. import _lib
from .._compat import Env, spaces
from .narde import Narde


class NardeEnv(Env):
    metadata = {"render_modes": ["human"], "render_fps": 4}

    def __init__(self, render_mode=None):
        super().__init__()
        self.game = Narde()
        self.current_player = 1
        self.render_mode = render_mode
        self.observation_space = spaces.Box(low=-15, high=15, shape=(24,), dtype=np.int32)
        self.action_space = spaces.Tuple((spaces.Discrete(24 * 24), spaces.Discrete(24 * 24)))
        self._board = np.zeros((1, 24), np.int8)
        self._off = np.zeros((1, 2), np.uint8)
        self._ft = np.zeros((1, 2), np.uint8)
        self._pl = np.zeros(1, np.int8)
        self._dice = np.zeros((1, 2), np.uint8)
        self._act = np.zeros((1, 2), np.int16)
        self._obs = np.zeros((1, 24), np.int32)
        self._rew = np.zeros(1, np.int32)
        self._term = np.zeros(1, np.uint8)

    def _get_obs(self):
        return self.game.get_perspective_board(self.current_player)

    @staticmethod
    def _code(c):
        c = int(c)
        return c if 0 <= c < 576 else -1  # never matches a listed move (`move1 in valid_moves`, narde_env.py:63)

    def step(self, action):
        # narde_env.py:29 -- two draws from the global legacy RNG, roll order kept
        dice = [np.random.randint(1, 7), np.random.randint(1, 7)]
        m1, m2 = action
        g = self.game
        board = np.asarray(g.board)
        if board.shape != (24,) or np.abs(board).max(initial=0) > 15:
            raise ValueError("board must be 24 points with counts in [-15, 15]")
        self._board[0] = board
        self._off[0] = (g.borne_off_white, g.borne_off_black)
        self._ft[0] = (bool(g.first_turn_white), bool(g.first_turn_black))
        self._pl[0] = 1 if self.current_player == 1 else -1
        self._dice[0] = dice
        self._act[0] = (self._code(m1), self._code(m2))
        _lib.host_handle().call(
            "narde_host_step", 1, _lib.ptr(self._board), _lib.ptr(self._off), _lib.ptr(self._ft),
            _lib.ptr(self._pl), _lib.ptr(self._dice), _lib.ptr(self._act), _lib.ptr(self._obs),
            _lib.ptr(self._rew), _lib.ptr(self._term))
        g._load(self._board[0], self._off[0], self._ft[0])
        self.current_player = int(self._pl[0])
        return (self._obs[0].copy(), int(self._rew[0]), bool(self._term[0]), False, {})

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            np.random.seed(seed)
        self.game = Narde()
        while True:
            white_roll = np.random.randint(1, 7)
            black_roll = np.random.randint(1, 7)
            if white_roll != black_roll:
                break
        self.current_player = 1 if white_roll > black_roll else -1
        return self._get_obs(), {}

    def get_valid_actions(self, roll):
        """The README's env.get_valid_actions(roll) (README.md:156-165): the
        set of plays the next step would carry out for this roll and the
        current player (Narde.get_valid_plays; moves in the mover's
        perspective, as get_valid_moves returns them)."""
        return self.game.get_valid_plays(roll, self.current_player)

    def render(self):
        if self.render_mode == "human":
            s = ""
            for i in range(24):
                s += f"{self.game.board[i]:>3} "
                if (i + 1) % 6 == 0:
                    s += "\n"
            print(s)

    def close(self):
        pass

    def _check_game_ended(self):
        """narde_env.py:134-141 (host bookkeeping on the mirrored counters)."""
        if self.current_player == 1 and self.game.borne_off_white == 15:
            return True, 1 if self.game.borne_off_black > 0 else 2
        if self.current_player == -1 and self.game.borne_off_black == 15:
            return True, 1 if self.game.borne_off_white > 0 else 2
        return False, 0
