"""gymnasium surface (Env, spaces, TimeLimit) used by the facade.

When gymnasium is importable its own classes are used, so
`gym.make('gym_narde:narde-v0')` behaves exactly like the reference's
registration.  It is not installed on this image (nor on the GPU box), so a
minimal stand-in with the same attribute names is provided; only what the
reference env and its callers touch is implemented.
"""
import numpy as np

try:  # pragma: no cover - depends on the environment
    import gymnasium as _gym
    from gymnasium import spaces  # noqa: F401
    Env = _gym.Env
    HAVE_GYMNASIUM = True
except ImportError:
    _gym = None
    HAVE_GYMNASIUM = False

    class Env:
        metadata = {"render_modes": []}
        render_mode = None

        def __init__(self, *a, **k):
            pass

        @property
        def unwrapped(self):
            return self

        def close(self):
            pass

    class _Spaces:
        class Box:
            def __init__(self, low, high, shape, dtype):
                self.low = np.full(shape, low, dtype=dtype)
                self.high = np.full(shape, high, dtype=dtype)
                self.shape = tuple(shape)
                self.dtype = np.dtype(dtype)

            def contains(self, x):
                x = np.asarray(x)
                return x.shape == self.shape and bool(((x >= self.low) & (x <= self.high)).all())

            def sample(self):
                return np.random.randint(self.low, self.high + 1).astype(self.dtype)

        class Discrete:
            def __init__(self, n):
                self.n = int(n)

            def contains(self, x):
                return 0 <= int(x) < self.n

            def sample(self):
                return int(np.random.randint(self.n))

        class Tuple:
            def __init__(self, spaces_):
                self.spaces = tuple(spaces_)

            def contains(self, x):
                return len(x) == len(self.spaces) and all(s.contains(v) for s, v in zip(self.spaces, x))

            def sample(self):
                return tuple(s.sample() for s in self.spaces)

    spaces = _Spaces


class TimeLimit:
    """gymnasium.wrappers.TimeLimit semantics: truncated once the number of
    steps since reset reaches max_episode_steps."""

    def __init__(self, env, max_episode_steps):
        self.env = env
        self._max = int(max_episode_steps)
        self._elapsed = None

    def __getattr__(self, name):
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return self.env.unwrapped

    def reset(self, **kwargs):
        self._elapsed = 0
        return self.env.reset(**kwargs)

    def step(self, action):
        obs, reward, terminated, truncated, info = self.env.step(action)
        self._elapsed += 1
        if self._elapsed >= self._max:
            truncated = True
        return obs, reward, terminated, truncated, info
