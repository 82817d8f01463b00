"""MI355X-native Narde environment, drop-in for dmytroleonenko/gym-narde.

* `gym_narde.envs.NardeEnv` / `gym_narde.envs.narde.Narde` -- the reference's
  scalar API (gym_narde/envs/narde_env.py, narde.py), evaluated in HIP kernels.
* `gym_narde.vector.VecNardeEnv` -- B envs stepped in lockstep on one GPU.
* `gym_narde.distributed` -- one process per GPU, env-id sharding, one RCCL
  all-gather of episode statistics.

Registration mirrors gym_narde/__init__.py:1-7 of the reference
(`narde-v0`, TimeLimit 1000) when gymnasium is installed; `gym_narde.make`
gives the same wrapped env without it.
"""
from ._compat import HAVE_GYMNASIUM, TimeLimit

MAX_EPISODE_STEPS = 1000

if HAVE_GYMNASIUM:  # pragma: no cover - gymnasium is absent on this image
    from gymnasium.envs.registration import register

    register(id="narde-v0", entry_point="gym_narde.envs:NardeEnv",
             max_episode_steps=MAX_EPISODE_STEPS)


def make(id="narde-v0", **kwargs):
    """gym.make('gym_narde:narde-v0') equivalent (TimeLimit-wrapped NardeEnv)."""
    if id.split(":")[-1] != "narde-v0":
        raise ValueError(f"unknown env id {id!r}")
    from .envs import NardeEnv

    return TimeLimit(NardeEnv(**kwargs), MAX_EPISODE_STEPS)
