from gym_narde.envs.narde_env import NardeEnv  # noqa: F401  (gym_narde/envs/__init__.py:1)
