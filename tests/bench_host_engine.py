"""Test-only engine for bench.py's N-rank plumbing on a machine with no GPU.

bench.py loads this file only when NARDE_BENCH_TEST_ENGINE names it (the CPU
test tests/test_bench_ranks.py does); the product bench never does.  Each
rank plays its shard of global env ids with the host build of the device
rules engine (tests/hostcheck: narde_rules.h compiled for the CPU, the same
Philox draws keyed by the global env id), so the launcher (`--gpus N`
spawning N ranks), the env-id sharding, the barrier / max-over-ranks timing
and the all-gather of every rank's episode totals run exactly as on the GPU
box, over gloo.  Its numbers are NOT measurements: bench.py marks the line
with `engine` and keeps every secondary leg off.
"""
import ctypes
import os
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "hostcheck", "build", "libhostcheck.so")

NAME = "host rehearsal (tests/hostcheck: narde_rules.h on the CPU) -- not a measurement"


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class HostEvent:
    """Stands in for TimingEvent: the host clock when the launch that
    records it runs (the host engine's launches are synchronous)."""

    def __init__(self):
        self.t = None

    def elapsed_ms(self, stop):
        return (stop.t - self.t) * 1e3


class HostVecEnv:
    """The slice of VecNardeEnv bench.py's timed region uses (REF2 only)."""

    def __init__(self, lib, num_envs, seed, env_id_offset, max_episode_steps=1000):
        self.lib, self.n, self.first, self.seed = lib, int(num_envs), int(env_id_offset), int(seed)
        self.max_steps = int(max_episode_steps)
        n = self.n
        self.board = np.zeros((n, 24), np.int8)
        self.off = np.zeros((n, 2), np.uint8)
        self.ft = np.zeros((n, 2), np.uint8)
        self.player = np.zeros(n, np.int8)
        self.elapsed = np.zeros(n, np.uint16)
        self.stats = np.zeros((n, 3), np.int32)
        self.t = 0
        lib.hc_reset_batch(ctypes.c_int64(n), ctypes.c_int64(self.first), ctypes.c_uint64(self.seed),
                           ctypes.c_uint32(0), _p(self.board), _p(self.off), _p(self.ft), _p(self.player),
                           _p(self.elapsed))

    def rollout_buffers(self, plies):
        return dict(obs=None, reward=None, terminated=None, truncated=None, legal=None, actions=None)

    def rollout(self, plies, bufs=None):
        self.lib.hc_selfplay(ctypes.c_int64(self.n), ctypes.c_int64(self.first), ctypes.c_uint64(self.seed),
                             ctypes.c_uint32(self.t), ctypes.c_int(plies), ctypes.c_int(0),
                             ctypes.c_int(self.max_steps), _p(self.board), _p(self.off), _p(self.ft),
                             _p(self.player), _p(self.elapsed), _p(self.stats),
                             None, None, None, None, None, None, None, None)
        self.t += plies
        return bufs

    def rollout_launcher(self, plies, bufs, events=None, totals=None):
        ev0, ev1 = events if events is not None else (None, None)

        def launch():
            if ev0 is not None:
                ev0.t = time.perf_counter()
            self.rollout(plies, bufs)
            if totals is not None:
                totals.copy_(self.wg_totals())
            if ev1 is not None:
                ev1.t = time.perf_counter()

        return launch

    def wg_totals(self):
        """narde_rollout_timed's totals rows restated: row r sums the
        statistics of envs 256 r .. 256 r + 255."""
        rows = -(-self.n // 256)
        pad = np.zeros((rows * 256, 3), np.int64)
        pad[:self.n] = self.stats
        return torch.from_numpy(pad.reshape(rows, 256, 3).sum(1))

    def close(self):
        pass


class Engine:
    name = NAME
    device = torch.device("cpu")

    def __init__(self, local_rank):
        self.lib = ctypes.CDLL(LIB)

    def make_env(self, per, first, seed, rules):
        if rules != "ref2":
            raise ValueError("the host rehearsal engine plays REF2 only")
        return HostVecEnv(self.lib, per, seed, first)

    def timing_event(self):
        return HostEvent()

    def sync(self):
        pass
