"""World-size-2 and -4 rehearsals of the multi-GPU path on CPU (gloo).

Each rank owns a contiguous shard of global env ids (gym_narde.distributed.
env_shard) and plays it with the product's own rules engine -- narde_rules.h,
the source the HIP kernels are built from, compiled for the host
(tests/hostcheck: hc_reset_batch + hc_selfplay, the same per-env Philox
draws keyed by the global env id) because this container has no GPU -- and
the statistics are combined with the same gather_stats the GPU run uses
(RCCL there, gloo here).  The gathered result must equal the CPU oracle
playing all envs in one process: sharding cannot change any env's game."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import oracle as O

B, PLIES, SEED = 1024, 150, 77


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard_selfplay(lib, first, per):
    """The rank's shard through the host build of the device rules engine."""
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    b = np.zeros((per, 24), np.int8)
    off = np.zeros((per, 2), np.uint8)
    ft = np.zeros((per, 2), np.uint8)
    pl = np.zeros(per, np.int8)
    el = np.zeros(per, np.uint16)
    st = np.zeros((per, 3), np.int32)
    lib.hc_reset_batch(ctypes.c_int64(per), ctypes.c_int64(first), ctypes.c_uint64(SEED), ctypes.c_uint32(0),
                       P(b), P(off), P(ft), P(pl), P(el))
    lib.hc_selfplay(ctypes.c_int64(per), ctypes.c_int64(first), ctypes.c_uint64(SEED), ctypes.c_uint32(0),
                    ctypes.c_int(PLIES), ctypes.c_int(0), ctypes.c_int(1000), P(b), P(off), P(ft), P(pl), P(el),
                    P(st), None, None, None, None, None, None, None, None)
    return st


def _rows_of(st, nrows=64):
    """VecNardeEnv.totals()'s partial rows (narde_get_totals: row b sums
    the b-th contiguous range of ceil(n / 64) envs), restated on the host."""
    n = st.shape[0]
    per = -(-n // nrows)
    rows = np.zeros((nrows, 3), np.int64)
    for b in range(nrows):
        rows[b] = st[b * per:min(n, (b + 1) * per)].astype(np.int64).sum(0)
    return rows


def _rank_main(rank, world, port, lib_path, out_path):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "gym-narde_amd")]
    import torch.distributed as dist

    from gym_narde import distributed as D

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    r, w, _ = D.init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    first, per = D.env_shard(B, r, w)
    st = _shard_selfplay(ctypes.CDLL(lib_path), first, per)
    gathered = D.gather_stats(torch.from_numpy(st))
    totals = D.gather_totals(torch.from_numpy(st))
    rows = D.gather_total_rows(torch.from_numpy(_rows_of(st)))  # what bench.py's timed region gathers
    if r == 0:
        np.save(out_path, gathered.numpy())
        np.save(out_path + ".totals.npy", totals.numpy())
        np.save(out_path + ".rows.npy", rows.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_env_shard_partition():
    from gym_narde.distributed import env_shard

    for world in (1, 2, 4, 8):
        ranges = [env_shard(8 * 65536, r, world) for r in range(world)]
        assert ranges[0][0] == 0 and all(c == 8 * 65536 // world for _, c in ranges)
        assert all(ranges[i][0] + ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
    with pytest.raises(ValueError):
        env_shard(10, 0, 3)


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_shards_equal_single_process(tmp_path, hostcheck, world):
    out = str(tmp_path / "gathered.npy")
    mp.spawn(_rank_main, args=(world, _free_port(), hostcheck._name, out), nprocs=world, join=True)
    gathered = np.load(out)
    sp = O.SelfPlay(B, seed=SEED, env0=0)
    sp.reset(0)
    sp.run(PLIES, record=False)
    assert gathered.shape == (B, 3)
    assert np.array_equal(gathered, sp.stats)
    totals = np.load(out + ".totals.npy")  # (world, 3): each rank's shard summed
    per = B // world
    assert np.array_equal(totals, sp.stats.astype(np.int64).reshape(world, per, 3).sum(1))
    rows = np.load(out + ".rows.npy")  # (world, 64, 3) partial rows per rank
    assert rows.shape == (world, 64, 3) and np.array_equal(rows.sum(1), totals)
    from gym_narde.distributed import summarize

    s = summarize(torch.from_numpy(gathered))
    assert s["episodes"] > 0 and s["white_points"] + s["black_points"] > 0


def test_gather_totals_without_process_group():
    from gym_narde.distributed import gather_totals, summarize

    st = torch.tensor([[1, 2, 0], [3, 0, 6]], dtype=torch.int32)
    tot = gather_totals(st)
    assert tot.dtype == torch.int64 and tot.tolist() == [[4, 2, 6]]
    assert summarize(tot) == {"episodes": 4, "white_points": 2, "black_points": 6}


def test_gather_total_rows_without_process_group():
    from gym_narde.distributed import gather_total_rows

    rows = torch.arange(12, dtype=torch.int64).reshape(4, 3)
    out = gather_total_rows(rows)
    assert out.shape == (1, 4, 3) and torch.equal(out[0], rows)


class _FakeRccl:
    """Stands in for librccl in RcclGather's set-up: status
    codes per entry point, no device work."""

    def __init__(self, uid_rc=0, init_rc=0):
        self.uid_rc, self.init_rc, self.destroyed = uid_rc, init_rc, 0

    def ncclGetUniqueId(self, p):
        return self.uid_rc

    def ncclCommInitRank(self, comm, world, uid, rank):
        if self.init_rc == 0:
            ctypes.cast(comm, ctypes.POINTER(ctypes.c_void_p))[0] = 0x1234
        return self.init_rc

    def ncclCommDestroy(self, comm):
        self.destroyed += 1
        return 0

    def ncclGetErrorString(self, rc):
        return b"injected"


def _rccl_agree_main(rank, world, port, case, out_path):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "gym-narde_amd")]
    import torch.distributed as dist

    from gym_narde import distributed as D

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    D.init_from_env(backend="gloo")
    fake = _FakeRccl()
    if case == "load" and rank == 1:
        def _fail():
            raise OSError("injected: no librccl")
        D._rccl = _fail
    else:
        if case == "uid" and rank == 0:
            fake.uid_rc = 3
        if case == "init" and rank == world - 1:
            fake.init_rc = 2
        D._rccl = lambda: fake
    try:
        g = D.RcclGather(torch.zeros((4, 3), dtype=torch.int64))
        outcome = "built"
        g.close()
    except RuntimeError:
        outcome = "raised"
    # every rank reaches this barrier: no rank is left inside a collective
    dist.barrier()
    with open(f"{out_path}.{rank}", "w") as f:
        f.write(f"{outcome} {fake.destroyed}")
    dist.destroy_process_group()


@pytest.mark.parametrize("case", ["load", "uid", "init", "ok"])
def test_rccl_gather_setup_agrees_across_ranks(tmp_path, case):
    """A failure at any set-up stage on any one rank makes every rank raise
    (so bench.py falls back to the process group's collective on every rank
    alike); with no failure every rank builds its communicator."""
    world = 3
    out = str(tmp_path / "outcome")
    mp.spawn(_rccl_agree_main, args=(world, _free_port(), case, out), nprocs=world, join=True)
    got = [open(f"{out}.{r}").read().split() for r in range(world)]
    want = "built" if case == "ok" else "raised"
    assert [g[0] for g in got] == [want] * world, got
    if case == "init":  # the ranks whose init succeeded destroyed their communicator
        assert [int(g[1]) for g in got] == [1] * (world - 1) + [0]
