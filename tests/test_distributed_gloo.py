"""World-size-2 rehearsal of the multi-GPU path on CPU (gloo).

Each rank owns a contiguous shard of global env ids (gym_narde.distributed.
env_shard), runs its shard -- here with the CPU oracle standing in for the
GPU kernels, which this container lacks -- and the statistics are combined
with the same gather_stats the GPU run uses (RCCL there, gloo here).  The
gathered result must equal one process running all envs: device dice are
keyed by the global env id, so sharding cannot change any env's game."""
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


def _rank_main(rank, world, port, out_path):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "gym-narde_amd"), os.path.join(root, "oracle")]
    import torch.distributed as dist

    import oracle as Orc
    from gym_narde import distributed as D

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    r, w, _ = D.init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    first, per = D.env_shard(B, r, w)
    sp = Orc.SelfPlay(per, seed=SEED, env0=first)
    sp.reset(0)
    sp.run(PLIES, record=False)
    gathered = D.gather_stats(torch.from_numpy(sp.stats.copy()))
    if r == 0:
        np.save(out_path, gathered.numpy())
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


def test_gloo_world2_equals_single_process(tmp_path):
    out = str(tmp_path / "gathered.npy")
    mp.spawn(_rank_main, args=(2, _free_port(), out), nprocs=2, join=True)
    gathered = np.load(out)
    sp = O.SelfPlay(B, seed=SEED, env0=0)
    sp.reset(0)
    sp.run(PLIES, record=False)
    assert gathered.shape == (B, 3)
    assert np.array_equal(gathered, sp.stats)
    from gym_narde.distributed import summarize

    s = summarize(torch.from_numpy(gathered))
    assert s["episodes"] > 0 and s["white_points"] + s["black_points"] > 0
