"""The checker behind bench.py's parity_check leg (oracle/replay.py), on CPU.

A "device run" is played here by the oracle itself in one piece; the
checker, loaded with the state snapshotted before it, replays it in env
chunks on a thread pool and must report zero mismatches -- and exactly the
entries a test corrupts afterwards.  Both rules modes, a ragged batch (the
last chunk partly full), a start at an odd ply (the Philox block of a ply
pair is re-derived mid-pair) and a TimeLimit short enough that envs
truncate inside the replay.
"""
import numpy as np
import pytest

import oracle as O
import replay as R


def device_like(rec, full):
    """Oracle records in the device rollout buffers' dtypes."""
    out = dict(obs=rec["obs"].astype(np.int32), reward=rec["reward"].astype(np.int32),
               terminated=rec["terminated"].copy(), truncated=rec["truncated"].copy(),
               legal=rec["legal"].view(np.int64).copy())
    out["actions"] = rec["played"].view(np.int64).copy() if full else rec["action"].copy()
    return out


def state_of(sp):
    return dict(board=sp.board.copy(), off=sp.off.copy(), first_turn=sp.ft.copy(), player=sp.player.copy(),
                elapsed=sp.elapsed.astype(np.int16), stats=sp.stats.copy(), t=sp.t)


def played_run(full, n=5000, seed=77, env0=123, pre=25, plies=24, P=15, max_steps=40):
    sp = O.SelfPlay(n, seed=seed, env0=env0, max_steps=max_steps)
    sp.reset(0)
    run = sp.run_full if full else sp.run
    run(pre, record=False)
    before = state_of(sp)
    run(plies - P, record=False)
    rec = run(P)
    return before, device_like(rec, full), state_of(sp), sp


@pytest.mark.parametrize("full", [False, True])
def test_replay_equals_one_piece_run(full):
    before, bufs, after, sp = played_run(full)
    res = R.check(before, bufs, after, 24, 77, env0=123, full=full, threads=4, max_steps=40)
    assert res["mismatches"] == 0, res
    assert res["envs"] == 5000 and res["plies"] == 24 and res["plies_compared_per_output"] == 15
    assert set(res["by_field"]) >= {"obs", "reward", "terminated", "truncated", "actions", "legal",
                                    "final_state_envs"}
    assert bufs["truncated"].sum() > 0  # TimeLimit 40 truncates inside the replay


@pytest.mark.parametrize("full", [False, True])
def test_replay_counts_corrupted_entries(full):
    before, bufs, after, _ = played_run(full)
    bufs["legal"][3, 4999] ^= 1 << 5
    bufs["obs"][0, 17, 2] += 1
    bufs["actions"][8, 0] = bufs["actions"][8, 0] + 1
    after["board"][4096, 0] += 1  # the first env of the second chunk
    res = R.check(before, bufs, after, 24, 77, env0=123, full=full, threads=4, max_steps=40)
    f = res["by_field"]
    assert (f["legal"], f["obs"], f["actions"], f["final_state_envs"]) == (1, 1, 1, 1), f
    assert res["mismatches"] == 4


def test_replay_prefix_and_totals_rows():
    """A prefix of the batch (envs=...) and the launch's per-256-env totals rows."""
    before, bufs, after, sp = played_run(False)
    rows = np.zeros(((5000 + 255) // 256, 3), np.int64)
    for i in range(5000):
        rows[i // 256] += sp.stats[i]
    res = R.check(before, bufs, after, 24, 77, env0=123, threads=3, max_steps=40, totals_rows=rows)
    assert res["by_field"]["totals_rows"] == 0 and res["mismatches"] == 0
    rows[7, 1] += 1
    res = R.check(before, bufs, after, 24, 77, env0=123, threads=3, max_steps=40, totals_rows=rows)
    assert res["by_field"]["totals_rows"] == 1
    res = R.check(before, bufs, after, 24, 77, env0=123, envs=1000, threads=3, max_steps=40)
    assert res["envs"] == 1000 and res["mismatches"] == 0


def test_bench_parity_budget():
    import bench

    # the driver's shape: both rules' 20-ply launches are checked whole
    assert bench.parity_envs(65536, 20, "ref2", 160) == 65536
    assert bench.parity_envs(65536, 20, "full4", 160) == 65536
    # 1,000-ply FULL4 launches: a prefix of >= 16,384 envs, whole workgroups
    n = bench.parity_envs(65536, 1000, "full4", 160)
    assert n >= bench.PARITY_MIN_ENVS and n % 256 == 0 and n < 65536
    # the default bench's 200,000 timed plies cannot be replayed whole
    assert bench.parity_envs(65536, 200000, "ref2", 160) < 65536
