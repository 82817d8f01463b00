"""bench.py --gpus N starts and checks its N ranks.

Run plainly with --gpus 2 (no WORLD_SIZE), the bench must start two ranks
itself -- as the driver's SCALE run would get them from torchrun -- shard
the global env ids, time the region with barrier + max over ranks, and
gather both ranks' episode totals.  On this CPU-only machine every rank plays
its shard through the test-only host engine (tests/bench_host_engine.py:
the device rules engine compiled for the CPU) over gloo; the line is marked
as such and its timing means nothing.  The totals must equal the CPU oracle
playing the same global env ids in one process.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENGINE = os.path.join(ROOT, "tests", "bench_host_engine.py")
QUIET = ["--ramp-launches", "0", "--ramp-ms", "0", "--api-steps", "0", "--fused-launches", "0",
         "--other-launches", "0", "--dqn-steps", "0", "--no-cpu-baseline"]


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(NARDE_BENCH_TEST_ENGINE=ENGINE, OMP_NUM_THREADS="1", **(env_extra or {}))
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def _line(proc):
    assert proc.returncode == 0, proc.stderr[-4000:]
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, proc.stdout  # ONE line, from rank 0 only
    return json.loads(lines[0])


def _oracle_rank_totals(envs_per_rank, world, plies, seed):
    sp = O.SelfPlay(envs_per_rank * world, seed=seed, env0=0)
    sp.reset(0)
    sp.run(plies, record=False)
    return sp.stats.astype(np.int64).reshape(world, envs_per_rank, 3).sum(1)


def test_bench_gpus2_spawns_two_ranks(hostcheck):
    steps, warmup, ppl = 24, 6, 12
    p = _run(["--gpus", "2", "--steps", str(steps), "--warmup", str(warmup), "--plies-per-launch", str(ppl),
              "--envs", "65536", *QUIET], timeout=400)
    line = _line(p)
    assert line["n_gpus"] == 2
    cfg = line["config"]
    assert cfg["envs_per_gpu"] == 65536 and cfg["global_envs"] == 131072
    assert cfg["collective"] == {**cfg["collective"], "backend": "gloo", "world_size": 2}
    assert "not a measurement" in line["engine"]
    # both ranks' totals, gathered in the timed region, equal the oracle on
    # the same global ids: the untimed launch-path warm-up (3 x the first
    # and the last launch of the region, 12 plies each) + --warmup + --steps
    plies = 3 * 2 * ppl + warmup + steps
    want = _oracle_rank_totals(65536, 2, plies, seed=0)
    assert np.array_equal(np.array(cfg["rank_totals"], np.int64), want)
    assert cfg["episodes_finished"] == int(want[:, 0].sum())
    assert line["value"] > 0 and line["steps"] == steps


def test_bench_world_size_must_match_gpus(hostcheck):
    # under a launcher that started a different number of ranks: refuse
    p = _run(["--gpus", "2", "--steps", "4", "--envs", "256", *QUIET],
             env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr


def test_bench_gpus1_runs_one_rank(hostcheck):
    p = _run(["--gpus", "1", "--steps", "8", "--warmup", "2", "--plies-per-launch", "4", "--envs", "512",
              *QUIET])
    line = _line(p)
    assert line["n_gpus"] == 1 and line["config"]["global_envs"] == 512
    want = _oracle_rank_totals(512, 1, 3 * 2 * 4 + 2 + 8, seed=0)
    assert np.array_equal(np.array(line["config"]["rank_totals"], np.int64), want)


@pytest.mark.parametrize("world", [4])
def test_bench_gpus4_rank_totals(hostcheck, world):
    p = _run(["--gpus", str(world), "--steps", "10", "--warmup", "0", "--plies-per-launch", "10",
              "--envs", "1024", *QUIET])
    line = _line(p)
    assert line["n_gpus"] == world and line["config"]["global_envs"] == world * 1024
    want = _oracle_rank_totals(1024, world, 3 * 10 + 10, seed=0)
    assert np.array_equal(np.array(line["config"]["rank_totals"], np.int64), want)


def test_bench_gpus8_scale_line(hostcheck):
    """the N = 8 line the driver's SCALE run prints --
    8 ranks, configs[4] named at 8 x 65,536 global envs, a CPU baseline
    measured by the launching process before the ranks start, and every
    rank's totals equal to the oracle on the same global env ids."""
    steps, ppl = 4, 4
    quiet = [a for a in QUIET if a != "--no-cpu-baseline"]
    p = _run(["--gpus", "8", "--steps", str(steps), "--warmup", "0", "--plies-per-launch", str(ppl),
              "--envs", "65536", "--cpu-seconds", "0.3", "--cpu-cores", "2", *quiet], timeout=600)
    line = _line(p)
    assert line["n_gpus"] == 8
    cfg = line["config"]
    assert cfg["envs_per_gpu"] == 65536 and cfg["global_envs"] == 524288
    assert cfg["workload"].startswith("configs[4]: batch=524288 sharded 8 x MI355X")
    cpu = line["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["cores"] == 2 and cpu["kind"] == "port"
    assert isinstance(line["timed_region_host_us"]["start_skew_removed"], float)
    want = _oracle_rank_totals(65536, 8, 3 * 2 * ppl + steps, seed=0)
    assert np.array_equal(np.array(cfg["rank_totals"], np.int64), want)


def test_aligned_start_only_on_one_node(monkeypatch):
    """time.monotonic() is one clock only within a node; with
    ranks on several nodes the aligned start is skipped (plain barrier)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("narde_bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert bench.single_node(8) and not bench.single_node(16)
    assert bench.aligned_start(16, None) is None  # returns before any collective
    assert bench.aligned_start(1, None) == 0.0
    monkeypatch.delenv("LOCAL_WORLD_SIZE")
    assert bench.single_node(4)
