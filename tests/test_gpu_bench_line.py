"""bench.py --gpus 1 on the GPU ("a -m gpu test runs
--gpus 1 unchanged"): one rank, no launcher, the product engine (libnarde.so,
k_rollout_pc), and the line carries the world size, the env counts, the
roofline object and the episode totals the last timed launch reduced on the
device -- equal to the CPU oracle playing the same env ids for the same plies.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QUIET = ["--ramp-launches", "0", "--ramp-ms", "0", "--api-steps", "0", "--fused-launches", "0",
         "--other-launches", "0", "--dqn-steps", "0", "--no-cpu-baseline"]


def test_bench_gpus1_line_and_totals():
    envs, ppl, warmup, steps = 4096, 50, 100, 200
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "NARDE_BENCH_TEST_ENGINE"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--envs", str(envs),
                        "--plies-per-launch", str(ppl), "--warmup", str(warmup), "--steps", str(steps), *QUIET],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert "engine" not in line  # the product engine, not the host rehearsal
    assert line["n_gpus"] == 1 and line["steps"] == steps and line["warmup"] == warmup
    cfg = line["config"]
    assert cfg["envs_per_gpu"] == envs and cfg["global_envs"] == envs
    assert cfg["collective"]["world_size"] == 1
    assert line["roofline"]["bound"] == "hbm" and 0 < line["roofline"]["frac"] < 1.5
    assert line["value"] > 0 and line["ms_per_step"] > 0
    # the untimed launch-path warm-up (3 x the first and the last launch of
    # the region) + --warmup + --steps plies, from a fresh reset at seed 0
    plies = 3 * 2 * ppl + warmup + steps
    sp = O.SelfPlay(envs, seed=0, env0=0)
    sp.reset(0)
    sp.run(plies, record=False)
    want = sp.stats.astype(np.int64).sum(0, keepdims=True)
    assert np.array_equal(np.array(cfg["rank_totals"], np.int64), want)
