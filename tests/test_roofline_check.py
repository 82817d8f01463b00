"""tools/roofline_check.py recomputes a bench line's HBM and issue fractions
from the committed profiles."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(path):
    return subprocess.run([sys.executable, os.path.join(ROOT, "tools", "roofline_check.py"), path],
                          capture_output=True, text=True, timeout=60)


def test_roofline_check_recomputes_a_line(tmp_path):
    envs, plies, ms = 65536, 20, 0.0375
    nbytes = envs * (114 * plies + 64)
    frac = nbytes / (ms * 1e-3) / 8e12
    line = {"metric": "m", "steps": plies, "config": {"rules": "ref2", "envs_per_gpu": envs},
            "roofline": {"kernel_ms": ms, "frac": round(frac, 5), "issue": None},
            "other_rules": {"rules": "full4", "kernel_ms": 0.09,
                            "frac": round(envs * (118 * plies + 64) / 0.09e-3 / 8e12, 5), "issue": None}}
    p = tmp_path / "bench.json"
    p.write_text("banner\n" + json.dumps(line) + "\n")
    r = _run(str(p))
    assert r.returncode == 0, r.stdout + r.stderr
    rows = [json.loads(x) for x in r.stdout.splitlines()]
    assert [x["leg"] for x in rows] == ["headline", "other_rules"]
    assert abs(rows[0]["hbm_frac"] - frac) < 1e-5
    # a line whose fraction disagrees with its own kernel time fails
    line["roofline"]["frac"] = round(frac * 1.1, 5)
    p.write_text(json.dumps(line) + "\n")
    assert _run(str(p)).returncode == 1


def test_summaries_apply_only_to_their_kernel():
    """A PMC/SQ summary of another kernel (e.g. the retired k_rollout_full<true>)
    is never combined with a launch's timings, in bench.py and in the checker
    alike."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    sys.path.insert(0, ROOT)
    import bench
    import roofline_check as rc

    for full in (False, True):
        for plies in (1, 20, 32, 33, 1000):
            assert rc.launched_kernel(full, plies) == bench.kernel_name(full, plies)
    k = bench.kernel_name(True, 20)
    assert rc.matches({"envs": 65536, "plies": 20, "kernel": "k_rollout_pp_full<true>"}, 65536, 20, k)
    # round 5's per-length kernel names are another kernel's summaries
    assert not rc.matches({"envs": 65536, "plies": 20, "kernel": "k_rollout_pp_full<true, true>"}, 65536, 20, k)
    assert not rc.matches({"envs": 65536, "plies": 20, "kernel": "k_rollout_wave<true>"}, 65536, 20, k)
    assert not rc.matches({"envs": 65536, "plies": 20, "kernel": "k_rollout_full<true>"}, 65536, 20, k)
    assert not rc.matches({"envs": 65536, "plies": 20, "kernel": "k_rollout_pc"}, 65536, 20, k)
    # a summary naming no kernel applies to none ("" is a
    # substring of every name)
    assert not rc.matches({"envs": 65536, "plies": 20}, 65536, 20, k)
    assert not rc.matches({"envs": 65536, "plies": 20, "kernel": ""}, 65536, 20, k)
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "pmc.json")
        for kern in (None, ""):
            summ = {"envs": 65536, "plies": 20, "hbm_bytes_per_launch": 1}
            if kern is not None:
                summ["kernel"] = kern
            json.dump(summ, open(p, "w"))
            assert bench.load_traffic(p, 65536, 20, k) is None
        json.dump({"envs": 65536, "plies": 20, "hbm_bytes_per_launch": 1, "kernel": "k_rollout_pp_full"},
                  open(p, "w"))
        assert bench.load_traffic(p, 65536, 20, k) == 1


def test_cpu_baseline_handover_needs_this_launchs_marker(monkeypatch):
    """bench.py rank 0 takes a handed-over CPU baseline only when the marker
    names its own MASTER_PORT and an ancestor pid."""
    sys.path.insert(0, ROOT)
    import bench

    cpu = {"value": 1.0}
    monkeypatch.setenv("MASTER_PORT", "29611")
    monkeypatch.setenv(bench.CPU_BASELINE_ENV, json.dumps(cpu))  # unmarked: an outer shell's
    assert bench.handed_cpu_baseline() is None
    mark = {"launcher_pid": os.getppid(), "master_port": 29611, "cpu": cpu}
    monkeypatch.setenv(bench.CPU_BASELINE_ENV, json.dumps(mark))
    assert bench.handed_cpu_baseline() == cpu
    monkeypatch.setenv("MASTER_PORT", "29612")  # another launch
    assert bench.handed_cpu_baseline() is None
    mark["launcher_pid"] = 1 << 30  # not an ancestor
    monkeypatch.setenv("MASTER_PORT", "29611")
    monkeypatch.setenv(bench.CPU_BASELINE_ENV, json.dumps(mark))
    assert bench.handed_cpu_baseline() is None
