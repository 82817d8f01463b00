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
