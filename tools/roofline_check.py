#!/usr/bin/env python3
"""Recompute a bench line's roofline fractions from the committed profiles.

Reads one bench JSON line (a BENCH_rNN.json file, or bench.py's stdout) and
recomputes, from profiles/:
  * the HBM figure: the launch's algorithmic bytes (bench.py launch_bytes:
    114 B/env/ply REF2, 118 FULL4, + 64 B/env record r+w) / kernel_ms /
    8 TB/s, and the PMC traffic of profiles/pmc_k_rollout[_full][_p<P>].json;
  * the issue figure: VALU wave-instructions per launch from
    profiles/sq_k_rollout[_full]_p<P>.json / kernel_ms / the 1,024-SIMD
    integer issue peak of one VALU wave-instruction per 4 cycles
    (tools/sq_summary.py; measured in profiles/r05/issue_probe/),
for the headline (`roofline`) and `other_rules`, and prints them beside
the line's own numbers.  Exit status 1 if any recomputed fraction differs
from the line's by more than 1e-3.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HBM_PEAK = 8.0e12
ISSUE_PEAK = 1024 * 2.4e9 / 4  # basis: profiles/r05/issue_probe/summary.json (tools/sq_summary.py)


def bytes_per_launch(envs, plies, full):
    return envs * ((118 if full else 114) * plies + 64)


def profile(name):
    try:
        return json.load(open(os.path.join(ROOT, "profiles", name)))
    except (OSError, ValueError):
        return None


def launched_kernel(full, plies):
    """The kernel a launch of this shape runs (bench.py kernel_name)."""
    return "k_rollout_pp_full<true>" if full else "k_rollout_pc<true>"


def matches(summary, envs, plies, kernel):
    """A PMC/SQ summary applies only if it was measured at this shape on this
    kernel (its `kernel` filter is a prefix of the launched kernel's name; a
    summary that names no kernel applies to none)."""
    k = summary.get("kernel") if summary is not None else None
    return (summary is not None and summary.get("envs") == envs and summary.get("plies") == plies
            and bool(k) and k in kernel)


def check(label, full, envs, plies, kernel_ms, line_frac, line_issue):
    nbytes = bytes_per_launch(envs, plies, full)
    frac = nbytes / (kernel_ms * 1e-3) / HBM_PEAK
    stem = "k_rollout_full" if full else "k_rollout"
    kernel = launched_kernel(full, plies)
    pmc = profile(f"pmc_{stem}_p{plies}.json") or profile(f"pmc_{stem}.json")
    traffic = pmc["hbm_bytes_per_launch"] if matches(pmc, envs, plies, kernel) else None
    sq = profile(f"sq_{stem}_p{plies}.json")
    issue = None
    if matches(sq, envs, plies, kernel):
        issue = sq["valu_per_launch"] / (kernel_ms * 1e-3) / ISSUE_PEAK
    out = {"leg": label, "rules": "full4" if full else "ref2", "plies": plies, "kernel_ms": kernel_ms,
           "hbm_frac": round(frac, 5), "line_hbm_frac": line_frac,
           "traffic_over_algorithmic": round(traffic / nbytes, 4) if traffic else None,
           "issue_frac": round(issue, 4) if issue is not None else None, "line_issue_frac": line_issue}
    ok = abs(frac - line_frac) <= 1e-3 and (issue is None or line_issue is None or abs(issue - line_issue) <= 1e-3)
    return out, ok


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "BENCH.json")
    text = open(src).read() if src != "-" else sys.stdin.read()
    try:  # the driver's record (BENCH_rNN.json) wraps the line in "parsed"
        line = json.loads(text)
    except ValueError:  # bench.py's stdout: the last JSON line
        line = json.loads([ln for ln in text.splitlines() if ln.startswith("{")][-1])
    if "parsed" in line:  # "parsed" keeps a subset of the keys; other_rules from the stdout tail
        tail = line.get("tail", "")
        line = dict(line["parsed"])
        k = tail.find('"other_rules": {')
        if "other_rules" not in line and k >= 0:
            line["other_rules"] = json.JSONDecoder().raw_decode(tail[k + len('"other_rules": '):])[0]
    cfg, rl = line["config"], line["roofline"]
    full = cfg.get("rules") == "full4"
    envs = cfg["envs_per_gpu"]
    plies = line["steps"] if line["steps"] < 1000 else 1000
    results, good = [], True
    r, ok = check("headline", full, envs, min(plies, 1000), rl["kernel_ms"], rl["frac"],
                  (rl.get("issue") or {}).get("frac"))
    results.append(r)
    good &= ok
    other = line.get("other_rules")
    if other:
        r, ok = check("other_rules", other["rules"] == "full4", envs, min(plies, 1000), other["kernel_ms"],
                      other["frac"], (other.get("issue") or {}).get("frac"))
        results.append(r)
        good &= ok
    for r in results:
        print(json.dumps(r))
    return 0 if good else 1


if __name__ == "__main__":
    sys.exit(main())
