#!/usr/bin/env python3
"""DIAGNOSTIC (round 5): any SQ counters of one rocprofv3 --pmc pass over
tools/pmc_target.py, per launch and per 64-env group-ply (both waves of a
producer/consumer pair together).  SQ_INSTS_* count wave-instructions,
SQ_WAVE_CYCLES / SQ_ACTIVE_* / SQ_WAIT_* / SQ_INST_CYCLES_* quad-cycles
(tools/sq_summary.py).  Usage: sq_breakdown.py DIR KERNEL PLIES [ENVS]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from sq_summary import per_dispatch  # noqa: E402


def main():
    root, kernel, plies = sys.argv[1], sys.argv[2], int(sys.argv[3])
    envs = int(sys.argv[4]) if len(sys.argv) > 4 else 65536
    vals, dur = per_dispatch(root, kernel)
    groups = envs // 64
    out = {"kernel": kernel, "plies": plies, "dispatches": len(dur) - 1,
           "profiled_us": round(sum(dur[1:]) / len(dur[1:]) / 1e3, 2), "per_group_ply": {}}
    for c, v in sorted(vals.items()):
        m = sum(v[1:]) / len(v[1:])
        out["per_group_ply"][c] = round(m / (groups * plies), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
