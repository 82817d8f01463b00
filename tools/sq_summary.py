#!/usr/bin/env python3
"""Summarise one rocprofv3 SQ-counter pass into profiles/sq_<name>.json: the
issue side of SURVEY.md section 8(d)'s roofline ("also report ops/step x
steps/s vs the MI355X VALU peak as a secondary figure").

Input: the *_counter_collection.csv of one pass over tools/pmc_target.py
(at most 8 SQ_ counters per pass, MI355X_MICROARCH.md), e.g.
  rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \\
      SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU \\
      --output-format csv -d OUT -o sq -- python3 tools/pmc_target.py --plies 20 --launches 5
Keeps the dispatches of the named kernel, drops the first (warm-up) one and
averages per launch.  SQ_INSTS_* count wave-instructions; SQ_WAVE_CYCLES,
SQ_WAIT_* and SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md,
constants table).

The issue peak (measured, profiles/r05/issue_probe/summary.json from
tools/issue_probe.hip: every VALU kind the rules engine uses, at 1, 2 and 4
waves per SIMD, shader-clock cycles per wave and SQ_BUSY_CYCLES):
  * one wave alone issues a VALU instruction at most every 4 cycles,
    whatever the kind -- the bound of every kernel's rule wave (one per
    SIMD at B = 65,536: 64 envs a wave, 1,024 SIMDs);
  * two or more waves on a SIMD share it at 4 cycles per instruction for the
    "slow" kinds (shift left, bfe, add3, and_or / or3 / lshl_or, cndmask
    e64, bcnt, ffbl, min / max, perm, SDWA, mul) and at 2 cycles for the
    "fast" kinds (add / sub, and / or / xor / not, bitop3, shift right,
    f32 add / fma) -- MI355X_MICROARCH.md's "2 cycles (SIMD-32)" holds for
    the fast kinds only, and only across waves.
So peak = 1,024 SIMDs x 2.4 GHz / 4 = 6.144e11 VALU wave-instructions/s
(`issue_peak_basis`); a two-wave kernel (the producer/consumer rollouts)
could go up to 2x that on fast-class instructions, which bench.py reports
beside it (`roofline.issue.frac_of_two_wave_fast_peak`).  bench.py's
`roofline.issue.frac` = (VALU wave-instructions per launch, from this file)
/ (the launch's live duration) / peak.
"""
import argparse
import csv
import glob
import json
import os
import re

SIMDS = 1024
CLOCK_HZ = 2.4e9
CYCLES_PER_VALU = 4
ISSUE_PEAK = SIMDS * CLOCK_HZ / CYCLES_PER_VALU  # VALU wave-instructions per second


def per_dispatch(root, kernel):
    """{counter: [per-dispatch value, dispatch order]} of the dispatches whose
    kernel name contains `kernel`; plus their durations (ns, under the
    profiler: longer than unprofiled)."""
    vals, dur = {}, {}
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if kernel not in r.get("Kernel_Name", ""):
                continue
            d = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
            c = r["Counter_Name"]
            vals.setdefault(c, {})
            vals[c][d] = vals[c].get(d, 0.0) + float(r["Counter_Value"])
            dur[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    order = sorted(dur)
    return {c: [v[d] for d in order if d in v] for c, v in vals.items()}, [dur[d] for d in order]


def summarise(root, kernel, envs, plies):
    vals, dur = per_dispatch(root, kernel)
    if len(dur) < 2:
        raise SystemExit(f"too few dispatches of {kernel!r} under {root}: {len(dur)}")
    mean = {c: sum(v[1:]) / len(v[1:]) for c, v in vals.items()}
    valu = mean.get("SQ_INSTS_VALU")
    salu = mean.get("SQ_INSTS_SALU", 0.0)
    wave_cycles = mean.get("SQ_WAVE_CYCLES")
    out = {
        "kernel": kernel, "envs": envs, "plies": plies, "dispatches": len(dur) - 1,
        "counters_per_launch": {c: round(v) for c, v in sorted(mean.items())},
        "valu_per_launch": round(valu) if valu is not None else None,
        "salu_per_launch": round(salu),
        "valu_per_env_ply": round(valu / (envs * plies) * 64, 1) if valu else None,  # per 64-env wave-ply
        "issue_peak_valu_per_s": ISSUE_PEAK,
        "issue_peak_basis": f"{SIMDS} SIMDs x {CLOCK_HZ / 1e9} GHz / {CYCLES_PER_VALU} cycles per VALU wave-instruction "
                            "(one wave's rate, any kind; two waves' rate on the slow kinds: "
                            "profiles/r05/issue_probe/summary.json)",
        "profiled_duration_us": round(sum(dur[1:]) / len(dur[1:]) / 1e3, 2),
    }
    if valu and wave_cycles:
        # quad-cycles: the share of the waves' lifetime spent issuing VALU
        out["valu_busy_of_wave_cycles"] = round(mean.get("SQ_ACTIVE_INST_VALU", valu) / wave_cycles, 4)
        if "SQ_WAIT_ANY" in mean:
            out["wait_of_wave_cycles"] = round(mean["SQ_WAIT_ANY"] / wave_cycles, 4)
    if valu:
        out["frac_at_profiled_duration"] = round(valu / (out["profiled_duration_us"] * 1e-6) / ISSUE_PEAK, 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True, help="the SQ pass's rocprofv3 output dir")
    ap.add_argument("--kernel", required=True, help="kernel name substring, e.g. 'k_rollout_pc<true>'")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--plies", type=int, required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    kname = re.sub(r"\s+", " ", a.kernel)
    out = summarise(a.dir, kname, a.envs, a.plies)
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
