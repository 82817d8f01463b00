#!/usr/bin/env python3
"""The VALU issue rate of gfx950 on the rules engine's instruction mix
(tools/issue_probe.hip), at 1, 2 and 4 waves per SIMD.

  python3 tools/issue_probe.py --build        # here: the library + the loops' composition
  python3 tools/issue_probe.py --out F.json   # on the box: run, write the summary
  rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
      -- python3 tools/issue_probe.py --iters 2000   # the counter pass

--build also disassembles the probe's device code and records, per kernel,
every instruction of its inner loop (tools/build/issue_probe_loops.json), so
the summary prices exactly what ran: the kind's 32 VALU instructions plus the
loop's own s_add/s_cmp/s_cbranch and any s_nop the compiler put in for
hazards.  Measurement tool, never shipped.
"""
import argparse
import ctypes
import io
import json
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "issue_probe.hip")
BUILD = os.path.join(HERE, "build")
LIB = os.path.join(BUILD, "libissue_probe.so")
LOOPS = os.path.join(BUILD, "issue_probe_loops.json")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950"]


def build():
    os.makedirs(BUILD, exist_ok=True)
    subprocess.check_call([HIPCC, *FLAGS, "-shared", "-fPIC", "-o", LIB, SRC])
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "probe.asm")
        subprocess.check_call([HIPCC, *FLAGS, "--cuda-device-only", "-S", "-o", asm, SRC],
                              stderr=subprocess.DEVNULL)
        text = open(asm).read()
    loops = {}
    for m in re.finditer(r"^(_ZN\S*probe(?:32v|32|64)I\S+):.*?\n(.*?)s_endpgm", text, re.S | re.M):
        kind = re.search(r"INS_\d+(k_\w+?)E", m.group(1)).group(1)
        lm = re.search(r"(\.LBB\d+_\d+):\s*; =>This Inner Loop Header.*?\n(.*?)s_cbranch_scc1 \1", m.group(2), re.S)
        ins = [ln.split()[0] for ln in lm.group(2).splitlines()
               if ln.strip() and not ln.strip().startswith((";", "."))]
        ins.append("s_cbranch_scc1")
        loops[kind] = dict(Counter(ins))
    json.dump(loops, open(LOOPS, "w"), indent=1, sort_keys=True)
    return loops


def run(iters, entry="issue_probe_main"):
    lib = ctypes.CDLL(LIB)
    fn = getattr(lib, entry)
    fn.argtypes = [ctypes.c_int]
    # the library prints one JSON array on its stdout (fd 1): capture it
    r, w = os.pipe()
    saved = os.dup(1)
    sys.stdout.flush()
    os.dup2(w, 1)
    try:
        rc = fn(iters)
    finally:
        os.dup2(saved, 1)
        os.close(w)
        os.close(saved)
    data = io.open(r, "r").read()
    if rc != 0:
        raise SystemExit(f"{entry} failed: {rc}")
    return json.loads(data)


KIND_OF = {  # the probe's printed name -> its kernel's kind struct
    "v_add_u32": "k_add_u32", "v_xor_b32": "k_xor_b32", "v_lshlrev_b32": "k_lshlrev_b32",
    "v_bfe_u32": "k_bfe_u32", "v_bitop3_b32": "k_bitop3_b32", "v_add3_u32": "k_add3_u32",
    "v_cndmask_b32_e64": "k_cndmask_b32", "v_sub_u32_sdwa": "k_sub_u32_sdwa",
    "v_bcnt_u32_b32": "k_bcnt_u32_b32", "v_ffbl_b32": "k_ffbl_b32", "v_perm_b32": "k_perm_b32",
    "v_cmp_eq_u32_e64": "k_cmp_eq_u32", "v_mul_hi_u32": "k_mul_hi_u32", "v_mul_lo_u32": "k_mul_lo_u32",
    "v_fma_f32": "k_fma_f32", "v_mad_u64_u32": "k_mad_u64_u32", "v_lshlrev_b64": "k_lshlrev_b64",
    "v_lshl_add_u64": "k_lshl_add_u64", "v_and_b32": "k_and_b32", "v_or_b32": "k_or_b32",
    "v_sub_u32": "k_sub_u32", "v_mov_b32": "k_mov_b32", "v_lshrrev_b32": "k_lshrrev_b32",
    "v_not_b32": "k_not_b32", "v_min_u32": "k_min_u32", "v_max_i32": "k_max_i32", "v_or3_b32": "k_or3_b32",
    "v_and_or_b32": "k_and_or_b32", "v_lshl_or_b32": "k_lshl_or_b32", "v_cndmask_b32_e32": "k_cndmask_vcc",
    "v_readlane_b32": "k_readlane_b32", "v_add_f32": "k_add_f32", "v_pk_add_u16": "k_pk_add_u16",
    "v_mul_u32_u24": "k_mul_u32_u24", "v_cmp_e32+v_cndmask_e32 (vcc)": "k_cmp_cnd_vcc",
    "v_cmp_e64+v_cndmask_e64 (sgpr)": "k_cmp_cnd_sgpr",
    "v_cndmask_b32_e32 (vcc from a VALU compare)": "k_cndmask_vcc_valu",
    "v_add_u32+s_add_u32": "k_add_sadd", "v_add_u32+s_and_b64": "k_add_sand64", "s_add_u32": "k_sadd_only",
    "v_add_u32+s_cmp+s_cbranch (not taken)": "k_add_cbranch_nt",
    "v_add_u32+s_branch (taken)": "k_add_branch_taken",
}


def summarise(rows, loops):
    out = []
    for r in rows:
        comp = loops.get(KIND_OF[r["kind"]], {})
        trips = r["insts_per_wave"] / 32.0
        nops = comp.get("s_nop", 0)
        # the SIMD's span: its W waves do not all start together at W = 4, so
        # the slowest wave's cycles (first start .. last end ~ the launch) and
        # not the mean measure what the SIMD delivered
        span_trip = r["cycles_per_wave_max"] / trips
        r = dict(r, loop=comp, cycles_per_trip_mean_wave=round(r["cycles_per_wave"] / trips, 2),
                 # the SIMD's cycles per loop trip of ONE of its W waves' worth of work
                 simd_cycles_per_trip=round(span_trip / r["waves_per_simd"], 2),
                 # charging the s_nops at 4 cycles each (one wave's issue slot)
                 # and the scalar loop control at 0, what is left per VALU
                 simd_cycles_per_valu_ex_nop=round((span_trip - 4.0 * nops) / r["waves_per_simd"] / 32.0, 3))
        out.append(r)
    return out


def summarise_sq(csv_path):
    """The counter pass (rocprofv3 --pmc ... -- issue_probe.py) reduced per kind
    and waves per SIMD: SQ_INSTS_VALU, SQ_BUSY_CYCLES (the SQ's busy cycles,
    summed over the chip's SEs) and SQ_WAVE_CYCLES, last dispatch of each."""
    import csv
    from collections import defaultdict
    per = defaultdict(lambda: defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(csv_path)):
        m = re.search(r"::(k_\w+)>", r["Kernel_Name"])
        if not m:
            continue
        key = (m.group(1), int(r["Workgroup_Size"]) // 256, int(r["Dispatch_Id"]))
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[key] = True
    last = {}
    for (kind, w, d) in sorted(per):
        last[(kind, w)] = per[(kind, w, d)]
    out = defaultdict(dict)
    for (kind, w), c in last.items():
        out[kind][str(w)] = {k: int(v) for k, v in sorted(c.items())}
    # busy cycles per VALU instruction, relative to the same kind at one wave per SIMD
    for kind, d in out.items():
        base = d.get("1", {})
        for w, c in d.items():
            if base.get("SQ_BUSY_CYCLES") and c.get("SQ_INSTS_VALU"):
                c["busy_per_valu_vs_1wave"] = round((c["SQ_BUSY_CYCLES"] / c["SQ_INSTS_VALU"])
                                                    / (base["SQ_BUSY_CYCLES"] / base["SQ_INSTS_VALU"]), 3)
    return dict(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--sq-csv", help="summarise a counter pass's sq_counter_collection.csv")
    ap.add_argument("--iters", type=int, default=20000)
    ap.add_argument("--out")
    ap.add_argument("--scalar", action="store_true",
                    help="only the scalar kinds: an SALU instruction, a lane-mask combine, a not-taken and a "
                         "taken branch beside each VALU instruction (cycles per loop trip of 32 pairs)")
    a = ap.parse_args()
    if a.build:
        loops = build()
        print(json.dumps(loops)[:400])
        return
    if a.sq_csv:
        text = json.dumps(summarise_sq(a.sq_csv), indent=1)
        if a.out:
            open(a.out, "w").write(text + "\n")
        print(text)
        return
    loops = json.load(open(LOOPS)) if os.path.exists(LOOPS) else {}
    rows = summarise(run(a.iters, "issue_probe_scalar" if a.scalar else "issue_probe_main"), loops)
    res = {"tool": "tools/issue_probe.hip", "iters": a.iters, "rows": rows}
    one = {r["kind"]: {w: x["simd_cycles_per_trip"] / 32.0 for w in (1, 2, 4)
                       for x in rows if x["kind"] == r["kind"] and x["waves_per_simd"] == w}
           for r in rows}
    res["simd_cycles_per_valu_by_waves"] = {k: {str(w): round(v, 3) for w, v in d.items()} for k, d in one.items()}
    text = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(text + "\n")
    print(json.dumps(res["simd_cycles_per_valu_by_waves"]))


if __name__ == "__main__":
    main()
