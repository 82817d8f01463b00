#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into profiles/pmc_k_rollout.json.

Reads the *_counter_collection.csv of a FETCH_SIZE pass and a WRITE_SIZE pass
(separate runs, MI355X_MICROARCH.md "rocprofv3 PMC slots": they do not fit
one pass), keeps the dispatches of the named kernel, drops the first
(warm-up) one and averages.  Units: FETCH_SIZE/WRITE_SIZE are KiB.
gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the
bytes of a 16-B/lane coalesced read stream -- the only reads of k_rollout are
the 16-B/lane record loads -- so fetch bytes = 2 x FETCH_SIZE x 1024.
WRITE_SIZE is exact for 16-B/lane streaming stores; the narrower output
stores (reward/flags/actions) are uncalibrated (< 12 % of the bytes).
"""
import argparse
import csv
import glob
import json
import os


def per_dispatch(path_glob, kernel, counter):
    vals = {}
    for path in glob.glob(path_glob, recursive=True):
        for row in csv.DictReader(open(path)):
            if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                key = int(row.get("Dispatch_Id") or row.get("Correlation_Id") or len(vals))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True, help="dir of the FETCH_SIZE pass")
    ap.add_argument("--write", required=True, help="dir of the WRITE_SIZE pass")
    ap.add_argument("--kernel", default="k_rollout_pc<true>")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--plies", type=int, default=1000)
    ap.add_argument("--bytes-per-ply", type=int, default=114, help="114 REF2, 118 FULL4")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                  "pmc_k_rollout.json"))
    a = ap.parse_args()
    f = per_dispatch(os.path.join(a.fetch, "**", "*counter_collection.csv"), a.kernel, "FETCH_SIZE")
    w = per_dispatch(os.path.join(a.write, "**", "*counter_collection.csv"), a.kernel, "WRITE_SIZE")
    if len(f) < 2 or len(w) < 2:
        raise SystemExit(f"too few dispatches: fetch {len(f)} write {len(w)}")
    f, w = f[1:], w[1:]
    fetch_kib = sum(f) / len(f)
    write_kib = sum(w) / len(w)
    algo = a.envs * (a.bytes_per_ply * a.plies + 64)
    hbm = (2 * fetch_kib + write_kib) * 1024
    out = {
        "kernel": a.kernel, "envs": a.envs, "plies": a.plies, "dispatches": len(f),
        "FETCH_SIZE_KiB": round(fetch_kib, 1), "WRITE_SIZE_KiB": round(write_kib, 1),
        "fetch_bytes_per_launch": round(2 * fetch_kib * 1024), "write_bytes_per_launch": round(write_kib * 1024),
        "hbm_bytes_per_launch": round(hbm), "algorithmic_bytes_per_launch": algo,
        "traffic_over_algorithmic": round(hbm / algo, 4),
        "correction": "fetch = 2 x FETCH_SIZE (gfx950, 16-B/lane stream); write = WRITE_SIZE",
    }
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
