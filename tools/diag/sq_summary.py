#!/usr/bin/env python3
"""Summarise a rocprofv3 SQ-counter pass (counter_collection.csv): per kernel
name, the mean of each counter over its dispatches.  DIAGNOSTIC."""
import collections
import csv
import glob
import re
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(dict))
for path in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "k_rollout" not in k:
            continue
        k = re.search(r"k_rollout\w*<[^>]*>", k).group(0)
        d = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        vals[k][r["Counter_Name"]][d] = vals[k][r["Counter_Name"]].get(d, 0.0) + float(r["Counter_Value"])
for k, cs in vals.items():
    out = {c: round(sum(v.values()) / len(v)) for c, v in sorted(cs.items())}
    print(k, out)
