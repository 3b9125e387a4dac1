#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per kernel name, the mean of each counter over its
dispatches and the sum over them.  python scripts/pmc_summary.py gpurun_out/pmc"""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"].replace("(rtxd::Params)", "").replace("void rtxd::", "")
        if not any(k in name for k in ("render", "trace_paths", "shade_paths", "reduce")):
            continue
        key = (row["Dispatch_Id"], f)
        vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for name, cs in vals.items():
    print(name)
    for c in sorted(cs):
        v = cs[c]
        print(f"   {c:24s} {sum(v) / len(v):16.4g}  sum {sum(v):14.4g}  (n={len(v)})")
