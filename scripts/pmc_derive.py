#!/usr/bin/env python3
"""Derived ratios of one kernel from the rocprofv3 --pmc passes of scripts/gpu_pmc.sh.

  python scripts/pmc_derive.py <pmc_dir> --workload NAME [--kernel render_items<false] [--out x.json]

VALU issue = 2 cycles x SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs); lane use =
SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU); waits = SQ_WAIT_ANY / SQ_WAVE_CYCLES (s_waitcnt:
LDS or memory results outstanding); LDS conflicts = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;
L2 hit rate = TCC_HIT / (TCC_HIT + TCC_MISS); HBM-side bytes = FETCH_SIZE x 2 (gfx950 16-B/lane
read correction) + WRITE_SIZE, KiB units (MI355X_MICROARCH.md, HBM/rocprofv3 section).
"""
import argparse
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("pmc_dir")
ap.add_argument("--workload", required=True)
ap.add_argument("--kernel", default="render_items<false,render_drain<",
                help="comma-separated kernel-name substrings (the render's passes; render_drain: near + far, DESIGN.md §21)")
ap.add_argument("--out")
args = ap.parse_args()

v = {}
for f in glob.glob(os.path.join(args.pmc_dir, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if any(k in r["Kernel_Name"] for k in args.kernel.split(",")):
                v.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
c = {k: sum(x) / len(x) for k, x in v.items()}  # mean over the passes' launches
kname = None
for f in glob.glob(os.path.join(args.pmc_dir, "**", "*kernel_trace.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if any(k in r["Kernel_Name"] for k in args.kernel.split(",")):
                kname = r["Kernel_Name"]
clk = c["GRBM_GUI_ACTIVE"] / 8.0
out = {
    "workload": args.workload,
    "kernel": kname,
    "shader_cycles": clk,
    "valu_issue_frac": round(2.0 * c["SQ_INSTS_VALU"] / (clk * 1024), 4),
    "valu_lane_frac": round(c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_INSTS_VALU"]), 4),
    "salu_per_valu": round(c["SQ_INSTS_SALU"] / c["SQ_INSTS_VALU"], 4),
    "wait_frac": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4),
    "issue_stall_frac": round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4),
    "lds_conflict_frac": round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4),
    "l2_hit_frac": round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4),
    "l2_requests": c["TCC_HIT_sum"] + c["TCC_MISS_sum"],
    "hbm_fetch_bytes": 2048.0 * c["FETCH_SIZE"],
    "hbm_write_bytes": 1024.0 * c["WRITE_SIZE"],
    "counters": {k: c[k] for k in sorted(c)},
}
print(json.dumps(out, indent=1))
if args.out:
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
