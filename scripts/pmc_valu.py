#!/usr/bin/env python3
"""VALU issue utilisation of the bench kernel from rocprofv3 --pmc passes.

  python scripts/pmc_valu.py <pmc_dir> <out.json> --workload random_spheres:1920x1080x500

The render is VALU-issue bound, so this is its meaningful roofline:
SQ_INSTS_VALU wave64 instructions x 2 issue cycles each per SIMD, over the SIMD-cycles of
the launch (GRBM_GUI_ACTIVE is summed over the 8 XCDs: / 8 = shader clocks; x 1024 SIMDs).
"""
import argparse
import csv
import glob
import hashlib
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("pmc_dir")
ap.add_argument("out")
ap.add_argument("--workload", required=True)
ap.add_argument("--kernel", default="render_items<false,render_drain<",
                help="comma-separated kernel-name substrings (the render's passes; render_drain: near + far, DESIGN.md §21)")
ap.add_argument("--simds", type=int, default=1024)
ap.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                              "raytracer-go_amd", "librtx.so"),
                help="the library the profiled run loaded: its hash ties the profile to the code (bench.py checks it)")
ap.add_argument("--renders", type=int, default=0,
                help="renders in the profiled run (bench.py --steps 1 --warmup 0: 1); every dispatch of the "
                     "matching kernels (each pass of each sample chunk) is summed and divided by it.  0: the "
                     "dispatches of one kernel (a one-chunk render)")
args = ap.parse_args()

# Per counter: the sum over every dispatch of the matching kernels (a tiered render launches its
# near, far and redo passes: DESIGN.md §14), divided by the renders (the dispatches of each kernel).
# All from the one pass that holds every counter needed (GRBM_GUI_ACTIVE is in other passes too).
need = ["SQ_INSTS_VALU", "GRBM_GUI_ACTIVE", "SQ_THREAD_CYCLES_VALU"]
vals, disp = {}, {}
for f in sorted(glob.glob(os.path.join(args.pmc_dir, "**", "*counter_collection.csv"), recursive=True)):
    with open(f) as fh:
        rows = [r for r in csv.DictReader(fh) if any(k in r["Kernel_Name"] for k in args.kernel.split(","))]
    if not all(any(r["Counter_Name"] == k for r in rows) for k in need):
        continue
    for r in rows:
        vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        disp.setdefault((f, r["Counter_Name"], r["Kernel_Name"]), set()).add(r.get("Dispatch_Id", ""))
    break
assert all(k in vals for k in need), f"missing {need} for {args.kernel} under {args.pmc_dir}"
renders = {c: args.renders or max(len(d) for (f, cc, k), d in disp.items() if cc == c) for c in need}
insts = vals["SQ_INSTS_VALU"] / renders["SQ_INSTS_VALU"]
cycles = vals["GRBM_GUI_ACTIVE"] / renders["GRBM_GUI_ACTIVE"] / 8.0
thread_cycles = vals["SQ_THREAD_CYCLES_VALU"] / renders["SQ_THREAD_CYCLES_VALU"]
out = {
    "workload": args.workload,
    "kernel": args.kernel,
    "valu_insts_per_launch": insts,
    "shader_cycles_per_launch": cycles,
    "valu_issue_frac": round(insts * 2.0 / (cycles * args.simds), 4),
    "valu_lane_frac": round(thread_cycles / (64.0 * insts), 4),
    "kernels": sorted({k for (f, c, k) in disp}),
    "librtx_sha256_16": hashlib.sha256(open(args.lib, "rb").read()).hexdigest()[:16],
    # every counter of the pass per launch (SQ_INSTS_SALU, SQ_WAIT_ANY, SQ_WAVE_CYCLES, ... when collected)
    "counters_per_launch": {c: v / (args.renders or renders["SQ_INSTS_VALU"]) for c, v in sorted(vals.items())},
    "method": "rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE ...; "
              "issue frac = 2 cycles x SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)",
}
if args.out.endswith(".jsonl"):  # one line per (workload, library): replace this one's, keep the others
    keep = []
    if os.path.exists(args.out):
        with open(args.out) as fh:
            keep = [ln for ln in fh.read().splitlines() if ln.strip() and
                    (json.loads(ln).get("workload"), json.loads(ln).get("librtx_sha256_16")) !=
                    (out["workload"], out["librtx_sha256_16"])]
    with open(args.out, "w") as fh:
        fh.write("\n".join(keep + [json.dumps(out)]) + "\n")
else:
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
print(json.dumps(out))
