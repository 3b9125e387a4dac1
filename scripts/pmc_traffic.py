#!/usr/bin/env python3
"""HBM traffic per launch of the bench kernel from rocprofv3 --pmc passes.

  python scripts/pmc_traffic.py <pmc_dir> <out.json> --workload random_spheres:1920x1080x500

Reads FETCH_SIZE and WRITE_SIZE (separate passes, MI355X_MICROARCH.md §HBM) for the
production kernel (render_wave<false, ...>, the non-counting instantiation the timed
steps launch) and writes the per-launch byte count bench.py reports as roofline.traffic.
Units: both counters are KiB (calibrated on this box: a 24,883,200-byte torch fill reads
WRITE_SIZE 24300).  gfx950 correction: FETCH_SIZE counts half the bytes of 16-B-per-lane
reads (the scene copy into LDS is exactly that), so it is doubled.
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("pmc_dir")
ap.add_argument("out")
ap.add_argument("--workload", required=True)
ap.add_argument("--kernel", default="render_items<false,render_drain<",
                help="comma-separated kernel-name substrings (the render's passes; render_drain: near + far, DESIGN.md §21)")
ap.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                              "raytracer-go_amd", "librtx.so"),
                help="the library the profiled run loaded: its hash ties the profile to the code (bench.py checks it)")
ap.add_argument("--renders", type=int, default=0,
                help="renders in the profiled run: every dispatch summed and divided by it (a render of several "
                     "sample chunks dispatches each pass per chunk); 0: the median dispatch of each kernel")
args = ap.parse_args()

# Per counter and kernel, the median over its dispatches; summed over the matching kernels (a
# tiered render launches its near, far and redo passes: DESIGN.md §14).
vals = {"FETCH_SIZE": {}, "WRITE_SIZE": {}}
for f in glob.glob(os.path.join(args.pmc_dir, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if any(k in r["Kernel_Name"] for k in args.kernel.split(",")) and r["Counter_Name"] in vals:
                vals[r["Counter_Name"]].setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
assert vals["FETCH_SIZE"] and vals["WRITE_SIZE"], f"no {args.kernel} rows with FETCH_SIZE/WRITE_SIZE under {args.pmc_dir}"
agg = (lambda v: sum(v) / args.renders) if args.renders else statistics.median
fetch = sum(agg(v) for v in vals["FETCH_SIZE"].values()) * 1024 * 2  # KiB -> B, x2 gfx950
write = sum(agg(v) for v in vals["WRITE_SIZE"].values()) * 1024
out = {
    "workload": args.workload,
    "kernel": args.kernel,
    "launches": {c: {k: len(v) for k, v in d.items()} for c, d in vals.items()},
    "fetch_bytes_per_launch": fetch,
    "write_bytes_per_launch": write,
    "hbm_bytes_per_launch": fetch + write,
    "librtx_sha256_16": hashlib.sha256(open(args.lib, "rb").read()).hexdigest()[:16],
    "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes); "
              "KiB units; FETCH_SIZE x2 (gfx950 16-B/lane read correction)",
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
