#!/usr/bin/env python3
"""Collect scripts/ab.py logs into JSON lines: one line per (log, variant) with its median / min kernel ms and the
image hash.   python scripts/ab_to_jsonl.py <note> <lib-label>=<log> ... > profiles/xxx.jsonl"""
import json
import re
import sys

note = sys.argv[1]
for arg in sys.argv[2:]:
    label, path = arg.split("=", 1)
    text = open(path).read()
    m = re.search(r"image sha256 (\w+)", text)
    for line in text.splitlines():
        v = re.match(r"(\S+)\s+median\s+([\d.]+) ms\s+min\s+([\d.]+).*identical=(\w+)", line)
        if v:
            print(json.dumps({"note": note, "lib": label, "log": path.split("gpurun_out/")[-1], "variant": v.group(1),
                              "median_ms": float(v.group(2)), "min_ms": float(v.group(3)),
                              "image_sha256_16": m.group(1) if m else None, "identical": v.group(4) == "True"}))
