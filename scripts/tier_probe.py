#!/usr/bin/env python3
"""Measurement tool (not product code): the oracle's work per segment on a crop of a scene, for
the caller's tree (collapsed as the library plans it) against the tiered walk (near tree for
segments that start in the near region, the caller's / guarded tree from a path's first other
segment on).  Runs on the CPU (host-only C-ABI calls + the oracle).

  RTX_NEAR_GROW=1 python scripts/tier_probe.py stress_100k --width 1920 --spp 4 --crop 0,0,1920,1080,0,24
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytracer-go_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import oracle_binding as ob  # noqa: E402
import rtx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("scene")
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--spp", type=int, default=4)
ap.add_argument("--crop", default="", help="x0,y0,w,h,rank,world (default: every 24th row)")
ap.add_argument("--flags", type=int, default=0)
args = ap.parse_args()

s = rtx.HostScene(args.scene, 1)
cam = s.camera(width=args.width, spp=args.spp)
W, H = cam.image_width, cam.image_height
reg = rtx.Region(*[int(v) for v in args.crop.split(",")]) if args.crop else rtx.Region(0, 0, W, H, 0, 24)
t0 = time.time()
ref_skip = rtx.node_skip(s.desc, rtx.walk_skip(s.desc, cam, rtx.RTX_SCENE_REFERENCE_BVH))
a, ca = ob.render(s.desc, cam, 2024, reg, ob.ORDER_ITERATIVE, skip=ref_skip)
seg = ca["segments"]
print(f"caller's tree (collapsed): box {ca['node_visits'] / seg:.2f} sphere {ca['prim_tests'] / seg:.2f} "
      f"per segment, {seg} segments, {time.time() - t0:.1f} s")
box, active = rtx.walk_near_region(s.desc, cam, args.flags)
print("near region", box, "active", active)
if box is None:
    sys.exit(0)
near = rtx.walk_near_desc(s.desc, cam, args.flags)
far = rtx.walk_tree_desc(s.desc, cam, args.flags)
far_skip = rtx.node_skip(far, rtx.walk_skip(s.desc, cam, args.flags)) if far is not s.desc else ref_skip
t0 = time.time()
b, cb = ob.render(near, cam, 2024, reg, ob.ORDER_ITERATIVE, tier=(box, far, far_skip), rank=ob.sphere_ranks(s.desc))
print(f"tiered (near tree uncollapsed): box {cb['node_visits'] / seg:.2f} sphere {cb['prim_tests'] / seg:.2f} "
      f"per segment, {time.time() - t0:.1f} s; image equal: {np.array_equal(a, b)}; "
      f"path counters equal: {all(ca[k] == cb[k] for k in ('segments', 'hits', 'rng_draws'))}")
