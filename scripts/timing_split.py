#!/usr/bin/env python3
"""GPU diagnostics: where the TIMED kernel's wave cycles go (RTX_FLAG_TIMING: the asm-walk kernel
with s_memtime splits), against the plain timed kernel's time.

  python scripts/timing_split.py [--scene random_spheres] [--width 1920] [--spp 100]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytracer-go_amd")]

import torch  # noqa: E402

import rtx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="random_spheres")
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--spp", type=int, default=100)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--no-tier", action="store_true", help="the guarded walk alone (RTX_SCENE_NO_TIER)")
a = ap.parse_args()
torch.cuda.set_device(0)
s = rtx.HostScene(a.scene, 1)
cam = s.camera(width=a.width, spp=a.spp)
dev = rtx.DeviceScene(s.desc, no_tier=a.no_tier)
reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
out = torch.empty((cam.image_height, cam.image_width, 3), dtype=torch.float32, device="cuda")
st = torch.cuda.current_stream().cuda_stream


def run(flags):
    best = None
    for _ in range(a.reps):
        x = dev.render_region(cam, 2024, reg, out.data_ptr(), st, timed=True, flags=flags)
        best = x if best is None or x.kernel_ms < best.kernel_ms else best
    return best


plain = run(0)
t = run(rtx.RTX_FLAG_TIMING)
cyc = t.trav_cycles + t.shade_cycles
res = {"scene": a.scene, "width": a.width, "spp": a.spp, "walk_layout": plain.walk_layout,
       "timed_ms": round(plain.kernel_ms, 3), "wave_gcycles": {"walk": round(t.trav_cycles / 1e9, 3),
       "shade": round(t.shade_cycles / 1e9, 3), "split": [round(v / 1e9, 3) for v in t.shade_split_cycles]},
       "timing_variant_ms": round(t.kernel_ms, 3),
       "walk_share": round(t.trav_cycles / cyc, 4), "shade_share": round(t.shade_cycles / cyc, 4),
       "split": {k: round(v / cyc, 4) for k, v in zip(("scatter", "shade", "claim_camera", "begin"), t.shade_split_cycles)}}
print(json.dumps(res), flush=True)
