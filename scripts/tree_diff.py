#!/usr/bin/env python3
"""GPU: whole frames of a BASELINE config rendered over the reference tree and over a rebuilt tree
(RTX_BVH=guarded / sah), compared pixel by pixel; prints one JSON line per (config, mode).

  python scripts/tree_diff.py [C2 C3 C4 C5] [--modes guarded sah]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytracer-go_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtx  # noqa: E402

CONFIGS = {"C2": ("random_spheres", 1920, 500), "C3": ("random_spheres", 1920, 2000),
           "C4": ("stress_100k", 1920, 100), "C5": ("earth_dielectric", 3840, 1000)}


def render(desc, cam, mode):
    if mode == "reference":
        os.environ["RTX_BVH"] = "reference"
    else:
        os.environ["RTX_BVH"] = mode
    dev = rtx.DeviceScene(desc)
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    out = torch.empty((cam.image_height, cam.image_width, 3), dtype=torch.float32, device="cuda")
    s = dev.render_region(cam, 2024, reg, out.data_ptr(), torch.cuda.current_stream().cuda_stream, timed=True)
    s2 = dev.render_region(cam, 2024, reg, out.data_ptr(), torch.cuda.current_stream().cuda_stream, timed=True)
    torch.cuda.synchronize()
    img = out.cpu().numpy()
    dev.close()
    return img, min(s.kernel_ms, s2.kernel_ms), s2.walk_layout


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["C2", "C5"])
    ap.add_argument("--modes", nargs="*", default=["guarded", "sah"])
    a = ap.parse_args()
    torch.cuda.set_device(0)
    for c in a.configs:
        scene, width, spp = CONFIGS[c]
        s = rtx.HostScene(scene, 1)
        cam = s.camera(width=width, spp=spp)
        ref, ref_ms, _ = render(s.desc, cam, "reference")
        for m in a.modes:
            t0 = time.time()
            img, ms, lay = render(s.desc, cam, m)
            d = np.abs(img - ref)
            px = np.argwhere((img != ref).any(axis=2))
            print(json.dumps({"config": c, "mode": m, "walk_layout": int(lay), "kernel_ms": round(ms, 3),
                              "reference_ms": round(ref_ms, 3), "pixels_differ": int(len(px)),
                              "pixels_over_1e-4": int((d.max(axis=2) > 1e-4).sum()), "max_abs_diff": float(d.max()),
                              "first": px[:6].tolist()}), flush=True)


if __name__ == "__main__":
    main()
