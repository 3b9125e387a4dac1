#!/usr/bin/env python3
"""Cost of the host-buffer boundary: the same render through rtx_render_region_device
(output left in HBM, bench.py's `value`), rtx_render (float32 image copied to the caller's
host buffer over PCIe) and rtx_render_ppm (encoded on the GPU, P3 text copied back).

  python scripts/boundary_rate.py [--width 1920] [--spp 500] [--reps 3]
Prints one JSON line with the median wall time of each path and the Mray/s each implies."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-go_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="random_spheres")
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--spp", type=int, default=500)
ap.add_argument("--depth", type=int, default=50)
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()

torch.cuda.set_device(0)
scene = rtx.HostScene(args.scene, seed=1)
cam = scene.camera(width=args.width, spp=args.spp, depth=args.depth)
W, H = cam.image_width, cam.image_height
dev = rtx.DeviceScene(scene.desc)
reg = rtx.Region(0, 0, W, H, 0, 1)
out = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
segments = dev.render_region(cam, 7, reg, out.data_ptr(), stream, counters=True, timed=True).as_dict()["segments"]


def timed(fn):
    ts = []
    for _ in range(args.reps + 1):  # first run untimed (allocations, code load)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts = sorted(ts[1:])
    return ts[len(ts) // 2]


L = rtx.load()
cap = int(L.rtx_ppm_max_bytes(W, H))
hbuf = np.empty(cap, dtype=np.uint8)
dtext = torch.empty(cap, dtype=torch.uint8, device="cuda")
n = ctypes.c_uint64()


def ppm_c():  # the C-ABI call alone, into a caller-owned host buffer
    rtx.check(L.rtx_render_ppm(dev.handle, ctypes.byref(cam), 7, hbuf.ctypes.data_as(ctypes.c_void_p), cap,
                               ctypes.byref(n), None))


def encode_only():  # rtx_encode_ppm_device on the image already in HBM
    rtx.check(L.rtx_encode_ppm_device(ctypes.c_void_p(out.data_ptr()), W, H, ctypes.c_void_p(dtext.data_ptr()), cap,
                                      ctypes.byref(n), ctypes.c_void_p(stream)))


paths = {
    "device": lambda: dev.render_region(cam, 7, reg, out.data_ptr(), stream),
    "host_f32": lambda: dev.render_host(cam, 7),
    "ppm": lambda: dev.render_ppm(cam, 7),
    "ppm_c_abi": ppm_c,
    "encode_only": encode_only,
}
res = {"workload": f"{args.scene} {W}x{H}x{args.spp}spp depth {args.depth}", "segments": segments}
for name, fn in paths.items():
    s = timed(fn)
    res[name] = {"ms": round(s * 1e3, 3), "mray_s": round(segments / s / 1e6, 1)}
img, _ = dev.render_host(cam, 7)
res["ppm_bytes"] = int(n.value)
res["host_equals_device"] = bool((torch.from_numpy(img) == out.cpu()).all())
print(json.dumps(res), flush=True)
