#!/usr/bin/env python3
"""Whole-frame parity evidence for the BASELINE configs (test infrastructure: runs the oracle).

  python scripts/full_frame_parity.py C2 C4 --out gpurun_out/ffp/ffp.jsonl [--stride C3=8 ...]

Per config: the timed kernel renders the whole frame at the config's own parameters (as bench.py does), and
the oracle (oracle/oracle.c, 16 threads) renders every `stride`-th row of it (stride 1: every pixel) on the
CALLER's tree in the iterative colour order and in the reference's recursive order.  The line records how
many pixels were compared, how many differ from the iterative order (each must then be the walked tree's
oracle value bit for bit: the trapped-path class of DESIGN.md §12), and the largest |delta| against the
reference order (the north-star bar is 1e-4).  The oracle runs in bands of rows, one progress line each.
tests/test_gpu_parity.py::test_config_rows_vs_oracle is the sampled, asserting version of the same check.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "raytracer-go_amd")]

import oracle_binding as ob  # noqa: E402
import rtx  # noqa: E402

CONFIGS = {  # scene, width, spp (BASELINE.json configs)
    "C1": ("random_spheres", 400, 100),
    "C2": ("random_spheres", 1920, 500),
    "C3": ("random_spheres", 1920, 2000),
    "C4": ("stress_100k", 1920, 100),
    "C5": ("earth_dielectric", 3840, 1000),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+", choices=list(CONFIGS))
    ap.add_argument("--out", required=True)
    ap.add_argument("--stride", action="append", default=[], help="NAME=S: every S-th row (default 1)")
    ap.add_argument("--offset", action="append", default=[], help="NAME=O: the first row compared (default 7 %% S)")
    ap.add_argument("--band", type=int, default=64, help="rows per oracle call (a progress line each)")
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()
    strides = {k: int(v) for k, v in (s.split("=") for s in args.stride)}
    offsets = {k: int(v) for k, v in (s.split("=") for s in args.offset)}

    import torch

    from parity import gpu_region, tier_of, walk_of

    torch.cuda.set_device(0)
    for name in args.configs:
        scene, width, spp = CONFIGS[name]
        stride = strides.get(name, 1)
        s = rtx.HostScene(scene, 1)
        dev = rtx.DeviceScene(s.desc)
        cam = s.camera(width=width, spp=spp)
        W, H = cam.image_width, cam.image_height
        t0 = time.time()
        gpu, st = gpu_region(torch, dev, cam, 2024, rtx.Region(0, 0, W, H, 0, 1), counters=False)
        gpu_s = time.time() - t0
        off = offsets.get(name, 7) % stride
        rows = np.arange(off, H, stride)
        want = gpu[rows]
        it = np.empty_like(want)
        ref = np.empty_like(want)
        t1 = time.time()
        band = max(stride, (args.band // stride) * stride)
        for b in range(0, H, band):
            reg = rtx.Region(0, b, W, min(band, H - b), off, stride)
            n = rtx.region_rows(reg)
            if n == 0:
                continue
            k0 = int(np.searchsorted(rows, b + off))
            it[k0:k0 + n], _ = ob.render(s.desc, cam, 2024, reg, ob.ORDER_ITERATIVE, threads=args.threads)
            ref[k0:k0 + n], _ = ob.render(s.desc, cam, 2024, reg, ob.ORDER_REFERENCE, threads=args.threads)
            print(f"{name}: rows {b}..{b + band - 1} done, {time.time() - t1:.0f} s", flush=True)
        oracle_s = time.time() - t1
        bad = np.argwhere((want != it).any(axis=2))
        walked_equal = 0
        if len(bad):  # each must be the walked tree's oracle value (the same check as the row test)
            tier = tier_of(dev, s.desc, cam)
            walk, skip, tw = tier if tier is not None else (*walk_of(dev, s.desc, cam), None)
            rank = ob.sphere_ranks(s.desc)
            for i, x in bad.tolist():
                y = int(rows[i])
                px, _ = ob.render(walk, cam, 2024, rtx.Region(int(x), y, 1, 1, 0, 1), ob.ORDER_ITERATIVE, skip=skip,
                                  tier=tw, rank=rank)
                walked_equal += int(np.array_equal(px[0, 0], want[i, x]))
        line = {
            "config": name, "scene": scene, "width": W, "height": H, "spp": spp, "row_stride": stride, "first_row": off,
            "pixels_compared": int(want.shape[0] * W), "pixels_total": int(W * H),
            "iterative_order_mismatches": int(len(bad)),
            "mismatches_equal_to_walked_tree_oracle": walked_equal,
            "max_abs_delta_vs_iterative": float(np.abs(want - it).max()),
            "max_abs_delta_vs_reference_order": float(np.abs(want - ref).max()),
            "tolerance": 1e-4, "walk_layout": int(st.walk_layout), "sample_chunks": int(st.sample_chunks),
            "gpu_render_s": round(gpu_s, 3), "oracle_s": round(oracle_s, 1), "oracle_threads": args.threads,
            "librtx_sha256_16": _lib_hash(),
        }
        print(json.dumps(line), flush=True)
        with open(args.out, "a") as fh:
            fh.write(json.dumps(line) + "\n")
        dev.close()


def _lib_hash():
    import hashlib

    path = os.environ.get("RTX_LIB") or os.path.join(ROOT, "raytracer-go_amd", "librtx.so")
    return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]


if __name__ == "__main__":
    main()
