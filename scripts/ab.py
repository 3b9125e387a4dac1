#!/usr/bin/env python3
"""A/B kernel variants on one device, interleaved rounds in one process (guide §5.4 rule 24).

  python scripts/ab.py [--width 1920] [--spp 100] [--rounds 3] [--variants v3,nolds,t40]
  (RTX_LIB=path selects another build of librtx.so: scripts/gpu_ab_libs.sh)
Checks that every variant's image is bit-identical to the first one."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-go_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtx  # noqa: E402

VARIANTS = {"v3": 0, "nolds": rtx.RTX_FLAG_NO_LDS}
for _t in range(1, 65):
    VARIANTS[f"t{_t}"] = rtx.RTX_FLAG_SHADE_THRESH(_t)

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="random_spheres")
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--spp", type=int, default=100)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--depth", type=int, default=0, help="max depth (0: the scene's)")
ap.add_argument("--variants", default="v3,nolds")
args = ap.parse_args()

torch.cuda.set_device(0)
scene = rtx.HostScene(args.scene, 1)
cam = scene.camera(width=args.width, spp=args.spp, depth=args.depth)
dev = rtx.DeviceScene(scene.desc)
reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
names = args.variants.split(",")
for n in names:  # "a+b" = the flags of a and b together
    if "+" in n:
        VARIANTS[n] = 0
        for part in n.split("+"):
            VARIANTS[n] |= VARIANTS[part]
ENV = {}  # "name@K=V;K2=V2": the flags of name with those environment knobs (read per render)
for n in names:
    if "@" in n:
        base, kv = n.split("@", 1)
        VARIANTS[n] = VARIANTS[base]
        ENV[n] = dict(x.split("=", 1) for x in kv.split(";"))
KNOBS = sorted({k for e in ENV.values() for k in e})


def setenv(n):
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update(ENV.get(n, {}))


outs = {n: torch.zeros((cam.image_height, cam.image_width, 3), device="cuda") for n in names}
stream = torch.cuda.current_stream().cuda_stream
st = dev.render_region(cam, 1, reg, outs[names[0]].data_ptr(), stream, counters=True, timed=True)
times = {n: [] for n in names}
for rnd in range(args.rounds + 1):
    for n in names:
        setenv(n)
        s = dev.render_region(cam, 1, reg, outs[n].data_ptr(), stream, timed=True, flags=VARIANTS[n])
        if rnd > 0:
            times[n].append(s.kernel_ms)
ref = outs[names[0]].cpu().numpy()
import hashlib  # noqa: E402
print(f"image sha256 {hashlib.sha256(np.ascontiguousarray(ref).tobytes()).hexdigest()[:16]} (compare across builds)",
      flush=True)
for n in names:
    same = np.array_equal(ref, outs[n].cpu().numpy())
    med = float(np.median(times[n]))
    print(f"{n:8s} median {med:9.2f} ms  min {min(times[n]):9.2f}  Gsamples/s {st.samples / med / 1e6:7.3f}  "
          f"Mray/s {st.segments / med / 1e3:9.1f}  identical={same}", flush=True)
# scheduling counters of each variant (a separate counting launch)
setenv("")
for n in names:
    c = dev.render_region(cam, 1, reg, outs[n].data_ptr(), stream, counters=True, timed=True, flags=VARIANTS[n])
    if c.cache_hits:
        print(f"{n:8s} LDS-cache hits {c.cache_hits / (c.node_visits + c.prim_tests):.3f} of the entries read "
              f"(node visits + primitive tests {(c.node_visits + c.prim_tests) / c.segments:.1f} per segment)", flush=True)
    if c.wave_iters:
        print(f"{n:8s} trav-lane util {c.lane_steps / (64 * c.wave_iters):.3f}  iters/segment(wave) "
              f"{c.wave_iters * 64 / c.segments:.1f}  entries/segment {(c.node_visits + c.prim_tests) / c.segments:.1f}"
              f"  shade lanes/phase {c.shade_lanes / max(c.shade_phases, 1):.1f}  phases/wave-iter "
              f"{c.shade_phases / c.wave_iters:.3f}  shade share {c.shade_cycles / max(c.trav_cycles + c.shade_cycles, 1):.3f}"
              f"  cyc/iter {c.trav_cycles / c.wave_iters:.0f}  cyc/shade {c.shade_cycles / max(c.shade_phases, 1):.0f}"
              f"  idle-lane frac {c.idle_lanes / (64 * c.wave_iters):.3f}"
              f"  parked {c.parked_lanes / (64 * c.wave_iters):.3f}  deferred {c.deferred_lanes / (64 * c.wave_iters):.3f}"
              f"  shade split (scatter/shade/claim/begin) "
              + "/".join(f"{x / max(c.shade_cycles, 1):.3f}" for x in c.shade_split_cycles),
              flush=True)
