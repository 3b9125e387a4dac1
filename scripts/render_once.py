"""One timed render of a main.go scene through the C-ABI (for profilers): python scripts/render_once.py
[--scene random_spheres] [--width 1920] [--spp 100] [--no-tier] [--reference-bvh]"""
import argparse
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
ap.add_argument("--no-tier", action="store_true")
ap.add_argument("--reference-bvh", action="store_true")
a = ap.parse_args()
torch.cuda.set_device(0)
s = rtx.HostScene(a.scene, 1)
cam = s.camera(width=a.width, spp=a.spp)
dev = rtx.DeviceScene(s.desc, no_tier=a.no_tier, reference_bvh=a.reference_bvh)
reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
out = torch.empty((cam.image_height, cam.image_width, 3), dtype=torch.float32, device="cuda")
st = dev.render_region(cam, 2024, reg, out.data_ptr(), torch.cuda.current_stream().cuda_stream, timed=True)
print(f"{a.scene} {a.width} {a.spp} layout {st.walk_layout} {st.kernel_ms:.3f} ms deferred {st.deferred_paths}")
