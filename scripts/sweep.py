"""GPU A/B sweep of the runtime knobs of the timed kernel in one process (best of --reps renders):
shading threshold (RTX_FLAG_SHADE_THRESH), primitive batch (RTX_PRIM_BATCH), samples per unit
(RTX_ITEM_SUB), tiered or not.  python scripts/sweep.py [--spp 100] [--scene random_spheres]"""
import argparse
import itertools
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
ap.add_argument("--thresh", default="48")
ap.add_argument("--batch", default="16")
ap.add_argument("--sub", default="0")
ap.add_argument("--tier", default="1,0")
ap.add_argument("--grow", default="25", help="RTX_NEAR_GROW values (percent) for the tiered scenes")
a = ap.parse_args()
torch.cuda.set_device(0)
s = rtx.HostScene(a.scene, 1)
cam = s.camera(width=a.width, spp=a.spp)
reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
out = torch.empty((cam.image_height, cam.image_width, 3), dtype=torch.float32, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
devs = {}
for t in map(int, a.tier.split(",")):
    for g in (a.grow.split(",") if t else ["-"]):
        if g != "-":
            os.environ["RTX_NEAR_GROW"] = g
        devs[(t, g)] = rtx.DeviceScene(s.desc, no_tier=(t == 0))
for (t, g), th, pb, sub in itertools.product(devs, a.thresh.split(","), a.batch.split(","), a.sub.split(",")):
    os.environ["RTX_PRIM_BATCH"] = pb
    os.environ["RTX_ITEM_SUB"] = sub
    ms = []
    for _ in range(a.reps):
        st = devs[(t, g)].render_region(cam, 2024, reg, out.data_ptr(), stream, timed=True,
                                   flags=rtx.RTX_FLAG_SHADE_THRESH(int(th)))
        ms.append(st.kernel_ms)
    print(json.dumps({"tier": t, "grow": g, "deferred": st.deferred_paths, "thresh": int(th), "batch": int(pb), "sub": int(sub), "ms": round(min(ms), 3),
                      "all": [round(x, 3) for x in ms]}), flush=True)
