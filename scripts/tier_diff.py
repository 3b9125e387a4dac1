"""Whole-frame A/B of the tiered walk against the guarded tree alone and the
caller's tree, on the GPU: which pixels differ (coordinates and values to JSON), and the kernel
times.  usage: python scripts/tier_diff.py SCENE WIDTH SPP OUT.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytracer-go_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtx  # noqa: E402
from parity import gpu_region  # noqa: E402

scene, width, spp, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
torch.cuda.set_device(0)
s = rtx.HostScene(scene, 1)
cam = s.camera(width=width, spp=spp)
reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
imgs, res = {}, {"scene": scene, "width": width, "spp": spp}
for name, kw in (("tiered", {}), ("guarded", {"no_tier": True}), ("reference", {"reference_bvh": True})):
    dev = rtx.DeviceScene(s.desc, **kw)
    img, st = gpu_region(torch, dev, cam, 2024, reg, counters=False)
    img2, st2 = gpu_region(torch, dev, cam, 2024, reg, counters=False)
    assert np.array_equal(img, img2), name
    imgs[name] = img
    res[name] = {"kernel_ms": [round(st.kernel_ms, 3), round(st2.kernel_ms, 3)], "walk_layout": st.walk_layout,
                 "deferred_paths": st.deferred_paths, "redo_chunks": st.redo_chunks}
    del dev
for a, b in (("tiered", "reference"), ("guarded", "reference"), ("tiered", "guarded")):
    d = np.argwhere((imgs[a] != imgs[b]).any(axis=2))
    res[f"{a}_vs_{b}"] = {"n": len(d), "max": float(np.abs(imgs[a] - imgs[b]).max()),
                          "pixels": [[int(y), int(x), imgs[a][y, x].tolist(), imgs[b][y, x].tolist()]
                                     for y, x in d[:64]]}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: (v if not isinstance(v, dict) or "pixels" not in v else {"n": v["n"], "max": v["max"]})
                  for k, v in res.items()}))
