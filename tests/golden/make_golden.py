#!/usr/bin/env python3
"""Regenerate the committed golden fixtures (run from the repo root after `make -C oracle`).

- philox4x32_10_kat.json: the published Random123 known-answer vectors for
  Philox4x32-10 (kat_vectors in the Random123 distribution), typed in by hand.
- oracle_random_spheres_48x27x8.{npy,json}: the oracle's render of randSpheres
  (main.go:227-289, scene seed 1) at 48x27, 8 spp, depth 50, render seed 7, in the
  reference colour order, plus its work counters.  This is a regression pin of the
  restatement (the Go reference cannot be run here: parity with it is unpinned).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import numpy as np  # noqa: E402

import oracle_binding as ob  # noqa: E402
import rtx  # noqa: E402

KATS = [
    {"ctr": [0, 0, 0, 0], "key": [0, 0], "out": [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]},
    {"ctr": [0xFFFFFFFF] * 4, "key": [0xFFFFFFFF] * 2, "out": [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]},
    {"ctr": [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], "key": [0xA4093822, 0x299F31D0],
     "out": [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]},
]


def main():
    with open(os.path.join(HERE, "philox4x32_10_kat.json"), "w") as f:
        json.dump(KATS, f, indent=1)
    meta = {"scene": "random_spheres", "scene_seed": 1, "width": 48, "spp": 8, "depth": 50, "render_seed": 7,
            "order": "reference"}
    scene = ob.OracleScene(meta["scene_seed"])
    cam = ob.rand_spheres_camera(meta["width"], meta["spp"], meta["depth"])
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    img, cnt = ob.render(scene.desc, cam, meta["render_seed"], reg, ob.ORDER_REFERENCE, threads=1)
    meta["height"] = cam.image_height
    meta["counters"] = cnt
    np.save(os.path.join(HERE, "oracle_random_spheres_48x27x8.npy"), img)
    with open(os.path.join(HERE, "oracle_random_spheres_48x27x8.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote fixtures:", meta)


if __name__ == "__main__":
    main()
