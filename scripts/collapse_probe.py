#!/usr/bin/env python3
"""Measurement tool (not product code): box tests per segment when a walk leaves out the box
tests of chosen interior nodes (a collapsed walk), on the oracle's own paths.

A child's box lies inside its parent's and the slab test is monotone in the box, so leaving a
node's test out changes no primitive test and no hit; a left-out node's children are tested
wherever its nearest tested ancestor passes.  With per-node pass counts P from a full walk, a
set K of tested nodes costs sum over X in K of P(nearest tested ancestor of X) box tests.

  python scripts/collapse_probe.py random_spheres 192 4      # the walked tree (rebuilt here)
  python scripts/collapse_probe.py stress_100k 192 2

Reports: the full walk, the optimum for the measured counts (an upper bound on the gain), and
the choice made from surface areas alone (what a builder can do without rendering).
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raytracer-go_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import oracle_binding as ob  # noqa: E402
import rtx  # noqa: E402


def children(desc):
    d = desc.contents
    n = d.n_nodes
    L = np.array([d.nodes[i].left for i in range(n)], np.int64)
    R = np.array([d.nodes[i].right for i in range(n)], np.int64)
    lo = np.array([list(d.nodes[i].bmin) for i in range(n)], np.float64)
    hi = np.array([list(d.nodes[i].bmax) for i in range(n)], np.float64)
    return L, R, lo, hi, int(d.roots[0])


def area(lo, hi):
    e = np.maximum(hi - lo, 0.0)
    return e[:, 0] * e[:, 1] + e[:, 1] * e[:, 2] + e[:, 2] * e[:, 0]


def choose(L, R, root, P, root_count):
    """Tested set minimising sum_{X in K} P(nearest tested ancestor); a node may be left out
    only when both its children are nodes.  Returns (cost, skip mask)."""
    n = len(L)
    order, parent, stack = [], np.full(n, -1, np.int64), [root]
    while stack:  # pre-order
        x = stack.pop()
        order.append(x)
        for c in (L[x], R[x]) if L[x] != R[x] else (L[x],):
            if c >= 0:
                parent[c] = x
                stack.append(c)
    depth = np.zeros(n, np.int64)
    for x in order:
        if parent[x] >= 0:
            depth[x] = depth[parent[x]] + 1
    # cost[x][j]: cost of x's subtree when its nearest tested ancestor is at depth j - 1
    # (j = 0: none, the walk's start, count root_count); ancestors of x are its depth-prefix
    cost, keep = {}, {}
    anc_count = {}
    for x in reversed(order):
        kids = [c for c in ((L[x], R[x]) if L[x] != R[x] else (L[x],)) if c >= 0]
        collapsible = L[x] >= 0 and R[x] >= 0 and L[x] != R[x]
        d = depth[x]
        # counts of the possible nearest tested ancestors: index j in 0..d
        chain, y = [], parent[x]
        while y >= 0:
            chain.append(P[y])
            y = parent[y]
        counts = [root_count] + chain[::-1]  # j = 0 .. d
        anc_count[x] = counts
        k_keep = sum(cost[c][d + 1] for c in kids)  # children's nearest tested ancestor = x
        arr_c, arr_k = [], []
        for j in range(d + 1):
            c_keep = counts[j] + k_keep
            if collapsible:
                c_drop = sum(cost[c][j] for c in kids)
                if c_drop < c_keep:
                    arr_c.append(c_drop)
                    arr_k.append(False)
                    continue
            arr_c.append(c_keep)
            arr_k.append(True)
        cost[x], keep[x] = arr_c, arr_k
        for c in kids:  # children's tables are no longer needed beyond the decisions
            pass
    # decisions top-down
    skip = np.zeros(n, np.uint8)
    stack = [(root, 0)]
    while stack:
        x, j = stack.pop()
        k = keep[x][j]
        if not k:
            skip[x] = 1
        nj = depth[x] + 1 if k else j
        for c in (L[x], R[x]) if L[x] != R[x] else (L[x],):
            if c >= 0:
                stack.append((c, nj))
    return cost[root][0], skip


def run(desc, cam, threads=8, skip=None):
    L = ob.load()
    n = desc.contents.n_nodes
    tested = np.zeros(n, np.uint64)
    passed = np.zeros(n, np.uint64)
    sk = None if skip is None else np.ascontiguousarray(skip, np.uint8)
    L.oracle_node_hooks.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.oracle_node_hooks(tested.ctypes.data, passed.ctypes.data, None if sk is None else sk.ctypes.data)
    try:
        reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
        img, c = ob.render(desc, cam, 7, reg, ob.ORDER_ITERATIVE, threads)
    finally:
        L.oracle_node_hooks(None, None, None)
    return img, c, tested, passed


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "random_spheres"
    width = int(sys.argv[2]) if len(sys.argv) > 2 else 192
    spp = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    s = rtx.HostScene(scene, 1)
    cam = s.camera(width=width, spp=spp)
    desc = rtx.walk_tree_desc(s.desc, cam)
    which = "rebuilt" if desc.contents.n_nodes != s.desc.contents.n_nodes or rtx.camera_octant(cam) and False else "walked"
    img, c, tested, passed = run(desc, cam)
    seg = c["segments"]
    L, R, lo, hi, root = children(desc)
    P = passed.astype(np.float64)
    full = tested.sum()
    print(f"{scene} {cam.image_width}x{cam.image_height}x{spp} ({which} tree, {len(L)} nodes): {seg} segments")
    print(f"  full walk      : box {full / seg:.2f} per segment")
    opt, skip_opt = choose(L, R, root, P, float(tested[root]))
    print(f"  optimum (meas.) : box {opt / seg:.2f} per segment, {int(skip_opt.sum())} nodes left out")
    A = area(lo, hi)
    est = float(tested[root]) * A / A[root]
    _, skip_sa = choose(L, R, root, est, float(tested[root]))
    img2, c2, t2, _ = run(desc, cam, skip=skip_sa)
    same = np.array_equal(img, img2) and all(c[k] == c2[k] for k in ("segments", "hits", "rng_draws", "prim_tests"))
    print(f"  surface areas   : box {t2.sum() / seg:.2f} per segment, {int(skip_sa.sum())} nodes left out; "
          f"image and primitive tests identical: {same}")
    if os.environ.get("SAMPLE"):  # counts measured on a small sample of the same camera
        sw, sspp = (int(x) for x in os.environ["SAMPLE"].split(","))
        scam = s.camera(width=sw, spp=sspp)
        _, sc, st, sp = run(desc, scam)
        _, skip_s = choose(L, R, root, sp.astype(np.float64), float(st[root]))
        _, _, t4, _ = run(desc, cam, skip=skip_s)
        print(f"  sample {sw}x{sspp} : box {t4.sum() / seg:.2f} per segment ({sc['segments']} sample segments)")
    img3, c3, t3, _ = run(desc, cam, skip=skip_opt)
    same = np.array_equal(img, img3) and all(c[k] == c3[k] for k in ("segments", "hits", "rng_draws", "prim_tests"))
    print(f"  optimum, walked : box {t3.sum() / seg:.2f} per segment; identical: {same}")


if __name__ == "__main__":
    main()
