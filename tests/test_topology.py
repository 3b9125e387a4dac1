"""The walk's own tree (rtx_topology.h) on the CPU: rtx_walk_tree builds it without a device.

The library walks a sphere scene's BVH over a rebuilt tree: the reference's leaf nodes (one or two
spheres, bvh.go:162-174) kept as they are, under a binned-SAH tree of unions of their boxes, each
node's near child first along the camera's viewing direction.  These tests pin the tree's shape
(every reference leaf once, boxes that contain their children, the same tree for every octant up
to child order), the scene policy, and — on the oracle — that walking it changes no path: the
image, segments, hits and draws equal the reference tree's, bit for bit.
"""
import ctypes

import numpy as np
import pytest

import oracle_binding as ob
import rtx


def walk_tree(desc, octant=0, flags=0):
    L = rtx.load()
    n, root = ctypes.c_uint32(), ctypes.c_int32()
    rtx.check(L.rtx_walk_tree(desc, flags, octant, None, 0, ctypes.byref(n), ctypes.byref(root)), "rtx_walk_tree")
    if n.value == 0:
        return None, root.value
    arr = (rtx.BvhNode * n.value)()
    rtx.check(L.rtx_walk_tree(desc, flags, octant, arr, n.value, ctypes.byref(n), ctypes.byref(root)), "rtx_walk_tree")
    return arr, root.value


def ref_leaves(desc):
    """The reference tree's leaf nodes (both children spheres), as (box, children) keys."""
    d = desc.contents
    out = []
    for i in range(d.n_nodes):
        nd = d.nodes[i]
        if nd.left < 0 and nd.right < 0:
            out.append((tuple(nd.bmin), tuple(nd.bmax), nd.left, nd.right))
    return sorted(out)


@pytest.mark.parametrize("scene", ["random_spheres", "earth_dielectric"])
def test_walk_tree_shape(built, scene):
    s = rtx.HostScene(scene, 1)
    desc = s.desc
    leaves = ref_leaves(desc)
    shapes = []
    for octant in range(8):
        arr, root = walk_tree(desc, octant)
        assert arr is not None and root == 0
        n = len(arr)
        internal = n - len(leaves)
        assert internal == len(leaves) - 1  # a binary tree over the reference's leaves
        # the unit nodes are the reference's leaves, unchanged
        units = sorted((tuple(arr[i].bmin), tuple(arr[i].bmax), arr[i].left, arr[i].right) for i in range(internal, n))
        assert units == leaves
        # every SAH node's box contains its children's; every node is reached once from the root
        seen = np.zeros(n, np.int32)
        stack = [root]
        while stack:
            i = stack.pop()
            seen[i] += 1
            if i >= internal:
                continue
            for c in (arr[i].left, arr[i].right):
                assert c >= 0
                for k in range(3):
                    assert arr[i].bmin[k] <= arr[c].bmin[k] and arr[i].bmax[k] >= arr[c].bmax[k]
                stack.append(c)
        assert (seen == 1).all()
        shapes.append(sorted((tuple(arr[i].bmin), tuple(arr[i].bmax), tuple(sorted((arr[i].left, arr[i].right))))
                             for i in range(n)))
    assert all(sh == shapes[0] for sh in shapes)  # octants differ only in child order


def test_octant_order_is_near_first(built):
    """The main.go camera (LookFrom (13,2,3), LookAt the origin) looks along -x, -y, -z: octant 7.
    Octant 7's tree is octant 0's with the children of every SAH node swapped (the high side of
    every split first); the reference's leaf nodes keep their order."""
    s = rtx.HostScene("random_spheres", 1)
    cam = s.camera(width=96, spp=1)
    assert rtx.camera_octant(cam) == 7
    a0, _ = walk_tree(s.desc, 0)
    a7, _ = walk_tree(s.desc, 7)
    internal = len(a0) - len(ref_leaves(s.desc))
    for i in range(len(a0)):
        if i < internal:
            assert (a0[i].left, a0[i].right) == (a7[i].right, a7[i].left)
        else:
            assert (a0[i].left, a0[i].right) == (a7[i].left, a7[i].right)


def test_policy(built, monkeypatch):
    # quads: kept
    assert walk_tree(rtx.HostScene("cornell_box", 1).desc)[0] is None
    # config 4: the precision gate keeps the reference tree (eps D^2 / r^2 = 0.3) ...
    c4 = rtx.HostScene("stress_100k", 1)
    assert walk_tree(c4.desc)[0] is None
    # ... unless forced
    monkeypatch.setenv("RTX_BVH", "guarded")
    assert walk_tree(c4.desc)[0] is not None
    monkeypatch.delenv("RTX_BVH")
    rs = rtx.HostScene("random_spheres", 1)
    assert walk_tree(rs.desc)[0] is not None
    assert walk_tree(rs.desc, flags=rtx.RTX_SCENE_REFERENCE_BVH)[0] is None
    monkeypatch.setenv("RTX_BVH", "reference")
    assert walk_tree(rs.desc)[0] is None
    monkeypatch.delenv("RTX_BVH")
    # a World root (linear scan, hittables.go:55-72): kept
    d = rs.desc.contents
    n = d.n_spheres
    roots = (ctypes.c_int32 * n)(*[rtx.ref_prim(rtx.RTX_PRIM_SPHERE, i) for i in range(n)])
    w = rtx.SceneDesc()
    for f, _ in rtx.SceneDesc._fields_:
        setattr(w, f, getattr(d, f))
    w.n_nodes, w.n_roots, w.roots = 0, n, roots
    assert walk_tree(ctypes.pointer(w))[0] is None


@pytest.mark.parametrize("scene,width,spp", [("random_spheres", 480, 6), ("earth_dielectric", 384, 4)])
def test_rebuilt_tree_changes_no_path(built, scene, width, spp):
    """The oracle walking the rebuilt tree against the oracle walking the reference's: the same
    image bit for bit, the same segments, hits, texel fetches and RNG draws; fewer box tests."""
    s = rtx.HostScene(scene, 1)
    cam = s.camera(width=width, spp=spp)
    desc = s.desc
    walk = rtx.walk_tree_desc(desc, cam)
    assert walk is not desc
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    a, ca = ob.render(desc, cam, 31, reg, ob.ORDER_ITERATIVE, 8)
    b, cb = ob.render(walk, cam, 31, reg, ob.ORDER_ITERATIVE, 8)
    assert np.array_equal(a, b)
    for k in ("samples", "segments", "hits", "texel_fetches", "rng_draws"):
        assert ca[k] == cb[k], k
    assert cb["node_visits"] < 0.8 * ca["node_visits"]


@pytest.mark.parametrize("octant", range(8))
def test_every_octant_changes_no_path(built, octant):
    """Each octant's child order on a small random_spheres render (cameras from every direction
    are represented by forcing the octant's tree on the main.go camera)."""
    s = rtx.HostScene("random_spheres", 1)
    cam = s.camera(width=96, spp=4)
    desc = s.desc
    arr, root = walk_tree(desc, octant)
    walk = rtx.desc_with_tree(desc, arr, len(arr), root)
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    a, ca = ob.render(desc, cam, 5, reg, ob.ORDER_ITERATIVE, 4)
    b, cb = ob.render(walk, cam, 5, reg, ob.ORDER_ITERATIVE, 4)
    assert np.array_equal(a, b)
    assert (ca["segments"], ca["hits"], ca["rng_draws"]) == (cb["segments"], cb["hits"], cb["rng_draws"])
