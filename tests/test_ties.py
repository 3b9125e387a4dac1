"""Exact ties between spheres (bvh.go:220-249 keeps the sphere it meets first: the right subtree is
clipped to the left's hit, strictly) on every walk the library takes of another tree or in another
storage order: the LDS layouts (entry index = the reference walk's rank), and the HBM layouts, whose
sphere entries carry a rank word (sphere_test RANK_WORD) — the near tree, the guarded tree and the
caller's tree read from HBM (RTX_FLAG_NO_LDS) or through the LDS cache of a big scene.

The scene: randSpheres' spheres plus exact copies of its three big spheres with other materials, under
a NewBVH-shaped tree (median splits, leaves of one or two spheres, boxes the unions of NewSphere's).  A
ray that hits a big sphere hits its copy at the same float32 root, so the pixels there show whichever
material the walk keeps.
"""
import ctypes

import numpy as np
import pytest

import oracle_binding as ob
import rtx

F = np.float32


def own_box(c, r):
    p1, p2 = c + F(r) * F(-1.0), c + F(r)
    return np.minimum(p1, p2), np.maximum(p1, p2)


def newbvh_desc(spheres, materials, base_desc):
    """A scene description whose tree is NewBVH-shaped over `spheres` (list of (centre, r, material))."""
    n = len(spheres)
    sph = (rtx.Sphere * n)()
    for i, (c, r, m) in enumerate(spheres):
        sph[i].center = (ctypes.c_float * 3)(*[float(v) for v in c])
        sph[i].radius = float(r)
        sph[i].material = m
    boxes = [own_box(np.array(c, F), r) for c, r, _ in spheres]
    nodes = []

    def build(ids, depth):
        ax = depth % 3
        ids = sorted(ids, key=lambda i: -float(boxes[i][0][ax]))  # descending box minimum, stable
        me = len(nodes)
        nodes.append(None)
        if len(ids) <= 2:
            kids = [rtx.ref_prim(rtx.RTX_PRIM_SPHERE, i) for i in ids]
            if len(kids) == 1:
                kids.append(kids[0])  # a one-element split: left == right (bvh.go:162-165)
            lo = np.min([boxes[i][0] for i in ids], axis=0)
            hi = np.max([boxes[i][1] for i in ids], axis=0)
        else:
            h = len(ids) // 2
            a, b = build(ids[:h], depth + 1), build(ids[h:], depth + 1)
            kids = [a, b]
            lo = np.minimum(np.array(nodes[a][0]), np.array(nodes[b][0]))
            hi = np.maximum(np.array(nodes[a][1]), np.array(nodes[b][1]))
        nodes[me] = (lo.astype(F), hi.astype(F), kids)
        return me

    root = build(list(range(n)), 0)
    arr = (rtx.BvhNode * len(nodes))()
    for i, (lo, hi, kids) in enumerate(nodes):
        arr[i].bmin = (ctypes.c_float * 3)(*[float(v) for v in lo])
        arr[i].bmax = (ctypes.c_float * 3)(*[float(v) for v in hi])
        arr[i].left, arr[i].right = kids
    d = base_desc.contents
    w = rtx.SceneDesc()
    for f, _ in rtx.SceneDesc._fields_:
        setattr(w, f, getattr(d, f))
    roots = (ctypes.c_int32 * 1)(root)
    w.spheres, w.n_spheres = ctypes.cast(sph, ctypes.POINTER(rtx.Sphere)), n
    w.nodes, w.n_nodes = ctypes.cast(arr, ctypes.POINTER(rtx.BvhNode)), len(nodes)
    w.roots, w.n_roots = ctypes.cast(roots, ctypes.POINTER(ctypes.c_int32)), 1
    p = ctypes.pointer(w)
    p._keep = (sph, arr, roots, base_desc)
    return p


@pytest.fixture(scope="module")
def tie_scene(built):
    host = rtx.HostScene("random_spheres", 1)
    d = host.desc.contents
    spheres = [(tuple(d.spheres[i].center), d.spheres[i].radius, d.spheres[i].material) for i in range(d.n_spheres)]
    big = [i for i, s in enumerate(spheres) if abs(s[1] - 1.0) < 1e-6]
    assert len(big) == 3
    mats = [spheres[i][2] for i in big]
    # each big sphere again, with the next big sphere's material (glass / diffuse / metal rotated)
    spheres += [(spheres[i][0], spheres[i][1], mats[(k + 1) % 3]) for k, i in enumerate(big)]
    return host, newbvh_desc(spheres, None, host.desc)


def test_ties_matter_on_the_near_tree(tie_scene):
    """CPU: the near tree walked without the tie rule differs from the reference walk on this scene, so
    the GPU tests below are sensitive to it; with the rule (oracle_sphere_rank) it is bit-identical."""
    host, desc = tie_scene
    cam = host.camera(width=128, spp=2)
    box, active = rtx.walk_near_region(desc, cam)
    assert active
    near = rtx.walk_near_desc(desc, cam)
    far = rtx.walk_tree_desc(desc, cam)
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    want, _ = ob.render(desc, cam, 5, reg, ob.ORDER_ITERATIVE)
    bare, _ = ob.render(near, cam, 5, reg, ob.ORDER_ITERATIVE, tier=(box, far, None))
    ranked, _ = ob.render(near, cam, 5, reg, ob.ORDER_ITERATIVE, tier=(box, far, None), rank=ob.sphere_ranks(desc))
    assert np.array_equal(ranked, want)
    assert (bare != want).any(axis=2).sum() > 50


@pytest.mark.gpu
@pytest.mark.parametrize("flags,no_tier", [(0, False), (rtx.RTX_FLAG_NO_LDS, False), (0, True),
                                           (rtx.RTX_FLAG_NO_LDS, True)])
def test_ties_gpu(tie_scene, flags, no_tier):
    """Both kernels bit-identical to the oracle (tests/parity.py) on the tie scene: the tiered walk (near
    tree + guarded tree) and the guarded tree alone, from the LDS copy (entry-index rank) and from HBM
    (rank words)."""
    import torch

    from parity import check_scene

    torch.cuda.set_device(0)
    host, desc = tie_scene
    dev = rtx.DeviceScene(desc, no_tier=no_tier)
    cam = host.camera(width=128, spp=2)
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    _, st, _ = check_scene(torch, dev, desc, cam, 5, reg, flags=flags)
    want = rtx.RTX_SCENE_IN_LDS if not flags else rtx.RTX_SCENE_IN_HBM
    assert st.scene_placement == want, (st.scene_placement, want)
    assert bool(st.walk_layout & rtx.RTX_LAYOUT_TIERED) == (not no_tier)
