"""A World nested inside the tree (ABI 5 list refs): a World handed to NewBVH as a child
(hittables.go:39-76, bvh.go:142-185).  (*World).Hit scans its items in Add order with a
running closest bound (hittables.go:55-72); on the device the items' entries simply follow
one another in the threaded walk (rtx_capi.hip emit).

CPU: the flattener's list refs, the C-ABI's checks on them, and two equivalences the
reference's semantics imply, checked on the oracle: a list of one item renders exactly as
the item, and a World root equals a one-list root.  GPU: main.go's randSpheres grid in Worlds
nested three deep inside the BVH, bit-exact against the oracle with identical counters.
"""
import ctypes

import numpy as np
import pytest

import oracle_binding as ob
import parity
import rtx
from test_capi import create, lambertian, make_desc, sphere, texture


def list_desc(base, lists, list_refs, roots):
    L = (rtx.List * max(1, len(lists)))(*[rtx.List(a, b) for a, b in lists])
    R = (ctypes.c_int32 * max(1, len(list_refs)))(*list_refs)
    T = (ctypes.c_int32 * len(roots))(*roots)
    base.lists, base.n_lists = L, len(lists)
    base.list_refs, base.n_list_refs = R, len(list_refs)
    base.roots, base.n_roots = T, len(roots)
    base._keep2 = (L, R, T)
    return base


def lst(i):
    return rtx.ref_prim(rtx.RTX_PRIM_LIST, i)


def sph(i):
    return rtx.ref_prim(rtx.RTX_PRIM_SPHERE, i)


def three_spheres():
    ss = []
    for k, (x, z) in enumerate([(-0.6, -1.0), (0.0, -1.5), (0.6, -1.0)]):
        s = sphere()
        s.center[:] = [x, 0.0, z]
        s.radius = 0.45
        ss.append(s)
    return ss


def test_flatten_emits_list_refs(built):
    sc = rtx.HostScene("nested_worlds", seed=1)
    d = sc.desc.contents
    assert d.n_lists >= 3, d.n_lists  # the grid rows, row 3's rest and its World of two spheres
    kinds = {}
    for i in range(d.n_list_refs):
        r = d.list_refs[i]
        k = "node" if r >= 0 else ("list" if ((~r) & 0xFFFFFFFF) >> 28 == rtx.RTX_PRIM_LIST else "prim")
        kinds[k] = kinds.get(k, 0) + 1
    assert kinds.get("list", 0) >= 1 and kinds.get("node", 0) >= 1 and kinds.get("prim", 0) > 100
    total = sum(d.lists[i].count for i in range(d.n_lists))
    assert total == d.n_list_refs


def test_capi_list_checks(built):
    base = lambda: make_desc(three_spheres(), [lambertian()], [texture()])  # noqa: E731
    assert "list ref 1 out of range" in create(list_desc(base(), [(0, 3)], [sph(0), sph(1), sph(2)], [lst(1)]))[1]
    # an empty World nested in the tree is a miss (hittables.go:55-72): accepted
    rc, msg = create(list_desc(base(), [(0, 3), (3, 0)], [sph(0), sph(1), sph(2)], [lst(1), lst(0)]))
    assert rc in (rtx.RTX_OK, rtx.RTX_ERR_NO_DEVICE), msg
    assert "items out of range" in create(list_desc(base(), [(1, 3)], [sph(0), sph(1), sph(2)], [lst(0)]))[1]
    # a list holding itself
    rc, msg = create(list_desc(base(), [(0, 2)], [sph(0), lst(0)], [lst(0)]))
    assert rc == rtx.RTX_ERR_INVALID_ARG and "cycle" in msg
    # valid: on this CPU-only host the scene is built, then no device is found
    rc, msg = create(list_desc(base(), [(0, 3)], [sph(0), sph(1), sph(2)], [lst(0)]))
    assert rc in (rtx.RTX_OK, rtx.RTX_ERR_NO_DEVICE), msg


def small_camera(w=32, h=18, spp=4):
    cam = rtx.Camera()
    cam.image_width, cam.image_height, cam.samples_per_pixel, cam.max_depth = w, h, spp, 8
    cam.center[:] = [0, 0, 0]
    cam.pixel00[:] = [-0.9, 0.5, -1]
    cam.pixel_du[:] = [1.8 / w, 0, 0]
    cam.pixel_dv[:] = [0, -1.0 / h, 0]
    cam.background[:] = [0.7, 0.8, 1.0]
    return cam


@pytest.mark.parametrize("order", [ob.ORDER_REFERENCE, ob.ORDER_ITERATIVE])
def test_oracle_list_equivalences(built, order):
    cam = small_camera()
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    world = make_desc(three_spheres(), [lambertian()], [texture()], roots=[sph(0), sph(1), sph(2)])
    one_list = list_desc(make_desc(three_spheres(), [lambertian()], [texture()]), [(0, 3)],
                         [sph(0), sph(1), sph(2)], [lst(0)])
    # a list per item, and lists of lists
    singles = list_desc(make_desc(three_spheres(), [lambertian()], [texture()]), [(0, 1), (1, 1), (2, 1), (3, 2)],
                        [sph(0), sph(1), sph(2), lst(1), lst(2)], [lst(0), lst(3)])
    a, ca = ob.render(ctypes.byref(world), cam, 5, reg, order)
    b, cb = ob.render(ctypes.byref(one_list), cam, 5, reg, order)
    c, cc = ob.render(ctypes.byref(singles), cam, 5, reg, order)
    assert np.array_equal(a, b) and np.array_equal(a, c)
    assert ca == cb == cc


@pytest.mark.gpu
def test_nested_worlds_gpu_tiered(built):
    """The nested-World scene under the tiered walk (its node boxes hold every sphere's own box, so it
    gets a near tree; the caller's tree with its Worlds is the far tree): both kernels bit-exact, with
    the tiered oracle's counters (tests/parity.py)."""
    import torch

    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    sc = rtx.HostScene("nested_worlds", seed=1)
    dev = rtx.DeviceScene(sc.desc)
    cam = sc.camera(width=192, spp=6, depth=50)
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    _, st, _ = parity.check_scene(torch, dev, sc.desc, cam, 11, reg)
    assert st.walk_layout == rtx.RTX_LAYOUT_REFERENCE | rtx.RTX_LAYOUT_TIERED


@pytest.mark.gpu
def test_nested_worlds_gpu_bitexact(built):
    """The caller's tree with Worlds nested in it, walked as it is (RTX_SCENE_NO_TIER)."""
    import torch

    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    sc = rtx.HostScene("nested_worlds", seed=1)
    dev = rtx.DeviceScene(sc.desc, no_tier=True)
    cam = sc.camera(width=192, spp=6, depth=50)
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    out = torch.full((cam.image_height, cam.image_width, 3), float("nan"), device="cuda")
    walk, skip = parity.walk_of(dev, sc.desc, cam)  # (the caller's tree; its collapsed walk's skips)
    it, cnt = ob.render(walk, cam, 11, reg, ob.ORDER_ITERATIVE, skip=skip)
    for counters in (True, False):  # the counting kernel (C++ walk) and the timed one (asm walk)
        st = dev.render_region(cam, 11, reg, out.data_ptr(), torch.cuda.current_stream().cuda_stream,
                               counters=counters, timed=True)
        torch.cuda.synchronize()
        gpu = out.cpu().numpy()
        assert np.array_equal(gpu, it), float(np.nanmax(np.abs(gpu - it)))
        if counters:
            assert (st.segments, st.node_visits, st.prim_tests, st.hits, st.rng_draws) == (
                cnt["segments"], cnt["node_visits"], cnt["prim_tests"], cnt["hits"], cnt["rng_draws"])
