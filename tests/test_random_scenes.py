"""Seeded random scenes on the GPU vs the oracle: spheres with radii from 1e-3 to 2.5, quads
(some degenerate), every material and texture kind, BVH trees built here (median splits on a
random axis), cameras at random places — including one looking exactly down an axis, whose
centre rays have zero direction components (1/dir = inf: the walk's select form, not the med3
one).  Both kernels run: the counting one (the C++ walk step, its counters pinned to the
oracle's) and the timed one (the asm walk).  Bit-exact against the oracle's iterative colour
order; the scenes are hand-made tables, so they also exercise the C-ABI with trees no main.go
scene builds.
"""
import ctypes

import numpy as np
import pytest

import oracle_binding as ob
import parity
import rtx

pytestmark = pytest.mark.gpu

F = np.float32


def f3(a):
    return [float(F(x)) for x in a]


def build_scene(seed: int, n_spheres: int, n_quads: int):
    rng = np.random.default_rng(seed)
    tex = []
    t = rtx.Texture()
    t.type = rtx.RTX_TEX_SOLID
    t.even[:] = [0.7, 0.3, 0.2]
    tex.append(t)
    t = rtx.Texture()
    t.type = rtx.RTX_TEX_CHECKERED
    t.scale = 0.37
    t.even[:] = [0.2, 0.3, 0.1]
    t.odd[:] = [0.9, 0.9, 0.9]
    tex.append(t)
    mats = []
    for k in range(12):
        m = rtx.Material()
        kind = k % 4
        m.type = [rtx.RTX_MAT_LAMBERTIAN, rtx.RTX_MAT_METAL, rtx.RTX_MAT_DIELECTRIC, rtx.RTX_MAT_DIFFUSE_LIGHT][kind]
        m.texture = int(rng.integers(0, 2)) if kind in (0, 3) else 0
        m.albedo[:] = f3(rng.uniform(0.1, 1.0, 3))
        m.fuzz = float(F(rng.uniform(0, 1)))
        m.ior = float(F(rng.uniform(1.0, 2.5)))
        mats.append(m)
    prims = []  # (ref, bmin, bmax)
    spheres = []
    for i in range(n_spheres):
        s = rtx.Sphere()
        c = rng.uniform(-6, 6, 3).astype(F)
        r = F(10.0 ** rng.uniform(-3, 0.4))
        if i == 0:
            c, r = np.array([0, -1000, 0], F), F(999.0)  # a ground the camera may stand on
        s.center[:] = f3(c)
        s.radius = float(r)
        s.material = int(rng.integers(0, len(mats)))
        spheres.append(s)
        prims.append((rtx.ref_prim(rtx.RTX_PRIM_SPHERE, i), c - r, c + r))
    quads = []
    for i in range(n_quads):
        q = rtx.Quad()
        Q = rng.uniform(-5, 5, 3).astype(F)
        u = rng.uniform(-3, 3, 3).astype(F)
        v = rng.uniform(-3, 3, 3).astype(F) if i % 7 else u * F(2)  # every 7th degenerate (u || v)
        n = np.cross(u.astype(np.float64), v.astype(np.float64))
        nn = np.linalg.norm(n)
        normal = (n / nn).astype(F) if nn > 0 else np.array([np.nan] * 3, F)
        D = F(np.dot(normal.astype(np.float64), Q.astype(np.float64)))
        w = (n / (nn * nn)).astype(F) if nn > 0 else np.array([np.nan] * 3, F)
        q.q[:] = f3(Q)
        q.u[:] = f3(u)
        q.v[:] = f3(v)
        q.w[:] = f3(w)
        q.normal[:] = f3(normal)
        q.d = float(D)
        q.material = int(rng.integers(0, len(mats)))
        quads.append(q)
        pts = np.array([Q, Q + u, Q + v, Q + u + v], F)
        prims.append((rtx.ref_prim(rtx.RTX_PRIM_QUAD, i), pts.min(0) - F(1e-3), pts.max(0) + F(1e-3)))
    nodes = []

    def build(items):
        if len(items) == 1:
            return items[0][0], items[0][1], items[0][2]
        axis = int(rng.integers(0, 3))
        items = sorted(items, key=lambda it: float(it[1][axis]))
        mid = len(items) // 2
        me = len(nodes)
        nodes.append(None)
        lref, lmin, lmax = build(items[:mid])
        rref, rmin, rmax = build(items[mid:])
        bmin, bmax = np.minimum(lmin, rmin), np.maximum(lmax, rmax)
        nd = rtx.BvhNode()
        nd.bmin[:] = f3(bmin)
        nd.bmax[:] = f3(bmax)
        nd.left, nd.right = lref, rref
        nodes[me] = nd
        return me, bmin, bmax

    root, _, _ = build(prims)
    d = rtx.SceneDesc()
    keep = []

    def arr(ctype, items):
        a = (ctype * max(1, len(items)))(*items)
        keep.append(a)
        return a

    d.nodes, d.n_nodes = arr(rtx.BvhNode, nodes), len(nodes)
    d.roots, d.n_roots = arr(ctypes.c_int32, [root]), 1
    d.spheres, d.n_spheres = arr(rtx.Sphere, spheres), len(spheres)
    d.quads, d.n_quads = arr(rtx.Quad, quads), len(quads)
    d.materials, d.n_materials = arr(rtx.Material, mats), len(mats)
    d.textures, d.n_textures = arr(rtx.Texture, tex), len(tex)
    d._keep = keep
    return d


def camera(seed: int, w: int, h: int, spp: int, axis_aligned: bool):
    rng = np.random.default_rng(seed + 1000)
    cam = rtx.Camera()
    cam.image_width, cam.image_height, cam.samples_per_pixel, cam.max_depth = w, h, spp, 12
    if axis_aligned:  # look down -z with du || x, dv || -y: centre rays have d.x == 0 or d.y == 0
        origin = np.array([0.5, 2.0, 14.0], F)
        du = np.array([0.25, 0, 0], F)
        dv = np.array([0, -0.25, 0], F)
        p00 = origin + np.array([-(w // 2) * 0.25, (h // 2) * 0.25, -8.0], F)
    else:
        origin = rng.uniform(-9, 9, 3).astype(F)
        origin[1] = abs(origin[1]) + F(0.5)
        look = rng.uniform(-2, 2, 3).astype(F)
        fwd = (look - origin) / np.linalg.norm(look - origin)
        right = np.cross(fwd, [0, 1, 0])
        right /= np.linalg.norm(right)
        up = np.cross(right, fwd)
        du = (right * (6.0 / w)).astype(F)
        dv = (-up * (6.0 / w)).astype(F)
        p00 = (origin + fwd * 4 - right * 3 + up * (3.0 * h / w)).astype(F)
    cam.center[:] = f3(origin)
    cam.pixel00[:] = f3(p00)
    cam.pixel_du[:] = f3(du)
    cam.pixel_dv[:] = f3(dv)
    cam.background[:] = [0.6, 0.7, 0.9]
    if seed % 2:
        cam.defocus_angle = 0.05
        cam.defocus_disk_u[:] = f3(du * 2)
        cam.defocus_disk_v[:] = f3(dv * 2)
    return cam


@pytest.mark.parametrize("seed,n_spheres,n_quads,axis_aligned", [
    (1, 120, 0, False), (2, 40, 14, False), (3, 200, 30, True), (4, 8, 0, True), (5, 1, 21, False)])
def test_random_scene_bitexact(built, seed, n_spheres, n_quads, axis_aligned):
    import torch

    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    d = build_scene(seed, n_spheres, n_quads)
    cam = camera(seed, 64, 36, 6, axis_aligned)
    pd = ctypes.pointer(d)
    dev = rtx.DeviceScene(pd)
    walk, skip = parity.walk_of(dev, pd, cam)  # the tree the scene walks (sphere-only trees may be rebuilt)
    tier = parity.tier_of(dev, pd, cam)  # ... and walk in two tiers
    if tier is not None:
        walk, skip, tier = tier
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    rank = ob.sphere_ranks(pd) if walk is not pd else None
    it, cnt = ob.render(walk, cam, seed, reg, ob.ORDER_ITERATIVE, skip=skip, tier=tier, rank=rank)
    if walk is not pd:  # the rebuilt tree: same image and paths as the caller's tree on the oracle
        it0, cnt0 = ob.render(pd, cam, seed, reg, ob.ORDER_ITERATIVE)
        assert np.array_equal(it, it0, equal_nan=True)
        assert all(cnt[k] == cnt0[k] for k in ("segments", "hits", "rng_draws"))
    out = torch.full((cam.image_height, cam.image_width, 3), float("nan"), device="cuda")
    for counters in (True, False):
        st = dev.render_region(cam, seed, reg, out.data_ptr(), torch.cuda.current_stream().cuda_stream,
                               counters=counters, timed=True)
        torch.cuda.synchronize()
        gpu = out.cpu().numpy()
        assert np.array_equal(gpu, it, equal_nan=True), (counters, float(np.nanmax(np.abs(gpu - it))))
        if counters:
            assert (st.segments, st.node_visits, st.prim_tests, st.hits, st.rng_draws) == (
                cnt["segments"], cnt["node_visits"], cnt["prim_tests"], cnt["hits"], cnt["rng_draws"])
