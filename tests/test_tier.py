"""The tiered walk on the CPU: rtx_walk_near_region / rtx_walk_tree(octant |
RTX_TREE_NEAR) build it without a device.

A tiered scene walks every segment that starts in the NEAR REGION on the near tree: the spheres
themselves as leaves, each behind its own box grown by the float32 sphere test's error bound for
origins in that region; a path whose segment starts outside it walks the guarded tree (the
reference's leaves) to its end.  These tests pin the region, the near tree's shape and margins, the
soundness claim the walk rests on — from any origin in the region, a hit the float32 sphere test
(hittables.go:96-116) reports lies where every box above its sphere passes (InBoundary,
bvh.go:84-102, with the bound just past the hit) — and, on the oracle, that the tiered walk changes no
path: image, segments, hits and draws equal the reference tree's, bit for bit.
"""
import ctypes
import math

import numpy as np
import pytest

import oracle_binding as ob
import rtx

F = np.float32


def near_tree(desc, cam, flags=0):
    L = rtx.load()
    n, root = ctypes.c_uint32(), ctypes.c_int32()
    oc = rtx.camera_octant(cam) | rtx.RTX_TREE_NEAR
    rtx.check(L.rtx_walk_tree(desc, flags, oc, None, 0, ctypes.byref(n), ctypes.byref(root)), "rtx_walk_tree")
    if n.value == 0:
        return None, root.value
    arr = (rtx.BvhNode * n.value)()
    rtx.check(L.rtx_walk_tree(desc, flags, oc, arr, n.value, ctypes.byref(n), ctypes.byref(root)), "rtx_walk_tree")
    return arr, root.value


def sphere_index(ref):
    p = (~ref) & 0xFFFFFFFF
    assert p >> 28 == rtx.RTX_PRIM_SPHERE
    return p & 0x0FFFFFFF


def margin(r, dmax, omax):
    """rtx_topology.h sphere_margin, restated: rho - r + 2^-20 (dmax + rho) + 2^-23 omax, rho = sqrt(r^2 + 24u
    (dmax^2 + r^2)), u = 2^-24 (the forward-error bound of DESIGN.md §15.1)."""
    rho = math.sqrt(r * r + 3.0 * math.ldexp(dmax * dmax + r * r, -21))
    return rho - r + math.ldexp(dmax + rho, -20) + math.ldexp(omax, -23)


def spheres_of(desc):
    d = desc.contents
    c = np.array([list(d.spheres[i].center) for i in range(d.n_spheres)], np.float32)
    r = np.array([d.spheres[i].radius for i in range(d.n_spheres)], np.float32)
    return c, r


@pytest.mark.parametrize("scene", ["random_spheres", "earth_dielectric"])
def test_near_region(built, scene):
    """The region holds every non-huge sphere and the camera's defocus disk, and is the core box grown
    by 1.5 times its largest extent (RTX_NEAR_GROW = 150 %); renders with the main.go camera qualify."""
    s = rtx.HostScene(scene, 1)
    cam = s.camera(width=96, spp=2)
    box, active = rtx.walk_near_region(s.desc, cam)
    assert box is not None and active
    lo, hi = np.array(box[:3]), np.array(box[3:])
    c, r = spheres_of(s.desc)
    small = np.abs(r) < 10  # all but the r = 1000 ground
    core_lo = (c[small] - np.abs(r[small])[:, None]).min(0)
    core_hi = (c[small] + np.abs(r[small])[:, None]).max(0)
    ext = (core_hi - core_lo).max()
    assert np.allclose(lo, core_lo - 1.5 * ext, atol=1e-4) and np.allclose(hi, core_hi + 1.5 * ext, atol=1e-4)
    assert (np.array(list(cam.center)) > lo).all() and (np.array(list(cam.center)) < hi).all()


@pytest.mark.parametrize("scene,flags,env", [("random_spheres", rtx.RTX_SCENE_NO_TIER, None),
                                             ("random_spheres", rtx.RTX_SCENE_REFERENCE_BVH, None),
                                             ("cornell_box", 0, "RTX_TIER_QUADS"), ("perlin_demo", 0, None)])
def test_no_near_tree(built, monkeypatch, scene, flags, env):
    """No tiers with RTX_SCENE_NO_TIER or the caller's tree (RTX_SCENE_REFERENCE_BVH), or for quads unless
    RTX_TIER_QUADS=1; a Perlin scene has a near tree but does not qualify."""
    if env:
        monkeypatch.setenv(env, "0")
    s = rtx.HostScene(scene, 1)
    cam = s.camera(width=64, spp=1)
    box, active = rtx.walk_near_region(s.desc, cam, flags)
    assert not active
    if scene != "perlin_demo":
        assert box is None and near_tree(s.desc, cam, flags)[0] is None


@pytest.mark.parametrize("scene", ["random_spheres", "earth_dielectric"])
def test_near_tree_shape(built, scene):
    """Every sphere is a leaf exactly once; every box contains its children's; the box just above a
    sphere contains the sphere's box grown by its margin for the farthest corner of the region."""
    s = rtx.HostScene(scene, 1)
    cam = s.camera(width=96, spp=2)
    box, _ = rtx.walk_near_region(s.desc, cam)
    arr, root = near_tree(s.desc, cam)
    assert arr is not None and root == 0
    c, r = spheres_of(s.desc)
    corners = np.array([[box[3 * ((m >> k) & 1) + k] for k in range(3)] for m in range(8)], np.float64)
    seen_nodes, seen_sph = np.zeros(len(arr), np.int32), np.zeros(len(c), np.int32)
    stack = [root]
    while stack:
        i = stack.pop()
        seen_nodes[i] += 1
        nd = arr[i]
        for ch in (nd.left, nd.right):
            if ch >= 0:
                for k in range(3):
                    assert nd.bmin[k] <= arr[ch].bmin[k] and nd.bmax[k] >= arr[ch].bmax[k]
                stack.append(ch)
                continue
            j = sphere_index(ch)
            seen_sph[j] += 1
            rr = abs(float(r[j]))
            dmax = float(np.sqrt(((corners - c[j].astype(np.float64)) ** 2).sum(1)).max())
            m = margin(rr, dmax, float(np.abs(corners).max()))
            for k in range(3):
                assert nd.bmin[k] <= float(c[j][k]) - rr - m and nd.bmax[k] >= float(c[j][k]) + rr + m
    assert (seen_nodes == 1).all() and (seen_sph == 1).all()


def sphere_t(o, d, c, r, tmin=F(0.001)):
    """Sphere.Hit's root (hittables.go:96-116) in float32, left-associative, no FMA; NaN = no hit."""
    oc = o - c
    a = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    hb = (d[:, 0] * oc[:, 0] + d[:, 1] * oc[:, 1]) + d[:, 2] * oc[:, 2]
    cc = ((oc[:, 0] * oc[:, 0] + oc[:, 1] * oc[:, 1]) + oc[:, 2] * oc[:, 2]) - r * r
    disc = hb * hb - a * cc
    ok = disc >= 0
    sq = np.sqrt(np.where(ok, disc, F(0)).astype(np.float64)).astype(F)
    t1 = (-hb - sq) / a
    t2 = (-hb + sq) / a
    t = np.where(t1 > tmin, t1, np.where(t2 > tmin, t2, F(np.nan)))
    return np.where(ok, t, F(np.nan)).astype(F)


def slab_pass(o, d, mn, mx, lo, hi):
    """(*Aabb).Hit (bvh.go:52-61, InBoundary :84-102) in float32, elementwise."""
    rmin, rmax = lo.copy(), hi.copy()
    ok = np.ones(len(o), bool)
    for k in range(3):
        inv = F(1) / d[:, k]
        t0 = (mn[:, k] - o[:, k]) * inv
        t1 = (mx[:, k] - o[:, k]) * inv
        sw = inv < 0
        t0, t1 = np.where(sw, t1, t0), np.where(sw, t0, t1)
        rmin = np.where(t0 > rmin, t0, rmin)
        rmax = np.where(t1 < rmax, t1, rmax)
        ok &= rmin < rmax
    return ok


def test_near_tree_reaches_every_reported_hit(built):
    """From origins in the near region, every hit the float32 sphere test reports — on near-tangent
    rays, where its error is largest — passes the slab test of every box above its sphere in the near
    tree with the running bound just past the hit: the walk reaches it."""
    s = rtx.HostScene("random_spheres", 1)
    cam = s.camera(width=96, spp=2)
    box, _ = rtx.walk_near_region(s.desc, cam)
    arr, root = near_tree(s.desc, cam)
    c, r = spheres_of(s.desc)
    parent_box = {}  # sphere -> boxes of its ancestors
    stack = [(root, [])]
    while stack:
        i, anc = stack.pop()
        chain = anc + [i]
        for ch in (arr[i].left, arr[i].right):
            if ch >= 0:
                stack.append((ch, chain))
            else:
                parent_box[sphere_index(ch)] = chain
    rng = np.random.default_rng(7)
    lo, hi = np.array(box[:3]), np.array(box[3:])
    n_hits = 0
    for trial in range(6):
        N = 100_000
        j = rng.integers(0, len(c), N)
        if trial % 3 == 0:
            j[:] = int(np.argmax(np.abs(r)))  # the ground sphere
        o = rng.uniform(lo, hi, (N, 3)).astype(F)
        cj, rj = c[j], np.abs(r[j])
        # aim at a point of the sphere's silhouette as seen from o, offset by a relative 1e-6 .. 1e-2
        u = (cj - o).astype(np.float64)
        u /= np.linalg.norm(u, axis=1)[:, None]
        w = rng.normal(size=(N, 3))
        w -= (w * u).sum(1)[:, None] * u
        w /= np.linalg.norm(w, axis=1)[:, None]
        off = rj * (1 + rng.normal(scale=[1e-6, 1e-4, 1e-2][trial % 3], size=N))
        d = ((cj.astype(np.float64) + w * off[:, None]) - o) * rng.uniform(0.1, 10, N)[:, None]
        d = d.astype(F)
        t = sphere_t(o, d, cj, rj.astype(F))
        hit = ~np.isnan(t)
        n_hits += int(hit.sum())
        bound = np.nextafter(t[hit], F(np.inf))
        oh, dh, jh = o[hit], d[hit], j[hit]
        for sph in np.unique(jh):
            sel = jh == sph
            for node in parent_box[int(sph)]:
                mn = np.tile(np.array(list(arr[node].bmin), F), (sel.sum(), 1))
                mx = np.tile(np.array(list(arr[node].bmax), F), (sel.sum(), 1))
                ok = slab_pass(oh[sel], dh[sel], mn, mx, np.full(sel.sum(), F(0.001)), bound[sel])
                assert ok.all(), (int(sph), node, int((~ok).sum()))
    assert n_hits > 100_000


def ancestors(arr, root):
    """sphere index -> the node indices above it in a near tree, root first."""
    out, stack = {}, [(root, [])]
    while stack:
        i, anc = stack.pop()
        chain = anc + [i]
        for ch in (arr[i].left, arr[i].right):
            if ch >= 0:
                stack.append((ch, chain))
            else:
                out[sphere_index(ch)] = chain
    return out


def tangent_rays(rng, o, c, r, rel, dscale=(1e-2, 1e2)):
    """Rays from o aimed at a point of the sphere's silhouette as seen from o, pushed out (rel > 0) or in
    (rel < 0) by rel * r, with direction lengths log-uniform in dscale (hittables.go does not normalise)."""
    u = (c - o).astype(np.float64)
    u /= np.linalg.norm(u, axis=1)[:, None]
    w = rng.normal(size=u.shape)
    w -= (w * u).sum(1)[:, None] * u
    w /= np.linalg.norm(w, axis=1)[:, None]
    d = (c.astype(np.float64) + w * (r * (1.0 + rel))[:, None]) - o
    return (d * np.exp(rng.uniform(np.log(dscale[0]), np.log(dscale[1]), len(o)))[:, None]).astype(F)


# (scene, spheres sampled (0: all), radius scale of the non-huge spheres, direction lengths): the BASELINE scenes
# with directions of length 1e-2 .. 1e2; randSpheres with radii x 0.01 (r = 2e-3 .. 1e-2 against D up to ~80: the
# margin is then ~40 radii) and with directions from 1e-8 to 1e8 (|1/d| up to 1e8 and |d|^2 down to 1e-16, the
# ends of Trav::safe's [2^-60, 2^60] and of near_fma_ok's |1/d| <= 2^64: the FMA form's products at their largest)
ADVERSARIAL = [("random_spheres", 0, 1.0, (1e-2, 1e2)), ("earth_dielectric", 0, 1.0, (1e-2, 1e2)),
               ("stress_100k", 3000, 1.0, (1e-2, 1e2)), ("random_spheres", 0, 0.01, (1e-2, 1e2)),
               ("random_spheres", 0, 1.0, (1e-8, 1e8))]


@pytest.mark.parametrize("scene,n_spheres,rscale,dscale", ADVERSARIAL,
                         ids=["random_spheres", "earth_dielectric", "stress_100k", "tiny_radii", "extreme_dirs"])
def test_margin_bound_adversarial(built, scene, n_spheres, rscale, dscale):
    """The forward-error bound behind sphere_margin, adversarially: from the near region's
    8 corners, its 6 face centres and random points in it, near-tangent rays (silhouette offsets of
    1e-7 .. 1e-1 of the radius, inside and out) at every sphere of the scene (a seeded sample of config 4's
    100k).  Every hit the float32 sphere test reports (hittables.go:96-116) lies within
    r + sphere_margin(r, D) of the centre (D = the origin's distance to it, evaluated exactly), so within
    the sphere's near-tree box, and every box above the sphere passes the float32 slab test (bvh.go:84-102)
    with the bound just past the hit.  The largest relative error met, K = (|P - c|^2 - r^2) / (u (D^2 + r^2)),
    stays below the 24 the margin assumes."""
    s = rtx.HostScene(scene, 1)
    cam = s.camera(width=96, spp=2)
    if rscale != 1.0:  # shrink every non-huge sphere in place: the caller's node boxes still contain them
        dd = s.desc.contents
        for i in range(dd.n_spheres):
            if abs(dd.spheres[i].radius) < 10:
                dd.spheres[i].radius = float(F(dd.spheres[i].radius) * F(rscale))
    box, active = rtx.walk_near_region(s.desc, cam)
    # (tiny radii fail the rebuild's precision gate: the region is then the core box grown by 1 %, the camera
    # outside it; the near tree and its margins are still built, and the bound is about them)
    assert box is not None and (active or rscale != 1.0)
    arr, root = near_tree(s.desc, cam)
    assert arr is not None
    anc = ancestors(arr, root)
    c_all, r_all = spheres_of(s.desc)
    bmin = np.array([list(arr[i].bmin) for i in range(len(arr))], F)
    bmax = np.array([list(arr[i].bmax) for i in range(len(arr))], F)
    A = np.full((len(c_all), max(len(v) for v in anc.values())), -1, np.int64)  # sphere -> its ancestors
    for sp, ch in anc.items():
        A[sp, :len(ch)] = ch
    rng = np.random.default_rng(11)
    sph = np.arange(len(c_all)) if not n_spheres else rng.choice(len(c_all), n_spheres, replace=False)
    lo, hi = np.array(box[:3], np.float64), np.array(box[3:], np.float64)
    corners = np.array([[box[3 * ((m >> k) & 1) + k] for k in range(3)] for m in range(8)], np.float64)
    faces = np.array([np.where(np.arange(3) == k, v, 0.5 * (lo + hi)) for k in range(3) for v in (lo[k], hi[k])])
    origins = np.concatenate([corners, faces, rng.uniform(lo, hi, (10, 3))]).astype(F)
    rels = np.array([1e-7, 1e-5, 1e-3, 1e-1, -1e-7, -1e-5, -1e-3, -1e-1])
    u = 2.0 ** -24
    n_hits, k_max = 0, 0.0
    for oi in range(len(origins)):
        j = np.repeat(sph, len(rels))
        rel = np.tile(rels, len(sph)) * rng.uniform(0.5, 2.0, len(j))
        o = np.repeat(origins[oi:oi + 1], len(j), axis=0)
        cj, rj = c_all[j], np.abs(r_all[j])
        d = tangent_rays(rng, o, cj, rj.astype(np.float64), rel, dscale)
        t = sphere_t(o, d, cj, rj)
        hit = ~np.isnan(t)
        n_hits += int(hit.sum())
        oh, dh, th, jh = o[hit].astype(np.float64), d[hit].astype(np.float64), t[hit].astype(np.float64), j[hit]
        ch, rh = c_all[jh].astype(np.float64), np.abs(r_all[jh]).astype(np.float64)
        D = np.linalg.norm(oh - ch, axis=1)
        dist = np.linalg.norm(oh + th[:, None] * dh - ch, axis=1)
        rho = np.sqrt(rh * rh + 3.0 * np.ldexp(D * D + rh * rh, -21))  # margin(), vectorised
        m = rho - rh + np.ldexp(D + rho, -20) + np.ldexp(np.abs(corners).max(), -23)
        assert (dist <= rh + m).all(), int((dist > rh + m).sum())
        k_max = max(k_max, float(((dist * dist - rh * rh) / (u * (D * D + rh * rh))).max()))
        bound = np.nextafter(t[hit], F(np.inf))
        chain = A[jh]  # every box above each hit's sphere, one depth at a time
        for lev in range(A.shape[1]):
            sel = chain[:, lev] >= 0
            if not sel.any():
                break
            nodes = chain[sel, lev]
            args = (o[hit][sel], d[hit][sel], bmin[nodes], bmax[nodes], np.full(int(sel.sum()), F(0.001)), bound[sel])
            ok = slab_pass(*args)  # the reference's form
            assert ok.all(), (lev, int((~ok).sum()))
            ok = ob.near_slab_pass(*args)  # the near walk's FMA form (§15.5)
            assert ok.all(), ("fma", lev, int((~ok).sum()))
    assert n_hits > 10_000
    assert k_max < 24.0, k_max
    print(f"{scene}: {n_hits} reported hits, largest K = {k_max:.2f} (the margin assumes 24)")


@pytest.mark.parametrize("scene,width,spp", [("random_spheres", 192, 4), ("earth_dielectric", 160, 3),
                                             ("cornell_box", 96, 4), ("quad_demo", 160, 4)])
def test_tiered_oracle_equals_reference(built, monkeypatch, scene, width, spp):
    """The oracle's tiered walk (near tree for paths in the near region, the guarded tree from a path's
    first segment outside it on) against the reference's tree: the same image bit for bit and the same
    segments, hits, texel fetches and draws; fewer box and sphere tests.  (Quads: RTX_TIER_QUADS=1)"""
    monkeypatch.setenv("RTX_TIER_QUADS", "1")
    s = rtx.HostScene(scene, 1)
    cam = s.camera(width=width, spp=spp)
    box, active = rtx.walk_near_region(s.desc, cam)
    assert active
    near = rtx.walk_near_desc(s.desc, cam)
    far = rtx.walk_tree_desc(s.desc, cam)
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    a, ca = ob.render(s.desc, cam, 2024, reg, ob.ORDER_ITERATIVE)
    b, cb = ob.render(near, cam, 2024, reg, ob.ORDER_ITERATIVE, tier=(box, far, None), rank=ob.sphere_ranks(s.desc))
    assert np.array_equal(a, b)
    for k in ("samples", "segments", "hits", "texel_fetches", "rng_draws"):
        assert ca[k] == cb[k], k
    if s.desc.contents.n_quads == 0:  # (a near tree over quads saves box tests only: DESIGN.md §26)
        assert cb["prim_tests"] < 0.7 * ca["prim_tests"] and cb["node_visits"] < 0.7 * ca["node_visits"]
    # every segment in the near tree alone (no far tier): the same image here too
    c, _ = ob.render(near, cam, 2024, reg, ob.ORDER_ITERATIVE, rank=ob.sphere_ranks(s.desc))
    assert np.array_equal(a, c)


@pytest.mark.parametrize("scene,width,spp,px,py,k", [
    ("random_spheres", 1920, 500, 269, 370, 371),     # a camera ray grazing a box face: the hit check defers it
    ("earth_dielectric", 3840, 1000, 1311, 469, 759),  # overlapping spheres 454 / 455 at one root: the tie rule
    ("earth_dielectric", 3840, 1000, 3487, 1098, 691),
])
def test_tiered_oracle_known_cases(built, scene, width, spp, px, py, k):
    """Single samples of the BASELINE frames where the near tree alone once differed from the reference
    (found on whole GPU frames, traced on the oracle): the tiered walk with its hit
    check and tie rule gives the reference's colour and path length."""
    L = ob.load()
    s = rtx.HostScene(scene, 1)
    cam = s.camera(width=width, spp=spp)
    box, active = rtx.walk_near_region(s.desc, cam)
    assert active
    near = rtx.walk_near_desc(s.desc, cam)
    far = rtx.walk_tree_desc(s.desc, cam)
    want, wc = ob.sample(s.desc, cam, 2024, px, py, k, ob.ORDER_ITERATIVE)
    rank = np.ascontiguousarray(ob.sphere_ranks(s.desc), np.uint32)
    L.oracle_sphere_rank(rank.ctypes.data_as(ctypes.c_void_p))
    L.oracle_tier((ctypes.c_float * 6)(*box), ctypes.cast(far, ctypes.c_void_p), None)
    try:
        got, gc = ob.sample(near, cam, 2024, px, py, k, ob.ORDER_ITERATIVE)
    finally:
        L.oracle_tier(None, None, None)
        L.oracle_sphere_rank(None)
    assert np.array_equal(np.asarray(got), np.asarray(want)), (got, want)
    assert gc["segments"] == wc["segments"] and gc["rng_draws"] == wc["rng_draws"]


# ---- quads in the near tree ----------------------------------------------------------------------
def quads_of(desc):
    d = desc.contents
    g = lambda f: np.array([list(getattr(d.quads[i], f)) for i in range(d.n_quads)], F)  # noqa: E731
    return g("q"), g("u"), g("v"), g("w"), g("normal"), np.array([d.quads[i].d for i in range(d.n_quads)], F)


def quad_t(o, d, Q, U, V, W, N, D, tmin=F(0.001)):
    """Quad.Hit (hittables.go:167-194) in float32, left-associative, no FMA: (t, point) with t NaN = no hit."""
    denom = (d[:, 0] * N[:, 0] + d[:, 1] * N[:, 1]) + d[:, 2] * N[:, 2]
    ok = ~(np.abs(denom.astype(np.float64)) < 1e-8)
    num = D - ((N[:, 0] * o[:, 0] + N[:, 1] * o[:, 1]) + N[:, 2] * o[:, 2])
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        t = (num / np.where(ok, denom, F(1))).astype(F)
    ok &= tmin < t
    P = (d * t[:, None] + o).astype(F)  # Add(Scale(dir, t), origin)
    php = (P - Q).astype(F)

    def cross(l, r):  # vec3.go:129-135
        return np.stack([l[:, 1] * r[:, 2] - l[:, 2] * r[:, 1], l[:, 2] * r[:, 0] - l[:, 0] * r[:, 2],
                         l[:, 0] * r[:, 1] - l[:, 1] * r[:, 0]], 1).astype(F)

    def dot(l, r):
        return ((l[:, 0] * r[:, 0] + l[:, 1] * r[:, 1]) + l[:, 2] * r[:, 2]).astype(F)

    alpha, beta = dot(W, cross(php, V)), dot(W, cross(U, php))
    ok &= ~((alpha < 0) | (1 < alpha) | (beta < 0) | (1 < beta))
    return np.where(ok, t, F(np.nan)).astype(F)


def quad_ancestors(arr, root):
    out, stack = {}, [(root, [])]
    while stack:
        i, anc = stack.pop()
        chain = anc + [i]
        for ch in (arr[i].left, arr[i].right):
            if ch >= 0:
                stack.append((ch, chain))
            elif ((~ch) & 0xFFFFFFFF) >> 28 == rtx.RTX_PRIM_QUAD:
                out[(~ch) & 0x0FFFFFFF] = chain
    return out


@pytest.mark.parametrize("scene", ["cornell_box", "quad_demo"])
def test_quad_margin_adversarial(built, monkeypatch, scene):
    """The bound behind quad_margin (rtx_topology.h), adversarially: from the near region's corners, face centres
    and random points, rays at every quad's edges and corners (in-plane offsets of 1e-7 .. 1e-1 of the edge,
    inside and out) and at grazing angles, direction lengths 1e-2 .. 1e2.  Every hit the float32 quad test reports
    lies within the quad's margin of its parallelogram — so inside its near-tree box — and every box above the quad
    passes the float32 slab test with the bound just past the hit (the near walk reaches it)."""
    monkeypatch.setenv("RTX_TIER_QUADS", "1")
    s = rtx.HostScene(scene, 1)
    cam = s.camera(width=96, spp=2)
    box, active = rtx.walk_near_region(s.desc, cam)
    assert box is not None and active
    arr, root = near_tree(s.desc, cam)
    anc = quad_ancestors(arr, root)
    Q, U, V, W, N, D = quads_of(s.desc)
    assert len(anc) == len(Q) > 0
    bmin = np.array([list(arr[i].bmin) for i in range(len(arr))], F)
    bmax = np.array([list(arr[i].bmax) for i in range(len(arr))], F)
    rng = np.random.default_rng(5)
    lo, hi = np.array(box[:3], np.float64), np.array(box[3:], np.float64)
    corners = np.array([[box[3 * ((m >> k) & 1) + k] for k in range(3)] for m in range(8)], np.float64)
    faces = np.array([np.where(np.arange(3) == k, v, 0.5 * (lo + hi)) for k in range(3) for v in (lo[k], hi[k])])
    origins = np.concatenate([corners, faces, rng.uniform(lo, hi, (20, 3))])
    omax = float(np.abs(corners).max())
    n_hits, worst = 0, 0.0
    for qi in range(len(Q)):
        q, u, v = Q[qi].astype(np.float64), U[qi].astype(np.float64), V[qi].astype(np.float64)
        # targets: points at the edges and corners, pushed in or out by a relative 1e-7 .. 1e-1 of the edges
        a = rng.choice([0.0, 1.0], 4000) + rng.choice([-1, 1], 4000) * 10.0 ** rng.uniform(-7, -1, 4000)
        b = np.where(rng.random(4000) < 0.5, rng.uniform(0, 1, 4000),
                     rng.choice([0.0, 1.0], 4000) + rng.choice([-1, 1], 4000) * 10.0 ** rng.uniform(-7, -1, 4000))
        swap = rng.random(4000) < 0.5
        a, b = np.where(swap, b, a), np.where(swap, a, b)
        tgt = q + a[:, None] * u + b[:, None] * v
        o = origins[rng.integers(0, len(origins), 4000)]
        # grazing rays (a quarter): the target seen from an origin moved along the plane
        n = np.cross(u, v)
        n /= np.linalg.norm(n)
        gr = rng.random(4000) < 0.25
        o = np.where(gr[:, None], tgt + (o - tgt) - ((o - tgt) @ n)[:, None] * n * (1 - 10.0 ** rng.uniform(-6, -2, 4000))[:, None], o)
        o = np.clip(o, lo, hi).astype(F)
        d = ((tgt - o.astype(np.float64)) * np.exp(rng.uniform(np.log(1e-2), np.log(1e2), 4000))[:, None]).astype(F)
        k = np.full(4000, qi)
        t = quad_t(o, d, Q[k], U[k], V[k], W[k], N[k], D[k])
        hit = ~np.isnan(t)
        n_hits += int(hit.sum())
        if not hit.any():
            continue
        X = o[hit].astype(np.float64) + t[hit].astype(np.float64)[:, None] * d[hit].astype(np.float64)
        # distance of the exact point from the parallelogram: solve X = q + a u + b v + c n
        M = np.stack([u, v, n], 1)
        abc = np.linalg.solve(M, (X - q).T).T
        ea = np.maximum(0, np.maximum(-abc[:, 0], abc[:, 0] - 1)) * np.linalg.norm(u)
        eb = np.maximum(0, np.maximum(-abc[:, 1], abc[:, 1] - 1)) * np.linalg.norm(v)
        dist = ea + eb + np.abs(abc[:, 2])
        m = margin_q(Q[qi], U[qi], V[qi], omax)
        worst = max(worst, float(dist.max() / m))
        assert (dist <= m).all(), (qi, float(dist.max()), m)
        bound = np.nextafter(t[hit], F(np.inf))
        for node in anc[qi]:
            cnt = int(hit.sum())
            ok = slab_pass(o[hit], d[hit], np.tile(bmin[node], (cnt, 1)), np.tile(bmax[node], (cnt, 1)),
                           np.full(cnt, F(0.001)), bound)
            assert ok.all(), (qi, node, int((~ok).sum()))
    assert n_hits > 5_000
    assert worst < 0.25, worst  # the hits stay well inside the margin
    print(f"{scene}: {n_hits} reported hits, the farthest at {worst:.4f} of the margin")


def margin_q(q, u, v, omax):
    """rtx_topology.h quad_margin, restated (K = 64)."""
    q, u, v = q.astype(np.float64), u.astype(np.float64), v.astype(np.float64)
    U, V, S = np.linalg.norm(u), np.linalg.norm(v), np.linalg.norm(np.cross(u, v))
    B = float((np.abs(q) + np.abs(u) + np.abs(v)).max())
    m = math.ldexp(64.0 * (U + V + 2 * B + 3 * omax) * (2 + 2 * U * V / S), -24)
    return m + math.ldexp(B + omax + m, -21)


def test_quad_ties_gate(built, monkeypatch):
    """Coplanar, overlapping quads enter a near tree only when a tie between them cannot change a path (the same
    material, not an image texture, and the same normal): the Cornell box's box bottoms on its floor qualify
    (RTX_TIER_QUADS=1; off by default)."""
    monkeypatch.setenv("RTX_TIER_QUADS", "1")
    s = rtx.HostScene("cornell_box", 1)
    cam = s.camera(width=64, spp=1)
    assert rtx.walk_near_region(s.desc, cam)[1]
    d = s.desc.contents
    floor = next(i for i in range(d.n_quads) if list(d.quads[i].normal) == [0.0, -1.0, 0.0] and d.quads[i].q[1] == 0.0
                 and d.quads[i].u[0] == 555.0)
    old = d.quads[floor].material
    d.quads[floor].material = next(m for m in range(d.n_materials) if m != old)  # another material: no tiers
    try:
        assert not rtx.walk_near_region(s.desc, cam)[1]
    finally:
        d.quads[floor].material = old
