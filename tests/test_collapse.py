"""The collapsed walk (rtx_collapse.h) on the CPU: rtx_walk_skip plans it without a device.

A walk may leave out the box test of a node whose children are all nodes with boxes inside its
own: InBoundary (bvh.go:84-102) is monotone in the box, so a child passes only where its parent
passes and the walk tests the same primitives in the same order against the same bounds.  These
tests pin the lemma itself on float32 edge cases, the plan's guards (primitive children, boxes
that do not nest, the opt-outs), and — on the oracle, with its walk hooks leaving out the same
tests — that the collapsed walk changes no image bit and no counter but the box tests.
"""
import ctypes

import numpy as np
import pytest

import oracle_binding as ob
import rtx

F = np.float32
PATH = ("samples", "segments", "hits", "texel_fetches", "rng_draws", "prim_tests")


def in_boundary(d, o, lo, hi, tmin, tmax):
    """InBoundary (bvh.go:84-102) in float32, elementwise."""
    with np.errstate(all="ignore"):
        inv = F(1) / d
        t0, t1 = (lo - o) * inv, (hi - o) * inv
        sw = inv < 0
        t0, t1 = np.where(sw, t1, t0), np.where(sw, t0, t1)
        tmin = np.where(t0 > tmin, t0, tmin)
        tmax = np.where(t1 < tmax, t1, tmax)
    return tmin < tmax, tmin, tmax


def aabb_hit(o, d, lo, hi, tmin, tmax):
    ok = np.ones(len(o), bool)
    tmin = np.full(len(o), tmin, F)
    tmax = np.full(len(o), tmax, F)
    for k in range(3):
        hit, a, b = in_boundary(d[:, k], o[:, k], lo[:, k], hi[:, k], tmin, tmax)
        tmin, tmax = np.where(ok, a, tmin), np.where(ok, b, tmax)
        ok &= hit
    return ok


def test_slab_test_is_monotone_in_the_box():
    """child box inside parent box => (child passes => parent passes), on rays and boxes built
    to hit the float32 corner cases: zero and signed-zero directions (1/d = +-inf, 0 * inf = NaN),
    origins on the box planes, +-0 coordinates, infinite directions, tiny and huge values."""
    rng = np.random.default_rng(5)
    n = 400_000
    special = np.array([0.0, -0.0, 1e-38, -1e-38, 1e-45, 3e38, -3e38, np.inf, -np.inf, 1.0, -1.0], F)

    def pick(shape, p_special=0.3):
        v = rng.uniform(-4, 4, shape).astype(F)
        m = rng.random(shape) < p_special
        v[m] = rng.choice(special, m.sum())
        return v

    # child box, then a parent box containing it (some faces shared exactly, some -0 / +0 swaps)
    c_lo = rng.integers(-4, 4, (n, 3)).astype(F) * F(0.5)
    c_hi = c_lo + rng.integers(0, 3, (n, 3)).astype(F) * F(0.5)
    grow_lo = np.where(rng.random((n, 3)) < 0.5, F(0), rng.integers(0, 3, (n, 3)).astype(F) * F(0.5))
    grow_hi = np.where(rng.random((n, 3)) < 0.5, F(0), rng.integers(0, 3, (n, 3)).astype(F) * F(0.5))
    p_lo, p_hi = c_lo - grow_lo, c_hi + grow_hi
    z = rng.random((n, 3)) < 0.2  # signed zeros on shared faces
    p_lo = np.where(z & (p_lo == 0), F(-0.0), p_lo)
    c_lo = np.where(z & (c_lo == 0), F(0.0), c_lo)
    assert (c_lo >= p_lo).all() and (c_hi <= p_hi).all()
    # origins often on a box plane, directions often with special components
    o = rng.integers(-5, 5, (n, 3)).astype(F) * F(0.5)
    o = np.where(rng.random((n, 3)) < 0.2, pick((n, 3), 0.0), o)
    target = c_lo + (c_hi - c_lo) * rng.random((n, 3)).astype(F)  # aimed at the child box, mostly
    d = (target - o).astype(F)
    sp = rng.random((n, 3)) < 0.25
    d[sp] = rng.choice(special, sp.sum())
    for tmax in (F(np.inf), F(3.0), F(0.25)):
        child = aabb_hit(o, d, c_lo, c_hi, F(0.001), tmax)
        parent = aabb_hit(o, d, p_lo, p_hi, F(0.001), tmax)
        assert child.sum() > 1000 and (~child).sum() > 1000
        bad = child & ~parent
        assert not bad.any(), (o[bad][:3], d[bad][:3], c_lo[bad][:3], c_hi[bad][:3], p_lo[bad][:3], p_hi[bad][:3])


def oracle_pair(desc, walk, cam, seed, skip_nodes):
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    a, ca = ob.render(walk, cam, seed, reg, ob.ORDER_ITERATIVE, 8)
    b, cb = ob.render(walk, cam, seed, reg, ob.ORDER_ITERATIVE, 8, skip=skip_nodes)
    return a, ca, b, cb


@pytest.mark.parametrize("scene,width,spp,min_gain", [
    ("random_spheres", 192, 3, 0.2), ("earth_dielectric", 160, 2, 0.2), ("cornell_box", 96, 3, 0.2),
    ("quad_demo", 96, 3, 0.0), ("simple_light_demo", 96, 3, 0.0), ("nested_worlds", 96, 2, 0.0)])
def test_collapsed_walk_changes_no_path(built, scene, width, spp, min_gain):
    s = rtx.HostScene(scene, 1)
    cam = s.camera(width=width, spp=spp)
    desc = s.desc
    walk = rtx.walk_tree_desc(desc, cam)
    skip = rtx.walk_skip(desc, cam)
    nodes = rtx.node_skip(walk, skip)
    a, ca, b, cb = oracle_pair(desc, walk, cam, 17, nodes)
    assert np.array_equal(a, b)
    for k in PATH:
        assert ca[k] == cb[k], k
    assert cb["node_visits"] <= (1.0 - min_gain) * ca["node_visits"]


def test_skips_only_nodes_over_nested_nodes(built):
    for scene in ("random_spheres", "cornell_box", "stress_100k"):
        s = rtx.HostScene(scene, 1)
        cam = s.camera(width=192, spp=1)
        walk = rtx.walk_tree_desc(s.desc, cam)
        nodes = rtx.node_skip(walk, rtx.walk_skip(s.desc, cam))
        d = walk.contents
        assert nodes.any()
        for i in np.flatnonzero(nodes):
            nd = d.nodes[int(i)]
            assert nd.left >= 0 and nd.right >= 0
            for c in (nd.left, nd.right):
                ch = d.nodes[c]
                assert all(ch.bmin[k] >= nd.bmin[k] and ch.bmax[k] <= nd.bmax[k] for k in range(3))


def test_opt_outs(built, monkeypatch):
    s = rtx.HostScene("random_spheres", 1)
    cam = s.camera(width=96, spp=1)
    assert rtx.walk_skip(s.desc, cam).any()
    assert not rtx.walk_skip(s.desc, cam, flags=rtx.RTX_SCENE_EVERY_BOX).any()
    monkeypatch.setenv("RTX_COLLAPSE", "0")
    assert not rtx.walk_skip(s.desc, cam).any()
    monkeypatch.delenv("RTX_COLLAPSE")
    # the reference tree can be collapsed too (its own skips, same node-entry count as its nodes)
    m = rtx.walk_skip(s.desc, cam, flags=rtx.RTX_SCENE_REFERENCE_BVH)
    assert m.any() and len(m) == s.desc.contents.n_nodes


def test_boxes_that_do_not_nest_keep_their_test(built):
    """A hand-made table whose root box is smaller than its children's: the root keeps its test
    (leaving it out would test spheres the reference never reaches)."""
    s = rtx.HostScene("random_spheres", 1)
    cam = s.camera(width=96, spp=1)
    d = s.desc.contents
    nodes = (rtx.BvhNode * d.n_nodes)()
    ctypes.memmove(nodes, d.nodes, ctypes.sizeof(rtx.BvhNode) * d.n_nodes)
    root = d.roots[0]
    base = rtx.walk_skip(s.desc, cam, flags=rtx.RTX_SCENE_REFERENCE_BVH)
    assert base[0] == 1  # the reference's root passes almost always: left out
    nodes[root].bmax[0] = nodes[root].bmin[0] + 1.0  # no longer holds its children
    w = rtx.desc_with_tree(s.desc, nodes, d.n_nodes, root)
    m = rtx.walk_skip(w, cam, flags=rtx.RTX_SCENE_REFERENCE_BVH)
    assert m[0] == 0
    a, ca, b, cb = oracle_pair(w, w, cam, 3, rtx.node_skip(w, m))
    assert np.array_equal(a, b) and all(ca[k] == cb[k] for k in PATH)


@pytest.mark.parametrize("seed,n_spheres,n_quads,axis_aligned", [(2, 40, 14, False), (3, 200, 30, True), (4, 8, 0, True)])
def test_hand_made_scenes(built, seed, n_spheres, n_quads, axis_aligned):
    """test_random_scenes' tables (quads, degenerate quads, tiny spheres, a camera looking down an
    axis: zero direction components) on the oracle, collapsed against full."""
    from test_random_scenes import build_scene, camera

    d = build_scene(seed, n_spheres, n_quads)
    cam = camera(seed, 64, 36, 4, axis_aligned)
    pd = ctypes.pointer(d)
    walk = rtx.walk_tree_desc(pd, cam)
    skip = rtx.walk_skip(pd, cam)
    a, ca, b, cb = oracle_pair(pd, walk, cam, seed, rtx.node_skip(walk, skip))
    assert np.array_equal(a, b, equal_nan=True)
    assert all(ca[k] == cb[k] for k in PATH)
