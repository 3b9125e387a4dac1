"""Quad / Box / DiffuseLight: host mirror, oracle KATs, GPU parity.

Reference: internal/hittables.go:138-216 (NewQuad, Quad.Hit, InPlane, Box),
materials.go:297-313 (DiffuseLight), ray.go:41-50 (emission), main.go:132-160 (quadDemo)
and main.go:194-225 (cornellBox, the scene main.go:55 selects).
"""
import ctypes

import numpy as np
import pytest

import oracle_binding as ob
import rtx
from parity import check_scene, gpu_region

f32 = np.float32


def go_cross(l, r):  # vec3.go:129-135, float32 ops
    return np.array([l[1] * r[2] - l[2] * r[1], l[2] * r[0] - l[0] * r[2], l[0] * r[1] - l[1] * r[0]], dtype=f32)


def go_dot(l, r):  # vec3.go:137-139, left to right
    return f32(f32(f32(l[0] * r[0]) + f32(l[1] * r[1])) + f32(l[2] * r[2]))


def go_unit(v):  # vec3.go:103-113: v * (1 / sqrt(lensq))
    l = np.sqrt(go_dot(v, v))
    inv = f32(f32(1) / l)
    return np.array([v[0] * inv, v[1] * inv, v[2] * inv], dtype=f32)


def quads_of(desc):
    d = desc.contents
    return [d.quads[i] for i in range(d.n_quads)]


def test_cornell_box_scene_shape(built):
    s = rtx.HostScene("cornell_box", 1)
    d = s.desc.contents
    assert d.n_quads == 18 and d.n_spheres == 0  # 6 walls/light + 2 Boxes x 6
    mats = [d.materials[i] for i in range(d.n_materials)]
    assert sorted(m.type for m in mats) == [rtx.RTX_MAT_LAMBERTIAN] * 3 + [rtx.RTX_MAT_DIFFUSE_LIGHT]
    light = next(m for m in mats if m.type == rtx.RTX_MAT_DIFFUSE_LIGHT)
    assert list(d.textures[light.texture].even) == [15.0, 15.0, 15.0]
    cam = s.camera()
    assert (cam.image_width, cam.image_height, cam.samples_per_pixel, cam.max_depth) == (600, 600, 200, 50)
    assert list(cam.background) == [0.0, 0.0, 0.0]
    demo = rtx.HostScene("quad_demo", 1)
    assert demo.desc.contents.n_quads == 5


@pytest.mark.parametrize("scene", ["cornell_box", "quad_demo"])
def test_quad_fields_are_newquads(built, scene):
    """normal = Unit(u x v), D = normal . Q, w = n / (n . n), as float32 (hittables.go:149-165)."""
    host = rtx.HostScene(scene, 1)  # owns the tables the structs point into
    for q in quads_of(host.desc):
        Q, u, v = (np.array(list(x), dtype=f32) for x in (q.q, q.u, q.v))
        n = go_cross(u, v)
        norm = go_unit(n)
        inv = f32(f32(1) / go_dot(n, n))
        w = np.array([n[0] * inv, n[1] * inv, n[2] * inv], dtype=f32)
        assert np.array_equal(np.array(list(q.normal), dtype=f32), norm)
        assert np.array_equal(np.array(list(q.w), dtype=f32), w)
        assert f32(q.d) == go_dot(norm, Q)


def test_quad_bounds_contain_quads(built):
    """Every quad lies inside each BVH node above it (padded Aabb, bvh.go:63-82)."""
    host = rtx.HostScene("cornell_box", 1)
    d = host.desc.contents
    def corners(q):
        Q, u, v = (np.array(list(x), dtype=np.float64) for x in (q.q, q.u, q.v))
        return np.array([Q, Q + u, Q + v, Q + u + v])
    def walk(ref, boxes):
        if ref >= 0:
            n = d.nodes[ref]
            b = (np.array(list(n.bmin)), np.array(list(n.bmax)))
            walk(n.left, boxes + [b])
            walk(n.right, boxes + [b])
            return
        p = (~ref) & 0xFFFFFFFF
        assert p >> 28 == rtx.RTX_PRIM_QUAD
        c = corners(d.quads[p & 0x0FFFFFFF])
        for lo, hi in boxes:
            assert (c >= lo - 1e-3).all() and (c <= hi + 1e-3).all()
    for i in range(d.n_roots):
        walk(d.roots[i], [])


def light_panel(emit=(1.0, 2.0, 3.0)):
    """One DiffuseLight quad, the whole world (a World list root): z = 0 plane,
    x, y in [-1, 1], facing a camera on +z."""
    quad = rtx.Quad()
    Q, u, v = np.array([-1, -1, 0], f32), np.array([2, 0, 0], f32), np.array([0, 2, 0], f32)
    n = go_cross(u, v)
    norm = go_unit(n)
    inv = f32(f32(1) / go_dot(n, n))
    quad.q[:] = list(Q)
    quad.u[:] = list(u)
    quad.v[:] = list(v)
    quad.w[:] = [float(n[0] * inv), float(n[1] * inv), float(n[2] * inv)]
    quad.normal[:] = list(norm)
    quad.d = float(go_dot(norm, Q))
    quad.material = 0
    tex = rtx.Texture()
    tex.type = rtx.RTX_TEX_SOLID
    tex.even[:] = list(emit)
    mat = rtx.Material()
    mat.type = rtx.RTX_MAT_DIFFUSE_LIGHT
    mat.texture = 0
    keep = dict(quads=(rtx.Quad * 1)(quad), mats=(rtx.Material * 1)(mat), texs=(rtx.Texture * 1)(tex),
                roots=(rtx.c_int32 * 1)(rtx.ref_prim(rtx.RTX_PRIM_QUAD, 0)))
    d = rtx.SceneDesc()
    d.n_nodes = 0
    d.n_roots = 1
    d.roots = keep["roots"]
    d.n_quads = 1
    d.quads = keep["quads"]
    d.n_materials = 1
    d.materials = keep["mats"]
    d.n_textures = 1
    d.textures = keep["texs"]
    return ctypes.pointer(d), keep


def light_panel_camera(width=32, spp=1):
    return ob.camera(f32(1.0), width, samples_per_pixel=spp, max_depth=50, look_from=(0, 0, 4), look_at=(0, 0, 0),
                     fov_degrees=40, defocus_degrees=0, background=(0, 0, 0))


def test_oracle_light_panel_kat(built):
    """A lit quad seen head-on: covered pixels are exactly its emission (DiffuseLight
    never scatters, ray.go:45-47), the rest the background; one prim test per sample."""
    desc, keep = light_panel()
    cam = light_panel_camera()
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    img, cnt = ob.render(desc, cam, 3, reg, ob.ORDER_REFERENCE)
    lit = (img == np.array([1, 2, 3], f32)).all(axis=2)
    dark = (img == 0).all(axis=2)
    assert (lit | dark).all()
    # tan(20 deg) * 4 = 1.456: the panel spans +-1 / 1.456 of the half image = 22 px of 32
    assert lit[16, 16] and lit[6, 6] and lit[25, 25] and not lit[1, 1] and not lit[30, 16]
    assert 18 * 18 <= lit.sum() <= 24 * 24
    assert cnt["prim_tests"] == cnt["segments"] == 32 * 32 and cnt["hits"] == lit.sum()
    assert cnt["node_visits"] == 0


def test_oracle_quad_demo_runs(built):
    """quadDemo at 8x8 crop x 4 spp: finite, both colour orders within 1e-4."""
    s = rtx.HostScene("quad_demo", 1)
    cam = s.camera(spp=4)
    reg = rtx.Region(180, 90, 16, 8, 0, 1)
    ref, cref = ob.render(s.desc, cam, 5, reg, ob.ORDER_REFERENCE)
    it, cit = ob.render(s.desc, cam, 5, reg, ob.ORDER_ITERATIVE)
    assert np.isfinite(ref).all() and cref == cit
    assert float(np.abs(ref - it).max()) <= 1e-4
    assert cref["prim_tests"] > 0 and cref["hits"] > 0


# ---------------------------------------------------------------------------------------
# GPU parity (through the C-ABI)
# ---------------------------------------------------------------------------------------
TOL = 1e-4


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    torch.cuda.set_device(0)
    return torch


def gpu_check(torch, desc, cam, seed, reg, flags=0):
    """Both kernels (timed and counting) vs the oracle (tests/parity.py); (timed image, stats)."""
    dev = rtx.DeviceScene(desc)
    gpu, st, _ = check_scene(torch, dev, desc, cam, seed, reg, flags=flags)
    return gpu, st


@pytest.mark.gpu
def test_gpu_light_panel(torch_cuda, built):
    desc, keep = light_panel()
    cam = light_panel_camera(spp=4)
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    gpu, st = gpu_check(torch_cuda, desc, cam, 3, reg)


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, rtx.RTX_FLAG_NO_LDS], ids=["v3", "v3-global"])
def test_gpu_quad_demo_full(torch_cuda, built, flags):
    s = rtx.HostScene("quad_demo", 1)
    cam = s.camera(spp=8)
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    gpu, st = gpu_check(torch_cuda, s.desc, cam, 7, reg, flags)


@pytest.mark.gpu
def test_gpu_cornell_box_crop_full_spp(torch_cuda, built):
    """A 48x32 window of the 600x600x200 cornellBox config (box edge, light, walls)."""
    s = rtx.HostScene("cornell_box", 1)
    cam = s.camera()
    assert cam.samples_per_pixel == 200
    reg = rtx.Region(250, 60, 48, 32, 0, 1)
    gpu, st = gpu_check(torch_cuda, s.desc, cam, 11, reg)


@pytest.mark.gpu
def test_gpu_cornell_box_full_low_spp_and_shards(torch_cuda, built):
    s = rtx.HostScene("cornell_box", 1)
    cam = s.camera(spp=2)
    reg = rtx.Region(0, 0, 600, 600, 0, 1)
    gpu, st = gpu_check(torch_cuda, s.desc, cam, 13, reg)
    dev = rtx.DeviceScene(s.desc)
    got = np.full_like(gpu, np.nan)
    for rank in range(3):
        part, _ = gpu_region(torch_cuda, dev, cam, 13, rtx.Region(0, 0, 600, 600, rank, 3), counters=False)
        got[rank::3] = part
    assert np.array_equal(got, gpu)
