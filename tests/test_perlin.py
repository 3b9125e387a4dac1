"""Perlin NoiseTexture: Go math.Sin restatement, the noise against an
independent numpy restatement, host tables, perlinDemo / simpleLightDemo GPU parity.

Reference: internal/materials.go:195-295 (Perlin, Noise, Turb, Permute, NoiseTexture),
math.go:58-92 (Lerp, BiLinearLerp, TriLinearLerp), main.go:106-130 and 162-192.
Go's math.Sin is the pure-Go sin.go / trig_reduce.go of Go 1.21 (Go is absent here:
parity with the Go binary is unpinned; the restatement is checked against libm to 1 ulp).
"""
import ctypes
import math

import numpy as np
import pytest

import oracle_binding as ob
import rtx
from parity import check_scene

f32 = np.float32


def ulp_diff(a: float, b: float) -> int:
    ia = np.frombuffer(np.float64(a).tobytes(), np.int64)[0]
    ib = np.frombuffer(np.float64(b).tobytes(), np.int64)[0]
    return abs(int(ia) - int(ib))


def test_go_sin_special_values(built):
    L = ob.load()
    assert L.oracle_go_sin(0.0) == 0.0 and math.copysign(1, L.oracle_go_sin(-0.0)) == -1
    assert math.isnan(L.oracle_go_sin(float("nan"))) and math.isnan(L.oracle_go_sin(float("inf")))
    assert L.oracle_go_sin(math.pi / 2) == 1.0


@pytest.mark.parametrize("lo,hi", [(-10.0, 10.0), (-1e4, 1e4)])
def test_go_sin_within_one_ulp_of_libm(built, lo, hi):
    """The Cody-Waite range (below 2^29, every argument the Perlin scenes produce)
    tracks libm to 1 ulp."""
    L = ob.load()
    rng = np.random.default_rng(int(abs(lo)) + 7)
    xs = rng.uniform(lo, hi, 4000)
    worst = max(ulp_diff(L.oracle_go_sin(float(x)), math.sin(float(x))) for x in xs)
    assert worst <= 1


@pytest.mark.parametrize("lo,hi", [(2.0**29, 2.0**40), (1e15, 1e300)])
def test_go_sin_payne_hanek_absolute(built, lo, hi):
    """trigReduce (>= 2^29) keeps ~53 bits of the reduced argument, so Go's result is
    within a few 1e-16 of libm in absolute terms (not in ulps near a zero of sin)."""
    L = ob.load()
    rng = np.random.default_rng(int(math.log2(lo)))
    xs = np.exp(rng.uniform(math.log(lo), math.log(hi), 4000))
    worst = max(abs(L.oracle_go_sin(float(x)) - math.sin(float(x))) for x in xs)
    assert worst <= 4.5e-16


def perlin_table(host):
    d = host.desc.contents
    tex = [d.textures[i] for i in range(d.n_textures)]
    noise = [t for t in tex if t.type == rtx.RTX_TEX_NOISE]
    assert len(noise) == 1
    t = noise[0]
    tab = np.ctypeslib.as_array(d.texels, shape=(d.n_texels,))[t.texel_offset:t.texel_offset + 1536].copy()
    return tab, float(t.scale)


def test_host_perlin_tables(built):
    host = rtx.HostScene("perlin_demo", 1)
    tab, scale = perlin_table(host)
    assert scale == 4.0
    grads = tab[:768].view(np.float32)
    assert ((grads >= -1) & (grads < 1)).all()
    for k in range(3):
        assert sorted(tab[768 + 256 * k: 1024 + 256 * k].tolist()) == list(range(256))
    # permutations differ (three Permute calls on the advancing global stream)
    assert not np.array_equal(tab[768:1024], tab[1024:1280])


def numpy_noise_texture(tab, scale, p):
    """materials.go:218-288 restated a third time, float32 step by step."""
    g = tab[:768].view(np.float32).reshape(256, 3)
    px, py, pz = f32(p[0]) * f32(scale), f32(p[1]) * f32(scale), f32(p[2]) * f32(scale)
    z0 = pz

    def lerp(t, x, y):
        return f32(f32(x * f32(f32(1) - t)) + f32(y * t))

    def corner(ix, iy, iz, x, y, z):
        h = int(tab[768 + ix]) ^ int(tab[1024 + iy]) ^ int(tab[1280 + iz])
        return f32(f32(f32(g[h, 0] * x) + f32(g[h, 1] * y)) + f32(g[h, 2] * z))

    total, weight = f32(0), f32(1)
    for _ in range(7):
        xi, yi, zi = (f32(math.floor(float(v))) for v in (px, py, pz))
        tx, ty, tz = f32(px - xi), f32(py - yi), f32(pz - zi)
        rx0, ry0, rz0 = (int(v) & 255 for v in (xi, yi, zi))
        rx1, ry1, rz1 = (rx0 + 1) & 255, (ry0 + 1) & 255, (rz0 + 1) & 255
        o = f32(1)
        c = {}
        for a, ix, x in ((0, rx0, tx), (1, rx1, f32(tx - o))):
            for b, iy, y in ((0, ry0, ty), (1, ry1, f32(ty - o))):
                for cc, iz, z in ((0, rz0, tz), (1, rz1, f32(tz - o))):
                    c[(a, b, cc)] = corner(ix, iy, iz, x, y, z)
        sm = [f32(f32(t * t) * f32(f32(3) - f32(f32(2) * t))) for t in (tx, ty, tz)]
        e = lerp(sm[1], lerp(sm[0], c[0, 0, 0], c[1, 0, 0]), lerp(sm[0], c[0, 1, 0], c[1, 1, 0]))
        f = lerp(sm[1], lerp(sm[0], c[0, 0, 1], c[1, 0, 1]), lerp(sm[0], c[0, 1, 1], c[1, 1, 1]))
        total = f32(total + f32(weight * lerp(sm[2], e, f)))
        weight = f32(weight * f32(0.5))
        px, py, pz = f32(px * f32(2)), f32(py * f32(2)), f32(pz * f32(2))
    turb = f32(abs(float(total)))
    s = f32(ob.load().oracle_go_sin(float(f32(z0 + f32(f32(10) * turb)))))
    return f32(f32(0.5) * f32(f32(1) + s))


def test_oracle_noise_texture_matches_numpy(built):
    host = rtx.HostScene("perlin_demo", 1)
    tab, scale = perlin_table(host)
    T = (ctypes.c_uint32 * 1536)(*tab.tolist())
    rng = np.random.default_rng(3)
    pts = np.concatenate([rng.uniform(-3, 3, (150, 3)), rng.uniform(-300, 300, (50, 3)),
                          np.array([[0, 0, 0], [-1e-3, 2, 0.5], [255.5, -256.25, 1e4]])]).astype(np.float32)
    for p in pts:
        got = ob.load().oracle_noise_texture(T, scale, (ctypes.c_float * 3)(*p.tolist()))
        assert f32(got) == numpy_noise_texture(tab, scale, p), p


def test_scene_shapes(built):
    ha = rtx.HostScene("perlin_demo", 1)
    a = ha.desc.contents
    assert a.n_spheres == 2 and a.n_quads == 0
    b = rtx.HostScene("simple_light_demo", 1)
    d = b.desc.contents
    assert d.n_spheres == 4
    assert sorted(d.materials[i].type for i in range(d.n_materials)) == [
        rtx.RTX_MAT_LAMBERTIAN, rtx.RTX_MAT_LAMBERTIAN, rtx.RTX_MAT_DIFFUSE_LIGHT]
    cam = b.camera()
    assert (cam.image_width, cam.samples_per_pixel) == (400, 500) and list(cam.background) == [0, 0, 0]


def test_oracle_perlin_orders_agree(built):
    s = rtx.HostScene("simple_light_demo", 1)
    cam = s.camera(spp=3)
    reg = rtx.Region(190, 100, 12, 8, 0, 1)
    ref, cref = ob.render(s.desc, cam, 4, reg, ob.ORDER_REFERENCE)
    it, cit = ob.render(s.desc, cam, 4, reg, ob.ORDER_ITERATIVE)
    assert np.isfinite(ref).all() and cref == cit
    assert float(np.abs(ref - it).max()) <= 1e-4


# ---------------------------------------------------------------------------------------
# GPU parity
# ---------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    torch.cuda.set_device(0)
    return torch


def gpu_check(torch, scene, cam, seed, reg, flags=0):
    """Both kernels (timed and counting) vs the oracle (tests/parity.py)."""
    desc = scene.desc
    check_scene(torch, rtx.DeviceScene(desc), desc, cam, seed, reg, flags=flags)


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, 64, rtx.RTX_FLAG_NO_LDS], ids=["v3", "removed-v1-flag", "global"])
def test_gpu_perlin_demo_full(torch_cuda, built, flags):
    """perlinDemo at 400x225x4 spp (the flag bit of the removed v1 schedule is ignored)."""
    s = rtx.HostScene("perlin_demo", 1)
    cam = s.camera(spp=4)
    gpu_check(torch_cuda, s, cam, 2, rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1), flags)


@pytest.mark.gpu
def test_gpu_simple_light_crop_full_spp(torch_cuda, built):
    """A 40x24 window of simpleLightDemo at its 500 spp (noise, red sphere, light)."""
    s = rtx.HostScene("simple_light_demo", 1)
    cam = s.camera()
    gpu_check(torch_cuda, s, cam, 6, rtx.Region(170, 95, 40, 24, 0, 1))
