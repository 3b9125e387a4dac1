"""The C-ABI boundary on the CPU: librtx.so / librtxhost.so load and export every symbol
their headers declare, and argument validation (which runs before any device call)
returns the documented error codes.  No compute call is made without a GPU."""
import ctypes
import os
import re

import pytest

import rtx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(header: str):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b((?:rtx|rtxhost)_[a-z_]+)\s*\(", text)) - {"rtx_region_rows_"})


@pytest.mark.parametrize("header,lib", [("rtx.h", "librtx.so"), ("rtx_host.h", "librtxhost.so")])
def test_exports_every_declared_symbol(built, header, lib):
    names = declared_functions(header)
    assert names, header
    L = ctypes.CDLL(os.path.join(ROOT, "raytracer-go_amd", lib))
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_binding_lists_match_headers(built):
    assert sorted(rtx.RTX_SYMBOLS) == declared_functions("rtx.h")
    assert sorted(rtx.RTXHOST_SYMBOLS) == declared_functions("rtx_host.h")


def test_version_and_build_info(built):
    L = rtx.load()
    assert L.rtx_version() == 10
    assert b"gfx950" in L.rtx_build_info()


def test_struct_layout_matches_header(built, tmp_path):
    """The ctypes mirror (what a cgo binding would also mirror) has the C header's sizes."""
    import subprocess

    structs = {"rtx_bvh_node": rtx.BvhNode, "rtx_sphere": rtx.Sphere, "rtx_quad": rtx.Quad,
               "rtx_material": rtx.Material, "rtx_texture": rtx.Texture, "rtx_scene_desc": rtx.SceneDesc, "rtx_list": rtx.List,
               "rtx_camera": rtx.Camera, "rtx_region": rtx.Region, "rtx_stats": rtx.Stats}
    src = tmp_path / "sizes.c"
    src.write_text('#include <stdio.h>\n#include "rtx.h"\nint main(void){\n' +
                   "".join(f'printf("%zu\\n", sizeof({n}));\n' for n in structs) + "return 0;}\n")
    exe = tmp_path / "sizes"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    sizes = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    for (name, cls), size in zip(structs.items(), sizes):
        assert ctypes.sizeof(cls) == size, name
    assert ctypes.sizeof(rtx.BvhNode) == 32 and ctypes.sizeof(rtx.Sphere) == 32


def make_desc(spheres, materials, textures, nodes=(), roots=None, quads=0):
    S = (rtx.Sphere * max(1, len(spheres)))(*spheres)
    M = (rtx.Material * max(1, len(materials)))(*materials)
    T = (rtx.Texture * max(1, len(textures)))(*textures)
    N = (rtx.BvhNode * max(1, len(nodes)))(*nodes)
    roots = roots if roots is not None else [rtx.ref_prim(rtx.RTX_PRIM_SPHERE, i) for i in range(len(spheres))]
    R = (ctypes.c_int32 * max(1, len(roots)))(*roots)
    d = rtx.SceneDesc()
    d.nodes, d.n_nodes = N, len(nodes)
    d.roots, d.n_roots = R, len(roots)
    d.spheres, d.n_spheres = S, len(spheres)
    d.materials, d.n_materials = M, len(materials)
    d.textures, d.n_textures = T, len(textures)
    d.n_quads = quads
    d._keep = (S, M, T, N, R)
    return d


def sphere(mat=0):
    s = rtx.Sphere()
    s.center[:] = [0, 0, -1]
    s.radius = 0.5
    s.material = mat
    return s


def lambertian(tex=0):
    m = rtx.Material()
    m.type = rtx.RTX_MAT_LAMBERTIAN
    m.texture = tex
    return m


def texture(kind=rtx.RTX_TEX_SOLID):
    t = rtx.Texture()
    t.type = kind
    return t


def create(d):
    h = ctypes.c_void_p()
    rc = rtx.load().rtx_scene_create(ctypes.byref(d), ctypes.byref(h))
    if rc == 0:
        rtx.load().rtx_scene_destroy(h)
    return rc, rtx.load().rtx_last_error().decode()


def test_null_arguments(built):
    L = rtx.load()
    h = ctypes.c_void_p()
    assert L.rtx_scene_create(None, ctypes.byref(h)) == rtx.RTX_ERR_INVALID_ARG
    assert L.rtx_render(None, None, 0, 1, None, None) == rtx.RTX_ERR_INVALID_ARG
    L.rtx_scene_destroy(None)  # no-op


def test_noise_texture_validation(built):
    """Perlin textures are on the GPU path; their RTX_NOISE_TEXELS tables must exist."""
    rc, msg = create(make_desc([sphere()], [lambertian()], [texture(rtx.RTX_TEX_NOISE)]))
    assert rc == rtx.RTX_ERR_INVALID_ARG and "Perlin tables out of range" in msg


def test_quad_validation(built):
    """Quads are on the GPU path (hittables.go:138-216); bad tables are rejected."""
    rc, msg = create(make_desc([sphere()], [lambertian()], [texture()], quads=1))
    assert rc == rtx.RTX_ERR_INVALID_ARG and "quads is NULL" in msg
    q = rtx.Quad()
    q.material = 5
    Q = (rtx.Quad * 1)(q)
    d = make_desc([sphere()], [lambertian()], [texture()], quads=1)
    d.quads = Q
    rc, msg = create(d)
    assert rc == rtx.RTX_ERR_INVALID_ARG and "quad 0 material" in msg
    q.material = 0
    Q = (rtx.Quad * 1)(q)
    d = make_desc([sphere()], [lambertian()], [texture()], quads=1,
                  roots=[rtx.ref_prim(rtx.RTX_PRIM_QUAD, 1)])
    d.quads = Q
    rc, msg = create(d)
    assert rc == rtx.RTX_ERR_INVALID_ARG and "quad ref 1 out of range" in msg


def test_material_out_of_range(built):
    rc, msg = create(make_desc([sphere(mat=3)], [lambertian()], [texture()]))
    assert rc == rtx.RTX_ERR_INVALID_ARG and "material" in msg


def test_texture_out_of_range(built):
    rc, msg = create(make_desc([sphere()], [lambertian(tex=2)], [texture()]))
    assert rc == rtx.RTX_ERR_INVALID_ARG


def test_bad_refs_and_cycles(built):
    n0 = rtx.BvhNode()
    n0.left, n0.right = 1, rtx.ref_prim(0, 0)
    n1 = rtx.BvhNode()
    n1.left, n1.right = 0, rtx.ref_prim(0, 0)  # cycle 0 -> 1 -> 0
    rc, msg = create(make_desc([sphere()], [lambertian()], [texture()], nodes=[n0, n1], roots=[0]))
    assert rc == rtx.RTX_ERR_INVALID_ARG and "cycle" in msg
    rc, _ = create(make_desc([sphere()], [lambertian()], [texture()], roots=[rtx.ref_prim(0, 5)]))
    assert rc == rtx.RTX_ERR_INVALID_ARG
    rc, _ = create(make_desc([sphere()], [lambertian()], [texture()], roots=[7]))
    assert rc == rtx.RTX_ERR_INVALID_ARG


def test_empty_scene(built):
    rc, _ = create(make_desc([sphere()], [lambertian()], [texture()], roots=[]))
    assert rc == rtx.RTX_ERR_INVALID_ARG


def gpu_present():
    return rtx.load().rtx_device_count() > 0


def test_valid_scene_without_gpu_reports_no_device(built):
    if gpu_present():
        pytest.skip("a GPU is visible")
    rc, msg = create(make_desc([sphere()], [lambertian()], [texture()]))
    assert rc in (rtx.RTX_ERR_NO_DEVICE, rtx.RTX_ERR_HIP, rtx.RTX_ERR_OOM), (rc, msg)
    assert msg


def test_ref_prim_encoding():
    assert rtx.ref_prim(0, 0) == -1
    assert rtx.ref_prim(0, 5) == ~5
    assert rtx.ref_prim(1, 3) == ~((1 << 28) | 3)


def test_image_texture_validation(built):
    """RTX_TEX_IMAGE holds width*height RGBA16 texels (2 words each) plus the border texel,
    at an even word offset (include/rtx.h)."""
    t = texture(rtx.RTX_TEX_IMAGE)
    t.width, t.height = 2, 2
    words = (ctypes.c_uint32 * 10)()
    d = make_desc([sphere()], [lambertian()], [t])
    d.texels, d.n_texels = words, 8  # the raster without its border texel
    rc, msg = create(d)
    assert rc == rtx.RTX_ERR_INVALID_ARG and "texels out of range" in msg
    t.texel_offset = 1
    d = make_desc([sphere()], [lambertian()], [t])
    d.texels, d.n_texels = words, 10
    rc, msg = create(d)
    assert rc == rtx.RTX_ERR_INVALID_ARG and "even" in msg
