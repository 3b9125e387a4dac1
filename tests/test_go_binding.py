"""The Go side of the drop-in boundary (go/internal/render_gpu.go), without a Go toolchain.

Go is not installed here or on the GPU box, so the cgo binding is checked two ways:
  - statically (CPU): every C identifier it names (functions, types, constants) is declared in
    include/rtx.h, every C call passes as many arguments as the prototype takes, and every field it
    sets or reads on an rtx.h struct exists (cgo spells a C field `type` as `_type`);
  - dynamically (GPU): the exact C-ABI call sequences the file issues — the flattened tree through
    rtx_scene_create + rtx_render_ppm + rtx_scene_destroy, and a World of spheres through
    rtx_scene_create_spheres(seed, draw0 = 0) + rtx_render_ppm — driven through ctypes with the tables
    the Go flattener builds (the C++ mirror's, raytracer-go_amd/host/flatten.cpp), held to the oracle.
"""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle_binding as ob
import rtx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = open(os.path.join(ROOT, "go", "internal", "render_gpu.go")).read()
HDR = open(os.path.join(ROOT, "include", "rtx.h")).read()

C_SCALARS = {"float", "int", "char", "uint32_t", "uint64_t", "int32_t", "GoString", "rtx_scene"}


def header_structs():
    """typedef struct name { fields } name; -> {name: set(field names)} from rtx.h."""
    out = {}
    for m in re.finditer(r"typedef struct (\w+)\s*\{(.*?)\}\s*(\w+);", HDR, re.S):
        body = re.sub(r"/\*.*?\*/", "", m.group(2), flags=re.S)
        fields = set()
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            for name in re.findall(r"(\w+)\s*(?:\[[^\]]*\])?\s*(?:,|$)", decl.split(None, 1)[1] if " " in decl else ""):
                fields.add(name)
        out[m.group(3)] = fields
    return out


def header_prototypes():
    """{function: number of parameters} of the rtx_* functions rtx.h declares."""
    out = {}
    flat = re.sub(r"/\*.*?\*/", "", HDR, flags=re.S)
    for m in re.finditer(r"\b(?:int|void|uint32_t|uint64_t|const char\*)\s+\*?(rtx_\w+)\(([^)]*)\);", flat):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else len(args.split(","))
    return out


def call_args(src, start):
    """The top-level comma-separated arguments of the call whose '(' is at src[start]."""
    depth, args, cur = 0, [], ""
    for ch in src[start:]:
        if ch in "([{":
            depth += 1
            if depth == 1:
                continue
        elif ch in ")]}":
            depth -= 1
            if depth == 0:
                if cur.strip():
                    args.append(cur)
                return args
        if ch == "," and depth == 1:
            args.append(cur)
            cur = ""
        else:
            cur += ch
    raise AssertionError("unbalanced call")


def test_every_c_identifier_is_declared():
    names = set(re.findall(r"\bC\.(\w+)", GO))
    missing = [n for n in sorted(names) if n not in C_SCALARS and not re.search(rf"\b{n}\b", HDR)]
    assert not missing, missing
    assert {"rtx_scene_create", "rtx_scene_create_spheres", "rtx_render_ppm", "rtx_render_ppm_ex", "rtx_scene_destroy",
            "rtx_last_error", "rtx_ppm_max_bytes"} <= names
    # several GPUs: the text is encoded on device 0 (rtx_render_ppm_ex), never formatted in Go
    assert "C.rtx_render(" not in GO and "ToGamma2()" not in GO


def test_c_calls_match_the_prototypes():
    protos = header_prototypes()
    seen = 0
    for m in re.finditer(r"\bC\.(rtx_\w+)\(", GO):
        fn = m.group(1)
        assert fn in protos, fn
        n = len(call_args(GO, m.end() - 1))
        assert n == protos[fn], (fn, n, protos[fn])
        seen += 1
    assert seen >= 7


def test_struct_fields_exist():
    structs = header_structs()
    # struct literals: C.rtx_xxx{field: ..., field: ...}
    for m in re.finditer(r"C\.(rtx_\w+)\{", GO):
        st = m.group(1)
        body = "".join(call_args(GO, m.end() - 1))
        keys = re.findall(r"(?:^|[\s,{])(\w+):", " " + body)
        for k in keys:
            assert k in structs[st], (st, k)
    # variables of an rtx.h struct type, per function: `var x C.rtx_xxx` then x.field
    for fn in re.split(r"\nfunc ", GO):
        types = dict(re.findall(r"\bvar (\w+) C\.(rtx_\w+)\b", fn))
        for var, st in types.items():
            for field in set(re.findall(rf"\b{var}\.(\w+)", fn)):
                name = "type" if field == "_type" else field
                assert name in structs[st], (st, field)


def test_options_and_hook_are_there():
    """The drop-in surface INTEGRATION.md documents: the camera options, the Render hook, the GPU-built
    BVH constructor, and the CPU fallback guard."""
    for sig in ("func WithGPUs(n int) CameraOpt", "func WithSeed(seed uint64) CameraOpt",
                "func (c *Camera) renderGPU(world Hittable, writer io.Writer) (bool, error)",
                "func NewBVHFromWorldGPU(w *World) Hittable",
                "func (c *Camera) RenderGPU(world Hittable, writer io.Writer, seed uint64, gpus int) error"):
        assert sig in GO, sig
    assert "cfg.fallback.Load()" in GO and "cfg.fallback.Store(true)" in GO


def oracle_ppm(rgb):
    h, w = rgb.shape[:2]
    return ("".join([f"P3\n{w} {h}\n255\n"] + [ob.ppm_pixel(px) + "\n" for px in rgb.reshape(-1, 3)])).encode()


def render_ppm(L, h, cam, seed):
    cap = int(L.rtx_ppm_max_bytes(cam.image_width, cam.image_height))
    buf = np.empty(cap, dtype=np.uint8)
    n = ctypes.c_uint64()
    rtx.check(L.rtx_render_ppm(h, ctypes.byref(cam), seed, buf.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(n),
                               None), "rtx_render_ppm")
    return buf[: n.value].tobytes()


def desc_from_export(entries: bytes, base_desc):
    """The scene description of a scene's threaded entries (rtx_scene_export: the reference walk's
    pre-order, a node's escape after its subtree; a one-element split's child once): its node table, and
    its sphere table rebuilt from the sphere entries (centre, radius, material; the GPU build numbers the
    spheres in pre-order, as the flattener does), with base_desc's materials and textures."""
    e = np.frombuffer(entries, np.uint32).reshape(-1, 8)
    fl = e.view(np.float32)
    sph = e[e[:, 7].view(np.int32) != -1]
    spheres = (rtx.Sphere * len(sph))()
    for row in sph:
        i = int(row[5])
        spheres[i].center = (ctypes.c_float * 3)(*[float(v) for v in row[:3].view(np.float32)])
        spheres[i].radius = float(row[3:4].view(np.float32)[0])
        spheres[i].material = int(row[7])
    n_spheres = len(sph)
    nodes = []

    def build(i):  # -> (ref, next entry)
        tag = int(e[i, 7].view(np.int32))
        if tag != -1:
            return rtx.ref_prim(rtx.RTX_PRIM_SPHERE, int(e[i, 5])), i + 1
        me = len(nodes)
        nodes.append(None)
        esc = int(e[i, 3])
        left, j = build(i + 1)
        right = left
        if j < esc:
            right, j = build(j)
        assert j == esc
        nodes[me] = (fl[i, 0:3].copy(), fl[i, 4:7].copy(), left, right)
        return me, esc

    root, end = build(0)
    assert end == len(e)
    arr = (rtx.BvhNode * len(nodes))()
    for k, (lo, hi, left, right) in enumerate(nodes):
        arr[k].bmin = (ctypes.c_float * 3)(*[float(v) for v in lo])
        arr[k].bmax = (ctypes.c_float * 3)(*[float(v) for v in hi])
        arr[k].left, arr[k].right = left, right
    p = rtx.desc_with_tree(base_desc, arr, len(nodes), root)
    p.contents.spheres = ctypes.cast(spheres, ctypes.POINTER(rtx.Sphere))
    p.contents.n_spheres = n_spheres
    p._keep = p._keep + (spheres,)
    return p


@pytest.fixture(scope="module")
def gpu(built):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    torch.cuda.set_device(0)
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["random_spheres", "cornell_box"])
def test_go_sequence_flattened_tree(gpu, scene):
    """renderOnDevices(gpus = 1) for a flattened tree: rtx_scene_create(&desc) -> rtx_render_ppm(scene,
    &cam, seed, text, cap, &n, NULL) -> rtx_scene_destroy; the P3 bytes are the oracle's Render output."""
    L = rtx.load()
    host = rtx.HostScene(scene, 1)
    cam = host.camera(width=96, spp=4)
    h = ctypes.c_void_p()
    rtx.check(L.rtx_scene_create(host.desc, ctypes.byref(h)), "rtx_scene_create")
    try:
        text = render_ppm(L, h, cam, 2024)
    finally:
        L.rtx_scene_destroy(h)
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    want, _ = ob.render(host.desc, cam, 2024, reg, ob.ORDER_ITERATIVE)
    assert text == oracle_ppm(want)


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["random_spheres", "stress_100k"])
def test_go_sequence_gpu_bvh(gpu, scene):
    """renderOnDevices for NewBVHFromWorldGPU(world): rtx_scene_create_spheres(spheres in Add order,
    materials, textures, texels, seed, draw0 = 0, &scene, NULL) -> rtx_render_ppm -> rtx_scene_destroy.
    The tree the device built (exported) is a NewBVH tree over every sphere once, and the P3 bytes are the
    oracle's Render output walking that tree."""
    L = rtx.load()
    host = rtx.HostScene(scene, 1)
    arr, n, _, _ = host.world_spheres()
    d = host.desc.contents
    cam = host.camera(width=64, spp=2)
    h = ctypes.c_void_p()
    rtx.check(L.rtx_scene_create_spheres(arr, n, d.materials, d.n_materials, d.textures, d.n_textures, d.texels,
                                         d.n_texels, 2024, 0, ctypes.byref(h), None), "rtx_scene_create_spheres")
    dev = rtx.DeviceScene(handle=h)
    try:
        text = render_ppm(L, h, cam, 2024)
        tree = desc_from_export(dev.export(), host.desc)
    finally:
        dev.close()
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    want, _ = ob.render(tree, cam, 2024, reg, ob.ORDER_ITERATIVE)
    assert text == oracle_ppm(want)


@pytest.mark.gpu
def test_go_sequence_several_gpus(gpu):
    """renderOnDevices(gpus > 1): rtx_scene_create(&desc) -> rtx_render_ppm_ex(scene, &cam, seed, gpus, text,
    cap, &n, NULL) -> rtx_scene_destroy, with no host formatting.  On a one-GPU box the same entry renders 8
    simulated bands on device 0 (RTX_SIM_BANDS=8: the rows of an 8-GPU node, assembled by the de-interleave
    kernel) and encodes them there; the P3 bytes are the oracle's Render output."""
    import os

    L = rtx.load()
    host = rtx.HostScene("random_spheres", 1)
    cam = host.camera(width=96, spp=4)
    h = ctypes.c_void_p()
    rtx.check(L.rtx_scene_create(host.desc, ctypes.byref(h)), "rtx_scene_create")
    cap = int(L.rtx_ppm_max_bytes(cam.image_width, cam.image_height))
    buf = np.empty(cap, dtype=np.uint8)
    n = ctypes.c_uint64()
    os.environ["RTX_SIM_BANDS"] = "8"
    try:
        rtx.check(L.rtx_render_ppm_ex(h, ctypes.byref(cam), 2024, 1, buf.ctypes.data_as(ctypes.c_void_p), cap,
                                      ctypes.byref(n), None), "rtx_render_ppm_ex")
    finally:
        os.environ.pop("RTX_SIM_BANDS", None)
        L.rtx_scene_destroy(h)
    reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
    want, _ = ob.render(host.desc, cam, 2024, reg, ob.ORDER_ITERATIVE)
    assert buf[: n.value].tobytes() == oracle_ppm(want)
