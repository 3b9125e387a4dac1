"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE (the checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes
import os
import sys
from ctypes import POINTER, c_char_p, c_float, c_int, c_int32, c_uint32, c_uint64, c_void_p

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "raytracer-go_amd")
if PKG not in sys.path:
    sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

import rtx  # noqa: E402

ORDER_REFERENCE = 0
ORDER_ITERATIVE = 1


class Counters(ctypes.Structure):
    _fields_ = [("samples", c_uint64), ("segments", c_uint64), ("node_visits", c_uint64),
                ("prim_tests_ref", c_uint64), ("prim_tests", c_uint64), ("hits", c_uint64),
                ("texel_fetches", c_uint64), ("rng_draws", c_uint64), ("texel_border", c_uint64)]

    def as_dict(self) -> dict:
        return {name: int(getattr(self, name)) for name, _ in self._fields_}


class CameraOpts(ctypes.Structure):
    _fields_ = [("samples_per_pixel", c_int32), ("max_depth", c_int32), ("fov_radians", c_float),
                ("look_from", c_float * 3), ("look_at", c_float * 3), ("vup", c_float * 3),
                ("defocus_radians", c_float), ("focus_dist", c_float), ("background", c_float * 3)]


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    path = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(path):
        raise OSError(f"{path} not built (make -C oracle)")
    L = ctypes.CDLL(path)
    L.oracle_philox4x32_10.argtypes = [POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32)]
    L.oracle_philox4x32_10.restype = None
    L.oracle_pixel_block.argtypes = [c_uint64, c_uint32, c_uint32, c_uint32, c_uint32, POINTER(c_uint32)]
    L.oracle_pixel_block.restype = None
    L.oracle_stream_u32.argtypes = [c_uint64, c_uint32, c_uint64]
    L.oracle_stream_u32.restype = c_uint32
    L.oracle_camera_defaults.argtypes = [POINTER(CameraOpts)]
    L.oracle_camera_defaults.restype = None
    L.oracle_to_radians.argtypes = [c_float]
    L.oracle_to_radians.restype = c_float
    L.oracle_camera_init.argtypes = [c_float, c_int32, POINTER(CameraOpts), POINTER(rtx.Camera)]
    L.oracle_camera_init.restype = None
    L.oracle_render.argtypes = [POINTER(rtx.SceneDesc), POINTER(rtx.Camera), c_uint64, POINTER(rtx.Region), c_int,
                                c_int, c_void_p, POINTER(Counters)]
    L.oracle_render.restype = c_int
    L.oracle_sample.argtypes = [POINTER(rtx.SceneDesc), POINTER(rtx.Camera), c_uint64, c_uint32, c_uint32, c_uint32,
                                c_int, POINTER(c_float), POINTER(Counters)]
    L.oracle_sample.restype = c_int
    L.oracle_ppm_pixel.argtypes = [POINTER(c_float), c_char_p]
    L.oracle_ppm_pixel.restype = c_int
    L.oracle_build_random_spheres.argtypes = [c_uint64]
    L.oracle_build_random_spheres.restype = c_void_p
    L.oracle_scene_desc.argtypes = [c_void_p]
    L.oracle_scene_desc.restype = POINTER(rtx.SceneDesc)
    L.oracle_scene_free.argtypes = [c_void_p]
    L.oracle_scene_free.restype = None
    L.oracle_region_rows.argtypes = [POINTER(rtx.Region)]
    L.oracle_region_rows.restype = c_uint32
    L.oracle_go_sin.argtypes = [ctypes.c_double]
    L.oracle_go_sin.restype = ctypes.c_double
    L.oracle_noise_texture.argtypes = [POINTER(c_uint32), c_float, POINTER(c_float)]
    L.oracle_noise_texture.restype = c_float
    L.oracle_ycbcr_rgba.argtypes = [ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8, POINTER(c_uint32)]
    L.oracle_ycbcr_rgba.restype = None
    L.oracle_ycbcr_rgba_all.argtypes = [c_void_p]
    L.oracle_ycbcr_rgba_all.restype = None
    L.oracle_ycbcr_texels.argtypes = [c_void_p, c_void_p, c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                      ctypes.c_int64, c_int, c_void_p]
    L.oracle_ycbcr_texels.restype = c_int
    L.oracle_node_hooks.argtypes = [c_void_p, c_void_p, c_void_p]
    L.oracle_node_hooks.restype = None
    L.oracle_tier.argtypes = [c_void_p, c_void_p, c_void_p]
    L.oracle_tier.restype = None
    L.oracle_sphere_rank.argtypes = [c_void_p]
    L.oracle_sphere_rank.restype = None
    L.oracle_near_slab_pass.argtypes = [c_void_p] * 7 + [c_uint64]
    L.oracle_near_slab_pass.restype = None
    _lib = L
    return L


def philox(ctr, key):
    L = load()
    C = (c_uint32 * 4)(*ctr)
    K = (c_uint32 * 2)(*key)
    O = (c_uint32 * 4)()
    L.oracle_philox4x32_10(C, K, O)
    return list(O)


def ycbcr_rgba(y: int, cb: int, cr: int):
    """color.YCbCr{y, cb, cr}.RGBA() (r, g, b) as the oracle restates it."""
    o = (c_uint32 * 3)()
    load().oracle_ycbcr_rgba(y, cb, cr, o)
    return tuple(o)


def ycbcr_rgba_all():
    """[2^24, 3] uint32: RGBA() of every (y, cb, cr), index y << 16 | cb << 8 | cr."""
    out = np.empty((1 << 24, 3), dtype=np.uint32)
    load().oracle_ycbcr_rgba_all(out.ctypes.data_as(c_void_p))
    return out


def ycbcr_texels(Y, Cb, Cr, w: int, h: int, ratio: int = 2):
    """The RTX_TEX_IMAGE words (RGBA16 raster + border) of an *image.YCbCr (0,0)-(w,h)."""
    cw = {0: w, 1: (w + 1) // 2, 2: (w + 1) // 2, 3: w, 4: (w + 3) // 4, 5: (w + 3) // 4}[ratio]
    Y, Cb, Cr = (np.ascontiguousarray(a, dtype=np.uint8) for a in (Y, Cb, Cr))
    out = np.empty(2 * (w * h + 1), dtype=np.uint32)
    rc = load().oracle_ycbcr_texels(Y.ctypes.data_as(c_void_p), Cb.ctypes.data_as(c_void_p),
                                    Cr.ctypes.data_as(c_void_p), w, h, w, cw, ratio, out.ctypes.data_as(c_void_p))
    if rc != 0:
        raise RuntimeError("oracle_ycbcr_texels rejected its arguments")
    return out


def region_rows(reg: rtx.Region) -> int:
    return int(load().oracle_region_rows(ctypes.byref(reg)))


def sphere_ranks(desc_ptr):
    """Each sphere's place in the reference walk of desc_ptr's tree (pre-order: roots in order, a
    node's left subtree then its right — once when left == right —, a nested World's items in
    order): the tie rule of a walk over another tree of the same spheres (oracle_sphere_rank)."""
    d = desc_ptr.contents
    rank = np.full(max(d.n_spheres, 1), 0xFFFFFFFF, np.uint32)
    k = 0
    for ri in range(d.n_roots):
        stack = [d.roots[ri]]
        while stack:
            ref = stack.pop()
            if ref >= 0:
                nd = d.nodes[ref]
                if nd.right != nd.left:
                    stack.append(nd.right)
                stack.append(nd.left)
                continue
            p = (~ref) & 0xFFFFFFFF
            typ, idx = p >> 28, p & 0x0FFFFFFF
            if typ == rtx.RTX_PRIM_LIST:
                lst = d.lists[idx]
                stack.extend(d.list_refs[lst.first + i] for i in reversed(range(lst.count)))
            elif typ == rtx.RTX_PRIM_SPHERE and rank[idx] == 0xFFFFFFFF:
                rank[idx] = k
            k += 1
    return rank


def render(desc_ptr, cam: rtx.Camera, seed: int, region: rtx.Region, order: int = ORDER_REFERENCE,
           threads: int = 0, skip=None, tier=None, rank=None):
    """Oracle render of a region -> (float32 array [rows, width, 3], counters dict).  skip: per node
    of desc_ptr's table, 1 = leave its box test out (a collapsed walk, rtx.node_skip).  tier: (near
    box, far description, far skip or None): the tiered walk (oracle_tier), desc_ptr being the near
    tree."""
    L = load()
    if rank is not None:  # the tie rule of a walk over a rebuilt tree (sphere_ranks of the caller's tree)
        rk = np.ascontiguousarray(rank, np.uint32)
        L.oracle_sphere_rank(rk.ctypes.data_as(c_void_p))
        try:
            return render(desc_ptr, cam, seed, region, order, threads, skip, tier)
        finally:
            L.oracle_sphere_rank(None)
    if tier is not None:
        box, far, fsk = tier
        boxa = (c_float * 6)(*box)
        fska = None if fsk is None else np.ascontiguousarray(fsk, np.uint8)
        L.oracle_tier(boxa, ctypes.cast(far, c_void_p), None if fska is None else fska.ctypes.data_as(c_void_p))
        try:
            return render(desc_ptr, cam, seed, region, order, threads, skip)
        finally:
            L.oracle_tier(None, None, None)
    if threads <= 0:
        threads = min(16, os.cpu_count() or 1)
    rows = region_rows(region)
    out = np.zeros((rows, region.width, 3), dtype=np.float32)
    cnt = Counters()
    sk = None if skip is None else np.ascontiguousarray(skip, np.uint8)
    if sk is not None:
        assert len(sk) >= desc_ptr.contents.n_nodes
        L.oracle_node_hooks(None, None, sk.ctypes.data_as(c_void_p))
    try:
        rc = L.oracle_render(desc_ptr, ctypes.byref(cam), seed, ctypes.byref(region), order, threads,
                             out.ctypes.data_as(c_void_p), ctypes.byref(cnt))
    finally:
        if sk is not None:
            L.oracle_node_hooks(None, None, None)
    if rc != 0:
        raise RuntimeError("oracle_render rejected its arguments")
    return out, cnt.as_dict()


def sample(desc_ptr, cam, seed, px, py, k, order=ORDER_REFERENCE):
    L = load()
    rgb = (c_float * 3)()
    cnt = Counters()
    rc = L.oracle_sample(desc_ptr, ctypes.byref(cam), seed, px, py, k, order, rgb, ctypes.byref(cnt))
    if rc != 0:
        raise RuntimeError("oracle_sample rejected its arguments")
    return np.array(list(rgb), dtype=np.float32), cnt.as_dict()


def ppm_pixel(rgb) -> str:
    L = load()
    v = (c_float * 3)(*[float(x) for x in rgb])
    buf = ctypes.create_string_buffer(64)
    n = L.oracle_ppm_pixel(v, buf)
    return buf.raw[:n].decode()


class OracleScene:
    """randSpheres built by the oracle's own builder (an independent restatement)."""

    def __init__(self, seed: int):
        L = load()
        self._h = L.oracle_build_random_spheres(seed)
        if not self._h:
            raise RuntimeError("oracle_build_random_spheres failed")

    @property
    def desc(self):
        return load().oracle_scene_desc(self._h)

    def close(self):
        if self._h:
            load().oracle_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def camera(aspect: float, width: int, **kw) -> rtx.Camera:
    """oracle_camera_init with reference defaults overridden by kw (degrees for fov/defocus)."""
    L = load()
    o = CameraOpts()
    L.oracle_camera_defaults(ctypes.byref(o))
    for k, v in kw.items():
        if k == "fov_degrees":
            o.fov_radians = L.oracle_to_radians(v)
        elif k == "defocus_degrees":
            o.defocus_radians = L.oracle_to_radians(v)
        elif k in ("look_from", "look_at", "vup", "background"):
            setattr(o, k, (c_float * 3)(*v))
        else:
            setattr(o, k, v)
    cam = rtx.Camera()
    L.oracle_camera_init(np.float32(aspect), width, ctypes.byref(o), ctypes.byref(cam))
    return cam


def rand_spheres_camera(width: int = 400, spp: int = 500, depth: int = 50) -> rtx.Camera:
    """main.go:228-239 camera."""
    return camera(np.float32(16.0) / np.float32(9.0), width, samples_per_pixel=spp, max_depth=depth,
                  look_from=(13, 2, 3), look_at=(0, 0, 0), fov_degrees=20, defocus_degrees=0.6,
                  focus_dist=10, background=(0.7, 0.8, 1.0))


def near_slab_pass(o, d, mn, mx, lo, hi):
    """The near walk's slab test (oracle_near_slab_pass: the FMA form for rays within its bounds), elementwise."""
    arrs = [np.ascontiguousarray(a, np.float32) for a in (o, d, mn, mx, lo, hi)]
    out = np.zeros(len(arrs[0]), np.uint8)
    load().oracle_near_slab_pass(*[a.ctypes.data_as(c_void_p) for a in arrs], out.ctypes.data_as(c_void_p), len(out))
    return out.astype(bool)
