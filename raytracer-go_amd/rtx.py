"""ctypes binding of librtx.so (include/rtx.h) and librtxhost.so (include/rtx_host.h).

This is plumbing for the Python test driver and bench.py — the drop-in boundary
itself is the C-ABI (a Go host binds it via cgo).  Loading fails
loudly if the native libraries are missing: there is no CPU fallback for the product
path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int32, c_uint32, c_uint64, c_void_p

HERE = os.path.dirname(os.path.abspath(__file__))

RTX_OK = 0
RTX_ERR_INVALID_ARG = -1
RTX_ERR_HIP = -2
RTX_ERR_RCCL = -3
RTX_ERR_UNSUPPORTED = -4
RTX_ERR_NO_DEVICE = -5
RTX_ERR_OOM = -6

RTX_PRIM_SPHERE = 0
RTX_PRIM_QUAD = 1
RTX_PRIM_LIST = 2  # a World nested in the tree (ABI 5)
RTX_MAT_LAMBERTIAN, RTX_MAT_METAL, RTX_MAT_DIELECTRIC, RTX_MAT_DIFFUSE_LIGHT = 0, 1, 2, 3
RTX_TEX_SOLID, RTX_TEX_CHECKERED, RTX_TEX_IMAGE, RTX_TEX_NOISE = 0, 1, 2, 3
RTX_FLAG_COUNTERS = 1
RTX_FLAG_NO_LDS = 4
RTX_FLAG_TIMING = 1 << 20  # diagnostics: timed kernel + wave-cycle split
RTX_SCENE_REFERENCE_BVH = 1  # rtx_scene_create_ex: keep the caller's tree and the reference's visit order
RTX_SCENE_EVERY_BOX = 2  # rtx_scene_create_ex: the walk leaves no box test out (ABI 7, rtx_collapse.h)
RTX_SCENE_NO_TIER = 4  # rtx_scene_create_ex: no tiered walk (ABI 8)
RTX_LAYOUT_REFERENCE = 8  # Stats.walk_layout of a scene walking the caller's tree
RTX_LAYOUT_TIERED = 16  # Stats.walk_layout bit: the render walked in two tiers (ABI 8)
RTX_TREE_NEAR = 0x100  # rtx_scene_topology / rtx_walk_tree octant bit: the near tree (ABI 8)
RTX_GATHER_NONE, RTX_GATHER_RCCL, RTX_GATHER_DEVICE, RTX_GATHER_HOST = 0, 1, 2, 3  # Stats.gather_kind
RTX_SCENE_IN_HBM, RTX_SCENE_IN_LDS, RTX_SCENE_LDS_CACHE = 0, 1, 2  # Stats.scene_placement
RTX_IMAGE_TEXEL_WORDS = 2  # RGBA16 image texels: two uint32 words each (rtx.h)


def RTX_FLAG_SHADE_THRESH(n: int) -> int:
    return (n & 0x7F) << 8


def ref_prim(ptype: int, index: int) -> int:
    """RTX_REF_PRIM: ~((type << 28) | index) as int32."""
    v = ((ptype << 28) | (index & 0x0FFFFFFF)) & 0xFFFFFFFF
    return ~v if v < 0x80000000 else ~(v - (1 << 32))


class BvhNode(ctypes.Structure):
    _fields_ = [("bmin", c_float * 3), ("left", c_int32), ("bmax", c_float * 3), ("right", c_int32)]


class Sphere(ctypes.Structure):
    _fields_ = [("center", c_float * 3), ("radius", c_float), ("material", c_uint32), ("pad", c_uint32 * 3)]


class Quad(ctypes.Structure):
    _fields_ = [("q", c_float * 3), ("material", c_uint32), ("u", c_float * 3), ("d", c_float),
                ("v", c_float * 3), ("pad0", c_float), ("w", c_float * 3), ("pad1", c_float),
                ("normal", c_float * 3), ("pad2", c_float)]


class Material(ctypes.Structure):
    _fields_ = [("type", c_uint32), ("texture", c_uint32), ("fuzz", c_float), ("ior", c_float),
                ("albedo", c_float * 3), ("pad", c_float)]


class Texture(ctypes.Structure):
    _fields_ = [("type", c_uint32), ("scale", c_float), ("width", c_uint32), ("height", c_uint32),
                ("even", c_float * 3), ("texel_offset", c_uint32), ("odd", c_float * 3), ("pad", c_float)]


class List(ctypes.Structure):  # rtx_list (ABI 5): a World nested in the tree
    _fields_ = [("first", c_uint32), ("count", c_uint32)]


class SceneDesc(ctypes.Structure):
    _fields_ = [("nodes", POINTER(BvhNode)), ("n_nodes", c_uint32), ("n_roots", c_uint32),
                ("roots", POINTER(c_int32)), ("spheres", POINTER(Sphere)), ("n_spheres", c_uint32),
                ("n_quads", c_uint32), ("quads", POINTER(Quad)), ("materials", POINTER(Material)),
                ("n_materials", c_uint32), ("n_textures", c_uint32), ("textures", POINTER(Texture)),
                ("texels", POINTER(c_uint32)), ("n_texels", c_uint64),
                ("lists", POINTER(List)), ("n_lists", c_uint32), ("n_list_refs", c_uint32),
                ("list_refs", POINTER(c_int32))]


class Camera(ctypes.Structure):
    _fields_ = [("image_width", c_uint32), ("image_height", c_uint32), ("samples_per_pixel", c_uint32),
                ("max_depth", c_uint32), ("center", c_float * 3), ("defocus_angle", c_float),
                ("pixel00", c_float * 3), ("pad0", c_float), ("pixel_du", c_float * 3), ("pad1", c_float),
                ("pixel_dv", c_float * 3), ("pad2", c_float), ("defocus_disk_u", c_float * 3), ("pad3", c_float),
                ("defocus_disk_v", c_float * 3), ("pad4", c_float), ("background", c_float * 3), ("pad5", c_float)]


class Region(ctypes.Structure):
    """rtx_region: columns [x0, x0 + width), the rows of [y0, y0 + height) in stripes of `stripe` rows (0 / 1:
    single rows) dealt round-robin: this shard takes stripes rank, rank + world, ... (ABI 9: stripe)."""
    _fields_ = [("x0", c_uint32), ("y0", c_uint32), ("width", c_uint32), ("height", c_uint32),
                ("rank", c_uint32), ("world", c_uint32), ("stripe", c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [("samples", c_uint64), ("segments", c_uint64), ("node_visits", c_uint64),
                ("prim_tests", c_uint64), ("hits", c_uint64), ("texel_fetches", c_uint64),
                ("rng_draws", c_uint64), ("kernel_ms", c_double), ("gather_ms", c_double),
                ("wave_iters", c_uint64), ("lane_steps", c_uint64), ("shade_phases", c_uint64),
                ("shade_lanes", c_uint64), ("trav_cycles", c_uint64), ("shade_cycles", c_uint64),
                ("idle_lanes", c_uint64), ("cache_hits", c_uint64), ("sample_chunks", c_uint64),
                ("parked_lanes", c_uint64), ("deferred_lanes", c_uint64), ("shade_split_cycles", c_uint64 * 4),
                ("walk_layout", c_uint64), ("gather_kind", c_uint64), ("scene_placement", c_uint64),
                ("deferred_paths", c_uint64), ("redo_chunks", c_uint64)]

    def as_dict(self) -> dict:
        return {name: (list(v) if not isinstance(v := getattr(self, name), (int, float)) else v)
                for name, _ in self._fields_}


RTX_SYMBOLS = [
    "rtx_version", "rtx_build_info", "rtx_last_error", "rtx_device_count", "rtx_scene_create",
    "rtx_scene_destroy", "rtx_scene_device_bytes", "rtx_render", "rtx_render_region_device", "rtx_region_rows",
    "rtx_ppm_max_bytes", "rtx_encode_ppm_device", "rtx_render_ppm", "rtx_scene_create_spheres", "rtx_scene_export",
    "rtx_release_device_memory", "rtx_device_scratch_bytes", "rtx_scene_create_ex", "rtx_scene_topology",
    "rtx_camera_octant", "rtx_walk_tree", "rtx_render_ex", "rtx_scene_walk_skip", "rtx_walk_skip",
    "rtx_scene_near_region", "rtx_scene_near_skip", "rtx_walk_near_region", "rtx_render_ppm_ex", "rtx_region_row",
    "rtx_device_check",
]
RTXHOST_SYMBOLS = [
    "rtxhost_build_scene", "rtxhost_scene_free", "rtxhost_scene_desc", "rtxhost_scene_camera",
    "rtxhost_render_ppm", "rtxhost_ppm_encode", "rtxhost_last_error", "rtxhost_scene_world_spheres",
    "rtxhost_synthetic_earth_ycbcr", "rtxhost_ycbcr_rgba",
]

_lib = None
_host = None


def lib_path(name: str) -> str:
    return os.path.join(HERE, name)


def load() -> ctypes.CDLL:
    """Load librtx.so (raises OSError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("RTX_LIB") or lib_path("librtx.so")  # RTX_LIB: A/B against another build
    if not os.path.exists(path):
        raise OSError(f"librtx.so not built at {path}: run __graft_entry__.build() (no CPU fallback exists)")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7 (the SONAME of
    # /opt/rocm's), and whichever loads first serves both.  With librtx first, torch then bound to
    # the system runtime and reported no GPU (torch.cuda.is_available() False); torch first works.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    L.rtx_version.restype = c_int
    L.rtx_build_info.restype = c_char_p
    L.rtx_last_error.restype = c_char_p
    L.rtx_device_count.restype = c_int
    L.rtx_scene_create.argtypes = [POINTER(SceneDesc), POINTER(c_void_p)]
    L.rtx_scene_create.restype = c_int
    L.rtx_scene_create_ex.argtypes = [POINTER(SceneDesc), c_uint32, POINTER(c_void_p)]
    L.rtx_scene_create_ex.restype = c_int
    L.rtx_scene_topology.argtypes = [c_void_p, c_uint32, POINTER(BvhNode), c_uint32, POINTER(c_uint32),
                                     POINTER(c_int32)]
    L.rtx_scene_topology.restype = c_int
    L.rtx_walk_tree.argtypes = [POINTER(SceneDesc), c_uint32, c_uint32, POINTER(BvhNode), c_uint32,
                                POINTER(c_uint32), POINTER(c_int32)]
    L.rtx_walk_tree.restype = c_int
    L.rtx_scene_walk_skip.argtypes = [c_void_p, POINTER(Camera), c_void_p, c_uint32, POINTER(c_uint32)]
    L.rtx_scene_walk_skip.restype = c_int
    L.rtx_walk_skip.argtypes = [POINTER(SceneDesc), c_uint32, POINTER(Camera), c_void_p, c_uint32, POINTER(c_uint32)]
    L.rtx_walk_skip.restype = c_int
    L.rtx_scene_near_region.argtypes = [c_void_p, POINTER(Camera), POINTER(c_float), POINTER(c_uint32)]
    L.rtx_scene_near_region.restype = c_int
    L.rtx_scene_near_skip.argtypes = [c_void_p, POINTER(Camera), c_void_p, c_uint32, POINTER(c_uint32)]
    L.rtx_scene_near_skip.restype = c_int
    L.rtx_walk_near_region.argtypes = [POINTER(SceneDesc), c_uint32, POINTER(Camera), POINTER(c_float),
                                       POINTER(c_uint32)]
    L.rtx_walk_near_region.restype = c_int
    L.rtx_camera_octant.argtypes = [POINTER(Camera)]
    L.rtx_camera_octant.restype = c_uint32
    L.rtx_scene_destroy.argtypes = [c_void_p]
    L.rtx_scene_destroy.restype = None
    L.rtx_scene_device_bytes.argtypes = [c_void_p]
    L.rtx_scene_device_bytes.restype = c_uint64
    L.rtx_render.argtypes = [c_void_p, POINTER(Camera), c_uint64, c_int, c_void_p, POINTER(Stats)]
    L.rtx_render.restype = c_int
    L.rtx_render_ex.argtypes = [c_void_p, POINTER(Camera), c_uint64, c_int, c_uint32, c_void_p, POINTER(Stats)]
    L.rtx_render_ex.restype = c_int
    L.rtx_render_region_device.argtypes = [c_void_p, POINTER(Camera), c_uint64, POINTER(Region), c_void_p,
                                           c_void_p, c_uint32, POINTER(Stats)]
    L.rtx_render_region_device.restype = c_int
    L.rtx_region_rows.argtypes = [POINTER(Region)]
    L.rtx_region_rows.restype = c_uint32
    L.rtx_ppm_max_bytes.argtypes = [c_uint32, c_uint32]
    L.rtx_ppm_max_bytes.restype = c_uint64
    L.rtx_encode_ppm_device.argtypes = [c_void_p, c_uint32, c_uint32, c_void_p, c_uint64, POINTER(c_uint64), c_void_p]
    L.rtx_encode_ppm_device.restype = c_int
    L.rtx_render_ppm.argtypes = [c_void_p, POINTER(Camera), c_uint64, c_void_p, c_uint64, POINTER(c_uint64),
                                 POINTER(Stats)]
    L.rtx_render_ppm.restype = c_int
    if hasattr(L, "rtx_render_ppm_ex"):  # ABI 9 (RTX_LIB may name an older build for A/B)
        L.rtx_render_ppm_ex.argtypes = [c_void_p, POINTER(Camera), c_uint64, c_int, c_void_p, c_uint64,
                                        POINTER(c_uint64), POINTER(Stats)]
        L.rtx_render_ppm_ex.restype = c_int
    L.rtx_scene_create_spheres.argtypes = [POINTER(Sphere), c_uint32, POINTER(Material), c_uint32, POINTER(Texture),
                                           c_uint32, POINTER(c_uint32), c_uint64, c_uint64, c_uint64,
                                           POINTER(c_void_p), POINTER(c_double)]
    L.rtx_scene_create_spheres.restype = c_int
    L.rtx_scene_export.argtypes = [c_void_p, c_void_p, c_uint64]
    L.rtx_scene_export.restype = c_uint64
    L.rtx_release_device_memory.argtypes = [c_int]
    L.rtx_release_device_memory.restype = c_int
    L.rtx_device_scratch_bytes.argtypes = [c_int]
    L.rtx_device_scratch_bytes.restype = c_uint64
    if hasattr(L, "rtx_device_check"):  # ABI 10 (RTX_LIB may name an older build for A/B)
        L.rtx_device_check.argtypes = [c_int]
        L.rtx_device_check.restype = c_int
    _lib = L
    return L


def load_host() -> ctypes.CDLL:
    global _host
    if _host is not None:
        return _host
    load()
    path = lib_path("librtxhost.so")
    if not os.path.exists(path):
        raise OSError(f"librtxhost.so not built at {path}")
    H = ctypes.CDLL(path)
    H.rtxhost_build_scene.argtypes = [c_char_p, c_uint64, POINTER(c_void_p)]
    H.rtxhost_build_scene.restype = c_int
    H.rtxhost_scene_free.argtypes = [c_void_p]
    H.rtxhost_scene_free.restype = None
    H.rtxhost_scene_desc.argtypes = [c_void_p]
    H.rtxhost_scene_desc.restype = POINTER(SceneDesc)
    H.rtxhost_scene_camera.argtypes = [c_void_p, c_int32, c_int32, c_int32, POINTER(Camera)]
    H.rtxhost_scene_camera.restype = c_int
    H.rtxhost_render_ppm.argtypes = [c_char_p, c_uint64, c_int32, c_int32, c_int32, c_uint64, c_int32, c_char_p]
    H.rtxhost_render_ppm.restype = c_int
    H.rtxhost_ppm_encode.argtypes = [c_void_p, c_uint32, c_uint32, c_void_p, c_uint64]
    H.rtxhost_ppm_encode.restype = c_uint64
    H.rtxhost_last_error.restype = c_char_p
    H.rtxhost_scene_world_spheres.argtypes = [c_void_p, POINTER(Sphere), c_uint64, POINTER(c_uint64), POINTER(c_uint64)]
    H.rtxhost_scene_world_spheres.restype = ctypes.c_int64
    H.rtxhost_synthetic_earth_ycbcr.argtypes = [c_uint64, c_int32, c_int32, c_void_p, c_void_p, c_void_p]
    H.rtxhost_synthetic_earth_ycbcr.restype = c_int
    H.rtxhost_ycbcr_rgba.argtypes = [ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8, POINTER(c_uint32)]
    H.rtxhost_ycbcr_rgba.restype = None
    _host = H
    return H


class RtxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"rtx error {code}: {msg}")
        self.code = code


def check(rc: int, where: str = "rtx") -> None:
    if rc != RTX_OK:
        msg = load().rtx_last_error().decode()
        raise RtxError(rc, f"{where}: {msg}")


class HostScene:
    """A main.go scene built by the C++ mirror (NewBVH + flatten)."""

    def __init__(self, name: str, seed: int = 1):
        H = load_host()
        h = c_void_p()
        rc = H.rtxhost_build_scene(name.encode(), seed, ctypes.byref(h))
        if rc != RTX_OK:
            raise RtxError(rc, H.rtxhost_last_error().decode())
        self._h = h
        self.name = name
        self.seed = seed

    @property
    def desc(self):
        d = load_host().rtxhost_scene_desc(self._h)
        d._owner = self  # the tables live in this scene: keep it alive as long as the pointer
        return d

    def camera(self, width: int = 0, spp: int = 0, depth: int = 0) -> Camera:
        cam = Camera()
        rc = load_host().rtxhost_scene_camera(self._h, width, spp, depth, ctypes.byref(cam))
        if rc != RTX_OK:
            raise RtxError(rc, load_host().rtxhost_last_error().decode())
        return cam

    def world_spheres(self):
        """(Sphere array in World.Add order, BVH draw position, seed): rtx_scene_create_spheres' inputs."""
        H = load_host()
        draw0, seed = c_uint64(), c_uint64()
        n = H.rtxhost_scene_world_spheres(self._h, None, 0, None, None)
        if n < 0:
            raise RtxError(int(n), H.rtxhost_last_error().decode())
        arr = (Sphere * max(int(n), 1))()
        H.rtxhost_scene_world_spheres(self._h, arr, n, ctypes.byref(draw0), ctypes.byref(seed))
        return arr, int(n), draw0.value, seed.value

    def close(self) -> None:
        if self._h:
            load_host().rtxhost_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceScene:
    """rtx_scene_create: the tables uploaded once to the current HIP device."""

    def __init__(self, desc_ptr=None, handle=None, reference_bvh: bool = False, every_box: bool = False,
                 no_tier: bool = False):
        L = load()
        self.build_ms = None
        if handle is not None:
            self._h = handle
            return
        h = c_void_p()
        flags = ((RTX_SCENE_REFERENCE_BVH if reference_bvh else 0) | (RTX_SCENE_EVERY_BOX if every_box else 0) |
                 (RTX_SCENE_NO_TIER if no_tier else 0))
        check(L.rtx_scene_create_ex(desc_ptr, flags, ctypes.byref(h)), "rtx_scene_create_ex")
        self._h = h

    @classmethod
    def from_spheres(cls, host: "HostScene") -> "DeviceScene":
        """rtx_scene_create_spheres: the BVH of host's World built on the GPU."""
        L = load()
        arr, n, draw0, seed = host.world_spheres()
        d = host.desc.contents
        h = c_void_p()
        ms = c_double()
        check(L.rtx_scene_create_spheres(arr, n, d.materials, d.n_materials, d.textures, d.n_textures, d.texels,
                                         d.n_texels, seed, draw0, ctypes.byref(h), ctypes.byref(ms)),
              "rtx_scene_create_spheres")
        obj = cls(handle=h)
        obj.build_ms = ms.value
        return obj

    def export(self) -> bytes:
        L = load()
        n = int(L.rtx_scene_export(self._h, None, 0))
        buf = ctypes.create_string_buffer(n)
        L.rtx_scene_export(self._h, buf, n)
        return buf.raw

    @property
    def handle(self):
        return self._h

    def device_bytes(self) -> int:
        return load().rtx_scene_device_bytes(self._h)

    def topology(self, octant: int):
        """(nodes ctypes array, root) of the tree the scene walks for a camera octant, or None when
        the scene walks the caller's tree (rtx_scene_topology)."""
        L = load()
        n, root = c_uint32(), c_int32()
        check(L.rtx_scene_topology(self._h, octant, None, 0, ctypes.byref(n), ctypes.byref(root)), "rtx_scene_topology")
        if n.value == 0 and root.value == -1:
            return None
        arr = (BvhNode * max(n.value, 1))()
        check(L.rtx_scene_topology(self._h, octant, arr, n.value, ctypes.byref(n), ctypes.byref(root)),
              "rtx_scene_topology")
        return arr, int(n.value), int(root.value)

    def walk_desc(self, desc_ptr, cam: Camera):
        """The scene description of the tree the scene walks for `cam` (the caller's own when the
        scene keeps it): same spheres, materials and textures, the walk's nodes and root.  The
        oracle rendering this description takes the kernel's box and primitive tests one for one."""
        t = self.topology(camera_octant(cam))
        if t is None:
            return desc_ptr
        arr, n, root = t
        return desc_with_tree(desc_ptr, arr, n, root)

    def near_region(self, cam: Camera):
        """(box (6 floats: min xyz, max xyz) or None, active) — rtx_scene_near_region."""
        box, act = (c_float * 6)(), c_uint32()
        for i in range(6):
            box[i] = float("nan")
        check(load().rtx_scene_near_region(self._h, ctypes.byref(cam), box, ctypes.byref(act)), "rtx_scene_near_region")
        vals = [float(v) for v in box]
        return (None if vals[0] != vals[0] else vals), bool(act.value)

    def near_desc(self, desc_ptr, cam: Camera):
        """The description of the near tree the scene walks for cam (rtx_scene_topology octant | RTX_TREE_NEAR)."""
        t = self.topology(camera_octant(cam) | RTX_TREE_NEAR)
        if t is None:
            return None
        arr, n, root = t
        return desc_with_tree(desc_ptr, arr, n, root)

    def near_skip(self, cam: Camera):
        """rtx_scene_near_skip: the near walk's skips for cam (numpy uint8)."""
        return _skip_mask(lambda buf, cap, n: load().rtx_scene_near_skip(self._h, ctypes.byref(cam), buf, cap, n),
                          "rtx_scene_near_skip")

    def walk_skip(self, cam: Camera):
        """rtx_scene_walk_skip: per node entry of the uncollapsed walk for cam (visit order), 1 where
        the collapsed walk leaves its box test out (numpy uint8)."""
        return _skip_mask(lambda buf, cap, n: load().rtx_scene_walk_skip(self._h, ctypes.byref(cam), buf, cap, n),
                          "rtx_scene_walk_skip")

    def render_region(self, cam: Camera, seed: int, region: Region, out_ptr: int, stream: int = 0,
                      counters: bool = False, timed: bool = False, flags: int = 0):
        """Enqueue (and optionally wait/time) a region render into device memory at out_ptr."""
        st = Stats() if (timed or counters) else None
        rc = load().rtx_render_region_device(self._h, ctypes.byref(cam), seed, ctypes.byref(region),
                                             c_void_p(out_ptr), c_void_p(stream),
                                             flags | (RTX_FLAG_COUNTERS if counters else 0),
                                             ctypes.byref(st) if st is not None else None)
        check(rc, "rtx_render_region_device")
        return st

    def render_host(self, cam: Camera, seed: int, n_gpus: int = 1, stats: bool = False, counters: bool = False,
                    out=None):
        """rtx_render (counters=False: the timed kernel) or rtx_render_ex(RTX_FLAG_COUNTERS) into a host array
        (`out`: a C-contiguous float32 [H, W, 3] to reuse, else a new one)."""
        import numpy as np
        if out is None:
            out = np.zeros((cam.image_height, cam.image_width, 3), dtype=np.float32)
        assert out.dtype == np.float32 and out.shape == (cam.image_height, cam.image_width, 3) and out.flags.c_contiguous
        st = Stats() if (stats or counters) else None
        if counters:
            rc = load().rtx_render_ex(self._h, ctypes.byref(cam), seed, n_gpus, RTX_FLAG_COUNTERS,
                                      out.ctypes.data_as(c_void_p), ctypes.byref(st))
        else:
            rc = load().rtx_render(self._h, ctypes.byref(cam), seed, n_gpus, out.ctypes.data_as(c_void_p),
                                   ctypes.byref(st) if st is not None else None)
        check(rc, "rtx_render")
        return out, st

    def render_ppm(self, cam: Camera, seed: int) -> bytes:
        """rtx_render_ppm: the P3 bytes Render writes, rendered and encoded on the GPU."""
        import numpy as np
        L = load()
        cap = int(L.rtx_ppm_max_bytes(cam.image_width, cam.image_height))
        buf = np.empty(cap, dtype=np.uint8)  # not zero-filled: 63 B per pixel of capacity, ~12 used
        n = c_uint64()
        check(L.rtx_render_ppm(self._h, ctypes.byref(cam), seed, buf.ctypes.data_as(c_void_p), cap, ctypes.byref(n),
                               None), "rtx_render_ppm")
        return buf[: n.value].tobytes()

    def render_ppm_ex(self, cam: Camera, seed: int, n_gpus: int = 1, stats: bool = False):
        """rtx_render_ppm_ex (ABI 9): the bands of rtx_render(n_gpus) gathered to device 0, the PPM encoded
        there; returns the bytes (and the Stats when stats=True)."""
        import numpy as np
        L = load()
        cap = int(L.rtx_ppm_max_bytes(cam.image_width, cam.image_height))
        buf = np.empty(cap, dtype=np.uint8)
        n = c_uint64()
        st = Stats()
        check(L.rtx_render_ppm_ex(self._h, ctypes.byref(cam), seed, n_gpus, buf.ctypes.data_as(c_void_p), cap,
                                  ctypes.byref(n), ctypes.byref(st)), "rtx_render_ppm_ex")
        out = buf[: n.value].tobytes()
        return (out, st) if stats else out

    def close(self) -> None:
        if self._h:
            load().rtx_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def release_device_memory(device: int = -1) -> None:
    """rtx_release_device_memory: free the per-device scratch (and RCCL communicators)."""
    check(load().rtx_release_device_memory(device), "rtx_release_device_memory")


def device_scratch_bytes(device: int = 0) -> int:
    return int(load().rtx_device_scratch_bytes(device))


def device_check(device: int = 0) -> None:
    """rtx_device_check (ABI 10): wait for every render enqueued on `device` and raise RtxError
    (RTX_ERR_HIP) if any of them failed in the kernel since the last report (watchdog, partial-wave claim)."""
    check(load().rtx_device_check(device), "rtx_device_check")


def synthetic_earth_ycbcr(seed: int, w: int = 2048, h: int = 1024):
    """(Y [h, w], Cb, Cr [(h+1)//2, (w+1)//2]) uint8 planes of the earth scenes' *image.YCbCr map."""
    import numpy as np
    cw, ch = (w + 1) // 2, (h + 1) // 2
    Y = np.empty((h, w), dtype=np.uint8)
    Cb = np.empty((ch, cw), dtype=np.uint8)
    Cr = np.empty((ch, cw), dtype=np.uint8)
    rc = load_host().rtxhost_synthetic_earth_ycbcr(seed, w, h, Y.ctypes.data_as(c_void_p), Cb.ctypes.data_as(c_void_p),
                                                   Cr.ctypes.data_as(c_void_p))
    if rc != RTX_OK:
        raise RtxError(rc, load_host().rtxhost_last_error().decode())
    return Y, Cb, Cr


def host_ycbcr_rgba(y: int, cb: int, cr: int):
    o = (c_uint32 * 4)()
    load_host().rtxhost_ycbcr_rgba(y, cb, cr, o)
    return tuple(o)


def desc_with_tree(desc_ptr, arr, n: int, root: int):
    """A copy of a scene description with another node table and root (same primitives and materials)."""
    d = desc_ptr.contents
    w = SceneDesc()
    for f, _ in SceneDesc._fields_:
        setattr(w, f, getattr(d, f))
    roots = (c_int32 * 1)(root)
    w.nodes = ctypes.cast(arr, POINTER(BvhNode))
    w.n_nodes = n
    w.n_roots = 1
    w.roots = ctypes.cast(roots, POINTER(c_int32))
    p = ctypes.pointer(w)
    p._keep = (arr, roots, desc_ptr)  # the arrays live as long as the pointer
    return p


def walk_near_region(desc_ptr, cam: Camera, flags: int = 0):
    """rtx_walk_near_region (host only): (box or None, active)."""
    box, act = (c_float * 6)(), c_uint32()
    for i in range(6):
        box[i] = float("nan")
    check(load().rtx_walk_near_region(desc_ptr, flags, ctypes.byref(cam), box, ctypes.byref(act)),
          "rtx_walk_near_region")
    vals = [float(v) for v in box]
    return (None if vals[0] != vals[0] else vals), bool(act.value)


def walk_near_desc(desc_ptr, cam: Camera, flags: int = 0):
    """rtx_walk_tree (host only) of the near tree for cam's octant, or None."""
    L = load()
    n, root = c_uint32(), c_int32()
    oc = camera_octant(cam) | RTX_TREE_NEAR
    check(L.rtx_walk_tree(desc_ptr, flags, oc, None, 0, ctypes.byref(n), ctypes.byref(root)), "rtx_walk_tree")
    if n.value == 0 and root.value == -1:
        return None
    arr = (BvhNode * max(n.value, 1))()
    check(L.rtx_walk_tree(desc_ptr, flags, oc, arr, n.value, ctypes.byref(n), ctypes.byref(root)), "rtx_walk_tree")
    return desc_with_tree(desc_ptr, arr, int(n.value), int(root.value))


def walk_tree_desc(desc_ptr, cam: Camera, flags: int = 0):
    """rtx_walk_tree (host only): the description of the tree a scene made from desc_ptr walks
    for cam's octant — desc_ptr itself when the scene would keep the caller's tree."""
    L = load()
    n, root = c_uint32(), c_int32()
    oc = camera_octant(cam)
    check(L.rtx_walk_tree(desc_ptr, flags, oc, None, 0, ctypes.byref(n), ctypes.byref(root)), "rtx_walk_tree")
    if n.value == 0 and root.value == -1:
        return desc_ptr
    arr = (BvhNode * max(n.value, 1))()
    check(L.rtx_walk_tree(desc_ptr, flags, oc, arr, n.value, ctypes.byref(n), ctypes.byref(root)), "rtx_walk_tree")
    return desc_with_tree(desc_ptr, arr, int(n.value), int(root.value))


def _skip_mask(call, where):
    import numpy as np
    n = c_uint32()
    check(call(None, 0, ctypes.byref(n)), where)
    m = np.zeros(max(n.value, 1), np.uint8)
    check(call(m.ctypes.data_as(c_void_p), n.value, ctypes.byref(n)), where)
    return m[: n.value]


def walk_skip(desc_ptr, cam: Camera, flags: int = 0):
    """rtx_walk_skip (host only): the skips a scene made from desc_ptr plans for a first render with cam."""
    return _skip_mask(lambda buf, cap, n: load().rtx_walk_skip(desc_ptr, flags, ctypes.byref(cam), buf, cap, n),
                      "rtx_walk_skip")


def node_skip(desc_ptr, skip):
    """Map a skip mask over node entries in visit order (emit's pre-order: a node, its left subtree,
    then its right, a one-element split's child once, a nested World's items in order) onto the
    description's node table, for the oracle's walk hooks.  A node met twice must agree."""
    import numpy as np
    d = desc_ptr.contents
    out = np.zeros(max(d.n_nodes, 1), np.uint8)
    seen = np.zeros(max(d.n_nodes, 1), np.uint8)
    k = 0
    for r in range(d.n_roots):
        stack = [d.roots[r]]
        while stack:
            ref = stack.pop()
            if ref >= 0:
                nd = d.nodes[ref]
                v = skip[k]
                k += 1
                if seen[ref] and out[ref] != v:
                    raise ValueError(f"node {ref} is walked twice with different skips")
                seen[ref], out[ref] = 1, v
                if nd.right != nd.left:
                    stack.append(nd.right)
                stack.append(nd.left)
            elif ((~ref) & 0xFFFFFFFF) >> 28 == RTX_PRIM_LIST:
                lst = d.lists[(~ref) & 0x0FFFFFFF]
                for i in reversed(range(lst.count)):
                    stack.append(d.list_refs[lst.first + i])
    if k != len(skip):
        raise ValueError(f"skip mask has {len(skip)} node entries, the walk {k}")
    return out[: d.n_nodes]


def camera_octant(cam: Camera) -> int:
    return int(load().rtx_camera_octant(ctypes.byref(cam)))


def region_rows(region: Region) -> int:
    return int(load().rtx_region_rows(ctypes.byref(region)))


def ppm_encode(rgb) -> bytes:
    import numpy as np
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = a.shape[0], a.shape[1]
    H = load_host()
    n = H.rtxhost_ppm_encode(a.ctypes.data_as(c_void_p), w, h, None, 0)
    buf = ctypes.create_string_buffer(int(n))
    H.rtxhost_ppm_encode(a.ctypes.data_as(c_void_p), w, h, buf, n)
    return buf.raw[: int(n)]


def encode_ppm_device(rgb_ptr: int, width: int, height: int, text_ptr: int, capacity: int, stream: int = 0) -> int:
    """rtx_encode_ppm_device on device buffers; returns the text length."""
    n = c_uint64()
    check(load().rtx_encode_ppm_device(rgb_ptr, width, height, text_ptr, capacity, ctypes.byref(n), stream),
          "rtx_encode_ppm_device")
    return n.value
