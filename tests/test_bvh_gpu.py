"""GPU BVH build: rtx_scene_create_spheres builds NewBVHFromWorld
(bvh.go:138-185) on the device; its threaded entries must equal, byte for byte, the ones
rtx_scene_create emits from the host-built tree (host mirror of bvh.go, seeded axis
stream), and it must render the same bits."""
import time

import numpy as np
import pytest

import rtx


def test_world_spheres_export(built):
    host = rtx.HostScene("random_spheres", 1)
    arr, n, draw0, seed = host.world_spheres()
    d = host.desc.contents
    assert n == d.n_spheres and seed == 1
    assert draw0 > 0  # the scene generation drew from the global stream before NewBVH
    assert all(arr[i].material < d.n_materials for i in range(n))
    with pytest.raises(rtx.RtxError):
        rtx.HostScene("cornell_box", 1).world_spheres()  # quads: not a World of spheres


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    torch.cuda.set_device(0)
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("bvh", ["reference", "default"])
@pytest.mark.parametrize("scene", ["random_spheres", "earth_dielectric", "simple_light_demo", "stress_100k"])
def test_gpu_build_equals_host_build(torch_cuda, built, monkeypatch, scene, bvh):
    """RTX_BVH=reference: the reference's own layout from both builds; default: the walk's tree
    (rtx_topology.h) over them, the same again."""
    if bvh == "reference":
        monkeypatch.setenv("RTX_BVH", "reference")
    host = rtx.HostScene(scene, 1)
    ref = rtx.DeviceScene(host.desc)
    gpu = rtx.DeviceScene.from_spheres(host)
    a, b = ref.export(), gpu.export()
    assert len(a) == len(b)
    if a != b:
        ea = np.frombuffer(a, np.uint32).reshape(-1, 8)
        eb = np.frombuffer(b, np.uint32).reshape(-1, 8)
        bad = np.nonzero((ea != eb).any(axis=1))[0]
        raise AssertionError(f"{len(bad)} entries differ, first {bad[:5]}: {ea[bad[0]]} vs {eb[bad[0]]}")
    print(f"{scene}: GPU build {gpu.build_ms:.1f} ms, {len(a) // 32} entries")


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7])
def test_gpu_build_small_worlds(torch_cuda, built, n):
    """Lists of 1 (left == right), 2 (ordered pair) and odd splits, from randSpheres' first spheres."""
    host = rtx.HostScene("random_spheres", 3)
    arr, total, draw0, seed = host.world_spheres()
    d = host.desc.contents
    L = rtx.load()
    import ctypes
    h = ctypes.c_void_p()
    rtx.check(L.rtx_scene_create_spheres(arr, n, d.materials, d.n_materials, d.textures, d.n_textures, d.texels,
                                         d.n_texels, seed, 77, ctypes.byref(h), None), "create_spheres")
    gpu = rtx.DeviceScene(handle=h)
    entries = np.frombuffer(gpu.export(), np.uint32).reshape(-1, 8)
    expect = {1: 2, 2: 3}.get(n)
    if expect:
        assert len(entries) == expect
    prims = entries[entries[:, 7].view(np.int32) != -1]
    assert len(prims) == n  # every sphere exactly once
    nodes = entries[entries[:, 7].view(np.int32) == -1]
    assert (nodes[:, 3] <= len(entries)).all()  # escapes inside the table


@pytest.mark.gpu
def test_gpu_built_scene_renders_identically(torch_cuda, built):
    host = rtx.HostScene("random_spheres", 1)
    cam = host.camera(width=160, spp=3)
    ref = rtx.DeviceScene(host.desc).render_host(cam, 4)[0]
    got = rtx.DeviceScene.from_spheres(host).render_host(cam, 4)[0]
    assert np.array_equal(ref, got)
