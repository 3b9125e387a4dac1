"""GPU PPM output: rtx_encode_ppm_device / rtx_render_ppm against the
oracle's restatement of camera.go:183-188, 212-215 and vec3.go:141-166, byte for byte."""
import numpy as np
import pytest

import oracle_binding as ob
import rtx


def oracle_ppm(rgb: np.ndarray) -> bytes:
    h, w = rgb.shape[:2]
    lines = [f"P3\n{w} {h}\n255\n"]
    for px in rgb.reshape(-1, 3):
        lines.append(ob.ppm_pixel(px) + "\n")
    return "".join(lines).encode()


def test_max_bytes_bound(built):
    L = rtx.load()
    assert L.rtx_ppm_max_bytes(0, 0) == len(b"P3\n0 0\n255\n")
    assert L.rtx_ppm_max_bytes(1920, 1080) == len(b"P3\n1920 1080\n255\n") + 1920 * 1080 * 63


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    torch.cuda.set_device(0)
    return torch


def gpu_encode(torch, rgb: np.ndarray) -> bytes:
    h, w = rgb.shape[:2]
    d_rgb = torch.from_numpy(np.ascontiguousarray(rgb, dtype=np.float32)).cuda()
    cap = int(rtx.load().rtx_ppm_max_bytes(w, h))
    d_text = torch.empty(cap, dtype=torch.uint8, device="cuda")
    n = rtx.encode_ppm_device(d_rgb.data_ptr(), w, h, d_text.data_ptr(), cap,
                              torch.cuda.current_stream().cuda_stream)
    return bytes(d_text[:n].cpu().numpy())


@pytest.mark.gpu
def test_encode_edge_values(torch_cuda, built):
    """Quantisation edges: 0, -0, negatives (sqrt -> NaN -> MinInt64), >1, inf, NaN,
    denormals, and the float32 values on both sides of every 255.999 step."""
    edges = [0.0, -0.0, -1e-30, -1.0, 1.0, 1.5, np.inf, -np.inf, np.nan, 1e-45, 1e-38, 0.25, 0.5, 0.999999]
    k = np.arange(256, dtype=np.float64)
    steps = ((k / 255.999) ** 2).astype(np.float32)  # gamma^-1 of each level boundary
    around = np.concatenate([np.nextafter(steps, np.float32(-1)), steps, np.nextafter(steps, np.float32(2))])
    vals = np.concatenate([np.array(edges, np.float32), around]).astype(np.float32)
    n = (len(vals) + 2) // 3 * 3
    vals = np.resize(vals, n).reshape(-1, 1, 3)  # a width-1 image
    rgb = np.ascontiguousarray(vals)
    assert gpu_encode(torch_cuda, rgb) == oracle_ppm(rgb)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(1, 1), (7, 3), (640, 360)])
def test_encode_random_images(torch_cuda, built, w, h):
    rng = np.random.default_rng(w * 1000 + h)
    rgb = rng.random((h, w, 3), dtype=np.float32) * np.float32(1.3)
    assert gpu_encode(torch_cuda, rgb) == oracle_ppm(rgb)


@pytest.mark.gpu
def test_encode_empty_image(torch_cuda, built):
    assert gpu_encode(torch_cuda, np.zeros((0, 0, 3), np.float32)) == b"P3\n0 0\n255\n"


@pytest.mark.gpu
def test_render_ppm_matches_render_plus_host_encode(torch_cuda, built):
    """rtx_render_ppm = the Render bytes: header + EncodePPM(rtx_render floats)."""
    s = rtx.HostScene("random_spheres", 1)
    cam = s.camera(width=160, spp=4)
    dev = rtx.DeviceScene(s.desc)
    text = dev.render_ppm(cam, 9)
    rgb, _ = dev.render_host(cam, 9)
    header = f"P3\n{cam.image_width} {cam.image_height}\n255\n".encode()
    assert text == header + rtx.ppm_encode(rgb)


@pytest.mark.gpu
def test_render_ppm_ex_bands_equal_one_device(built):
    """rtx_render_ppm_ex (ABI 9), the multi-GPU Render's output with no host formatting: the bands of
    rtx_render(n_gpus) gathered to device 0 and encoded there.  Its bytes equal rtx_render_ppm's one-device
    bytes for one band, for 8 simulated bands assembled by the de-interleave kernel (RTX_SIM_BANDS=8, the
    rows an 8-GPU node renders; H = 90 leaves ragged bands), for the same bands without RCCL (the per-band
    copies, then one upload), and for the RCCL path as a 1-rank ncclGather (RTX_FORCE_RCCL=1).  Run in a
    child process (its own time limit: an RCCL problem cannot hang the runner)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import os, sys, torch; sys.path[:0] = ['raytracer-go_amd', 'tests']; import rtx\n"
        "torch.cuda.set_device(0)\n"
        "s = rtx.HostScene('random_spheres', 1); d = rtx.DeviceScene(s.desc)\n"
        "cam = s.camera(width=160, spp=4)\n"
        "assert cam.image_height == 90\n"
        "want = d.render_ppm(cam, 9)\n"
        "cases = [({}, rtx.RTX_GATHER_NONE), ({'RTX_SIM_BANDS': '8'}, rtx.RTX_GATHER_DEVICE),\n"
        "         ({'RTX_SIM_BANDS': '8', 'RTX_NO_RCCL': '1'}, rtx.RTX_GATHER_HOST),\n"
        "         ({'RTX_FORCE_RCCL': '1'}, rtx.RTX_GATHER_RCCL)]\n"
        "for env, kind in cases:\n"
        "    for k in ('RTX_SIM_BANDS', 'RTX_NO_RCCL', 'RTX_FORCE_RCCL'): os.environ.pop(k, None)\n"
        "    os.environ.update(env)\n"
        "    got, st = d.render_ppm_ex(cam, 9, n_gpus=1, stats=True)\n"
        "    assert got == want, (env, len(got), len(want))\n"
        "    assert st.gather_kind == kind, (env, st.gather_kind)\n"
        "    print('ok', env, st.gather_kind, round(st.gather_ms, 3))\n"
        "rtx.release_device_memory(-1)\n")
    res = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=150)
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.count("ok ") == 4, res.stdout
