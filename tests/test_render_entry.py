"""rtx_render — the entry a Go host calls for the whole of Camera.Render (camera.go:180) — on
one device and row-interleaved over several with the RCCL band gather (include/rtx.h), plus
the device-memory lifetime of its sample scratch.

RCCL and the scratch-lifetime checks run in child processes (a clean device state, and an
RCCL problem cannot hang the test runner: each child has its own time limit).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import rtx

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(code: str, env: dict | None = None, timeout: int = 150) -> str:
    prelude = ("import sys, numpy as np, torch; sys.path[:0] = ['raytracer-go_amd', 'tests']; import rtx\n"
               "torch.cuda.set_device(0)\n")
    res = subprocess.run([sys.executable, "-c", prelude + code], cwd=ROOT, env=dict(os.environ, **(env or {})),
                         capture_output=True, text=True, timeout=timeout)
    assert res.returncode == 0, res.stdout + res.stderr
    # the child's own lines (RCCL prints a version banner to stdout first)
    return "\n".join(ln for ln in res.stdout.splitlines() if not ln.split(":")[0].strip() in RCCL_BANNER)


RCCL_BANNER = {"RCCL version", "HIP version", "ROCm version", "Hostname", "Librccl path"}


def test_rccl_gather_path_one_device(built):
    """RTX_FORCE_RCCL=1: the n_gpus > 1 assembly (ncclCommInitAll, ncclGather of the padded
    bands to device 0, de-interleave on device 0) run as a 1-rank gather: same bits as the
    direct copy, gather_ms timed."""
    out = child(
        "s = rtx.HostScene('random_spheres', 1); d = rtx.DeviceScene(s.desc)\n"
        "cam = s.camera(width=320, spp=4)\n"
        "import os\n"
        "os.environ['RTX_FORCE_RCCL'] = '0'; a, sa = d.render_host(cam, 7, n_gpus=1, stats=True)\n"
        "os.environ['RTX_FORCE_RCCL'] = '1'; b, sb = d.render_host(cam, 7, n_gpus=1, stats=True)\n"
        "assert np.array_equal(a, b), 'rccl path differs'\n"
        "assert sa.gather_ms == 0 and sb.gather_ms > 0, (sa.gather_ms, sb.gather_ms)\n"
        "assert (sa.gather_kind, sb.gather_kind) == (rtx.RTX_GATHER_NONE, rtx.RTX_GATHER_RCCL)\n"
        "assert sa.segments == sb.segments == 0 and sb.samples == 320 * 180 * 4  # the timed kernel\n"
        "rtx.release_device_memory(-1)\n"
        "print('ok', sb.gather_ms)\n")
    assert out.startswith("ok")


def test_rtx_render_every_device(built):
    """rtx_render(n_gpus = rtx_device_count()) == rtx_render(n_gpus = 1) bit for bit, and the
    combined counters are the single-device ones (skips on a one-GPU box)."""
    n = rtx.load().rtx_device_count()
    if n < 2:
        pytest.skip("one GPU visible: the multi-device gather is covered by the 1-rank RCCL test")
    out = child(
        f"n = {n}\n"
        "s = rtx.HostScene('random_spheres', 1); d = rtx.DeviceScene(s.desc)\n"
        "cam = s.camera(width=400, spp=8)\n"
        "a, sa = d.render_host(cam, 3, n_gpus=1, counters=True)\n"
        "b, sb = d.render_host(cam, 3, n_gpus=n, counters=True)\n"
        "c, sc = d.render_host(cam, 3, n_gpus=n, stats=True)\n"
        "assert np.array_equal(a, c) and sc.gather_kind == rtx.RTX_GATHER_RCCL\n"
        "assert np.array_equal(a, b)\n"
        "for k in ('samples', 'segments', 'node_visits', 'prim_tests', 'hits', 'rng_draws'):\n"
        "    assert getattr(sa, k) == getattr(sb, k), k\n"
        "assert sb.gather_ms > 0\n"
        "print('ok')\n")
    assert out.startswith("ok")


def test_scratch_freed_with_last_scene(built):
    """The per-device sample scratch (12 B per sample of a chunk) is freed when the last scene
    with a copy on the device is destroyed: device memory returns to its pre-render level (after
    one warm-up cycle, which leaves the HIP runtime's own one-time allocations in place)."""
    out = child(
        "s = rtx.HostScene('random_spheres', 1)\n"
        "cam = s.camera(width=1920, spp=16)\n"
        "w = rtx.DeviceScene(s.desc); w.render_host(s.camera(width=64, spp=1), 1); w.close()  # runtime warm-up\n"
        "assert rtx.device_scratch_bytes(0) == 0\n"
        "free0 = torch.cuda.mem_get_info()[0]\n"
        "d = rtx.DeviceScene(s.desc)\n"
        "img, st = d.render_host(cam, 1, stats=True)\n"
        "held = rtx.device_scratch_bytes(0)\n"
        "assert held >= 1920 * 1080 * 12 * 16, held\n"
        "free1 = torch.cuda.mem_get_info()[0]\n"
        "assert free0 - free1 >= held\n"
        "d.close()\n"
        "assert rtx.device_scratch_bytes(0) == 0\n"
        "free2 = torch.cuda.mem_get_info()[0]\n"
        "assert abs(free2 - free0) < (64 << 20), (free0, free2)\n"
        "print('ok', held)\n")
    assert out.startswith("ok")


def test_release_device_memory_then_render_again(built):
    out = child(
        "s = rtx.HostScene('random_spheres', 1); d = rtx.DeviceScene(s.desc)\n"
        "cam = s.camera(width=200, spp=4)\n"
        "a, _ = d.render_host(cam, 2)\n"
        "assert rtx.device_scratch_bytes(0) > 0\n"
        "rtx.release_device_memory(0)\n"
        "assert rtx.device_scratch_bytes(0) == 0\n"
        "b, _ = d.render_host(cam, 2)\n"
        "assert np.array_equal(a, b)\n"
        "try:\n"
        "    rtx.release_device_memory(99)\n"
        "    print('no error')\n"
        "except rtx.RtxError as e:\n"
        "    assert e.code == rtx.RTX_ERR_INVALID_ARG\n"
        "print('ok')\n")
    assert out.strip().endswith("ok") and "no error" not in out


def test_watchdog_stops_v3(built):
    """A render whose per-wave time limit (RTX_WATCHDOG_S) is exceeded stops claiming work and
    reports RTX_ERR_HIP instead of keeping the GPU busy."""
    out = child(
        "s = rtx.HostScene('random_spheres', 1); d = rtx.DeviceScene(s.desc); c = s.camera(width=400, spp=8000)\n"
        "o = torch.empty((225, 400, 3), device='cuda')\n"
        "try:\n"
        "    d.render_region(c, 1, rtx.Region(0, 0, 400, 225, 0, 1), o.data_ptr(), 0, timed=True)\n"
        "    print('NOERROR')\n"
        "except rtx.RtxError as e:\n"
        "    print('ERR', e.code)\n"
        "st = d.render_region(s.camera(width=64, spp=1), 1, rtx.Region(0, 0, 64, 36, 0, 1), o.data_ptr(), 0,"
        " timed=True)\n"
        "print('next render ok')\n",
        env={"RTX_WATCHDOG_S": "0.005"})
    assert f"ERR {rtx.RTX_ERR_HIP}" in out and "next render ok" in out, out


@pytest.mark.parametrize("bands,stripe", [(2, 1), (3, 1), (5, 1), (7, 1), (3, 8), (5, 8), (2, 4)])
def test_band_assembly_index_math_one_gpu(built, bands, stripe):
    """The n > 1 assembly on one GPU (RTX_SIM_BANDS=k: k bands rendered on device 0 — single rows interleaved, or
    stripes of RTX_STRIPE rows dealt round-robin —, each padded to band 0's rows, placed at band offsets as the RCCL
    gather places them, de-interleaved by the kernel; with RTX_NO_RCCL=1 each band's rows (stripes) copied straight
    into the caller's rows instead).  H = 112: ragged last bands, and 14 stripes of 8 for 3 and 5 bands."""
    out = child(
        f"k = {bands}\n"
        "import os\n"
        f"os.environ['RTX_STRIPE'] = '{stripe}'\n"
        "s = rtx.HostScene('random_spheres', 1); d = rtx.DeviceScene(s.desc)\n"
        "cam = s.camera(width=200, spp=3)\n"
        "assert cam.image_height == 112\n"
        "a, sa = d.render_host(cam, 9, counters=True)\n"
        "os.environ['RTX_SIM_BANDS'] = str(k)\n"
        "b, sb = d.render_host(cam, 9, counters=True)\n"
        "assert np.array_equal(a, b), 'device gather differs'\n"
        "assert sb.gather_kind == rtx.RTX_GATHER_DEVICE, sb.gather_kind\n"
        "for f in ('samples', 'segments', 'node_visits', 'prim_tests', 'hits', 'rng_draws'):  # every band's\n"
        "    assert getattr(sa, f) == getattr(sb, f), (f, getattr(sa, f), getattr(sb, f))\n"
        "os.environ['RTX_NO_RCCL'] = '1'\n"
        "c, sc = d.render_host(cam, 9, stats=True)\n"
        "assert np.array_equal(a, c), 'host band copies differ'\n"
        "assert sc.gather_kind == rtx.RTX_GATHER_HOST\n"
        "del os.environ['RTX_SIM_BANDS']\n"
        "os.environ['RTX_FORCE_RCCL'] = '1'  # the RCCL path with RCCL unavailable: host copies\n"
        "e, se = d.render_host(cam, 9, stats=True)\n"
        "assert np.array_equal(a, e) and se.gather_kind == rtx.RTX_GATHER_HOST\n"
        "rtx.release_device_memory(-1)\n"
        "print('ok')\n")
    assert out.strip().endswith("ok")


def test_rtx_render_stats_run_the_timed_kernel(built):
    """rtx_render(..., &stats) times the timed kernel (no work counters, about the kernel time of
    rtx_render_region_device without counters); rtx_render_ex(RTX_FLAG_COUNTERS) runs the
    counting kernel: same image, counters filled.  The buffers are reused across calls."""
    out = child(
        "s = rtx.HostScene('random_spheres', 1); d = rtx.DeviceScene(s.desc)\n"
        "cam = s.camera(width=1920, spp=24)\n"
        "reg = rtx.Region(0, 0, 1920, 1080, 0, 1)\n"
        "o = torch.empty((1080, 1920, 3), device='cuda')\n"
        "d.render_host(cam, 4, stats=True)  # warm-up\n"
        "t = [d.render_region(cam, 4, reg, o.data_ptr(), 0, timed=True).kernel_ms for _ in range(3)]\n"
        "free0 = torch.cuda.mem_get_info()[0]\n"
        "runs = [d.render_host(cam, 4, stats=True) for _ in range(3)]\n"
        "free1 = torch.cuda.mem_get_info()[0]\n"
        "a, sa = runs[-1]\n"
        "b, sb = d.render_host(cam, 4, counters=True)\n"
        "assert np.array_equal(a, b) and np.array_equal(a, o.cpu().numpy())\n"
        "assert sa.segments == 0 and sb.segments > 0 and sb.node_visits > 0\n"
        "k = min(r[1].kernel_ms for r in runs)\n"
        "assert abs(k - min(t)) < 0.1 * min(t), (k, t)\n"
        "assert sb.kernel_ms > 1.2 * k, (sb.kernel_ms, k)\n"
        "assert abs(free1 - free0) < (16 << 20), (free0, free1)  # no new buffers per call\n"
        "print('ok', k, min(t), sb.kernel_ms)\n")
    assert out.split()[0] == "ok"


def test_render_and_ppm_concurrently(built):
    """rtx_render and rtx_render_ppm on one scene from two threads at once (both take the scene's lock,
    then the render buffers' lock, in that order): no deadlock, and every result is the one a lone call
    gives."""
    out = child(
        "import threading\n"
        "s = rtx.HostScene('random_spheres', 1); d = rtx.DeviceScene(s.desc)\n"
        "cam = s.camera(width=160, spp=2)\n"
        "img0, _ = d.render_host(cam, 3)\n"
        "ppm0 = d.render_ppm(cam, 3)\n"
        "bad = []\n"
        "def a():\n"
        "    for _ in range(25):\n"
        "        img, _ = d.render_host(cam, 3)\n"
        "        bad.append(not np.array_equal(img, img0))\n"
        "def b():\n"
        "    for _ in range(25):\n"
        "        bad.append(d.render_ppm(cam, 3) != ppm0)\n"
        "ts = [threading.Thread(target=a), threading.Thread(target=b)]\n"
        "[t.start() for t in ts]\n"
        "[t.join(60) for t in ts]\n"
        "assert not any(t.is_alive() for t in ts), 'deadlock'\n"
        "assert len(bad) == 50 and not any(bad)\n"
        "print('ok')\n", timeout=100)
    assert out.strip().endswith("ok")
