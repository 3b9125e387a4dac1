"""The wave-level claim guard (raytracer-go_amd/csrc/rtx_kernel.hip partial_wave).

The megakernel's three claims — a unit of (tile, samples) from the unit queue, slots in the defer queue,
slots in the redo list — each take ONE atomic issued by lane 0 and broadcast its result with
readfirstlane.  That is only right when the whole wave reaches the claim.  Each site checks EXEC on
SALU first; a partial wave flags the render and claims nothing, every wave stops at its next check of
the flag, and rtx_render fails with RTX_ERR_HIP instead of hanging or returning a corrupt frame (the
round-4 early-claim refactor hung, then gave run-to-run different frames, on exactly this).

librtx_dbgclaim.so is the megakernel built with RTX_DEBUG_PARTIAL=1: claim site RTX_DEBUG_PARTIAL_SITE
(1 = defer queue, 2 = redo list, 3 = unit queue) is entered by the even lanes only.  Each case runs in a
child process with its own time limit, so a guard that failed to fire shows as a timeout, not a hung
runner.  The work every pixel needs done exactly once is camera.go:198-222's.
"""
import os
import subprocess
import sys

import pytest

import rtx

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DBG = os.path.join(ROOT, "raytracer-go_amd", "librtx_dbgclaim.so")

CHILD = """
import sys, hashlib, numpy as np, torch
sys.path[:0] = ['raytracer-go_amd', 'tests']
import rtx
torch.cuda.set_device(0)
s = rtx.HostScene('random_spheres', 1)
d = rtx.DeviceScene(s.desc)
cam = s.camera(width=96, spp=4)
try:
    img, st = d.render_host(cam, 7, n_gpus=1, stats=True)
    print('OK', hashlib.sha256(img.tobytes()).hexdigest()[:16], 'tiered' if st.walk_layout & rtx.RTX_LAYOUT_TIERED else 'one', st.deferred_paths)
except rtx.RtxError as e:
    print('ERR', e.code, e)
"""


def run_child(env: dict) -> str:
    res = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=dict(os.environ, **env), capture_output=True,
                         text=True, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    return res.stdout.strip().splitlines()[-1]


def test_debug_library_renders_like_the_product(built):
    """With no site selected the debug library takes the product's path: the same frame as librtx.so,
    tiered, with deferred paths (so the defer-queue claim ran)."""
    assert os.path.exists(DBG), "librtx_dbgclaim.so not built (make -C raytracer-go_amd)"
    want = run_child({})
    got = run_child({"RTX_LIB": DBG, "RTX_DEBUG_PARTIAL_SITE": "0"})
    assert want.startswith("OK") and got == want, (want, got)
    assert want.split()[2] == "tiered" and int(want.split()[3]) > 0, want


@pytest.mark.parametrize("site,extra", [(1, {}), (2, {"RTX_DEFER_CAP": "0"}), (3, {})],
                         ids=["defer_queue", "redo_list", "unit_queue"])
def test_partial_wave_claim_fails_loudly(built, site, extra):
    """Half a wave at a claim: rtx_render returns RTX_ERR_HIP naming the partial EXEC, promptly (the
    watchdog, set to 60 s, is not what stops it)."""
    env = {"RTX_LIB": DBG, "RTX_DEBUG_PARTIAL_SITE": str(site), "RTX_WATCHDOG_S": "60", **extra}
    out = run_child(env)
    assert out.startswith(f"ERR {rtx.RTX_ERR_HIP}"), out
    assert "without the whole wave" in out, out


PIPELINED = """
import os, sys, numpy as np, torch
sys.path[:0] = ['raytracer-go_amd', 'tests']
import rtx
torch.cuda.set_device(0)
s = rtx.HostScene('random_spheres', 1)
d = rtx.DeviceScene(s.desc)
cam = s.camera(width=96, spp=4)
reg = rtx.Region(0, 0, cam.image_width, cam.image_height, 0, 1)
o = torch.zeros((cam.image_height, cam.image_width, 3), device='cuda')
stream = torch.cuda.current_stream().cuda_stream
bad = int(sys.argv[1])
for i in range(3):  # enqueued back to back, no stats read between them (bench.py's timed loop)
    if i == bad:
        os.environ['RTX_DEBUG_PARTIAL_SITE'] = '3'
    d.render_region(cam, 7, reg, o.data_ptr(), stream)
    os.environ.pop('RTX_DEBUG_PARTIAL_SITE', None)
for k in range(2):
    try:
        rtx.device_check(0)
        print('OK', k)
    except rtx.RtxError as e:
        print('ERR', k, e.code, e)
"""


@pytest.mark.parametrize("bad", [-1, 1], ids=["clean", "second_of_three"])
def test_error_word_is_sticky_across_pipelined_renders(built, bad):
    """The kernel's error word survives later renders (no render zeroes it): a partial-wave claim
    in the 2nd of 3 renders enqueued back to back without stats is still reported by ONE rtx_device_check after
    the 3rd; the report is acknowledged (a second check passes), and a clean run passes both."""
    res = subprocess.run([sys.executable, "-c", PIPELINED, str(bad)], cwd=ROOT,
                         env=dict(os.environ, RTX_LIB=DBG, RTX_WATCHDOG_S="60"), capture_output=True, text=True,
                         timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    lines = res.stdout.strip().splitlines()[-2:]
    if bad < 0:
        assert lines == ["OK 0", "OK 1"], lines
    else:
        assert lines[0].startswith(f"ERR 0 {rtx.RTX_ERR_HIP}") and "without the whole wave" in lines[0], lines
        assert lines[1] == "OK 1", lines


def test_bench_fails_on_a_flagged_timed_step(built):
    """bench.py's timed renders are checked: a partial-wave claim in the 2nd of 3 timed steps (enqueued with no
    stats read) fails the bench with a non-zero status; without it, the last timed frame's hash is the verify
    render's (timed_frames_hash == framebuffer_sha256_16)."""
    cmd = [sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--width", "96", "--spp", "4", "--no-cpu"]
    env = dict(os.environ, RTX_LIB=DBG, RTX_WATCHDOG_S="60")
    ok = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert ok.returncode == 0, ok.stdout + ok.stderr
    import json

    line = json.loads([ln for ln in ok.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["timed_frames_hash"] == line["framebuffer_sha256_16"], line
    bad = subprocess.run(cmd + ["--debug-partial-step", "1"], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=300)
    assert bad.returncode != 0, bad.stdout + bad.stderr
    assert "without the whole wave" in bad.stderr, bad.stderr[-2000:]
