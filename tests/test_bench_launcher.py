"""bench.py's own rank launcher on the CPU: `python bench.py --gpus N` without torchrun starts
N rank processes (RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets them), and the
ranks run the multi-GPU plumbing of the bench — process group, row-interleaved shards, the
gather to rank 0, de-interleave, rank 0's single JSON line with the framebuffer hash — over
gloo, with each shard filled with its global pixel index instead of a render (the GPU path
swaps in "nccl" = RCCL and the megakernel)."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def expected_hash(W):
    H = W * 9 // 16
    img = np.repeat((np.arange(H * W, dtype=np.float32).reshape(H, W))[..., None], 3, axis=2)
    return hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest()[:16]


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_plain_launch_spawns_ranks(n):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    res = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--selftest-gloo", "--width", "64"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout  # only rank 0 prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["world_size"] == n
    assert out["backend"] == ("gloo" if n > 1 else None)
    assert out["framebuffer_sha256_16"] == expected_hash(64)


def test_failed_rank_fails_the_launch():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    # rank 1 exits before joining the process group, leaving rank 0 waiting in the rendezvous:
    # the launcher must stop it and return non-zero, not hang.
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--selftest-gloo", "--selftest-fail-rank", "1"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert res.returncode != 0


def _bench_line(args):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    res = subprocess.run([sys.executable, "-u", "bench.py"] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout  # only rank 0 prints
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [3, 4, 8])
def test_rank_processes_render_the_same_image_on_one_gpu(n):
    """The real multi-rank path on a one-GPU box: `bench.py --gpus N --rehearse-one-gpu` starts N rank
    processes on cuda:0, each renders its row-interleaved shard with the megakernel (8 x 8 tiles at N = 3,
    16 x 4 at N = 4, 32 x 2 at N = 8), and the shards are gathered (gloo, host copies: RCCL needs a GPU per
    rank) and de-interleaved on rank 0.  The framebuffer hash must equal the one-rank render's bit for bit."""
    common = ["--width", "192", "--spp", "8", "--steps", "1", "--warmup", "0", "--no-cpu"]
    one = _bench_line(["--gpus", "1"] + common)
    many = _bench_line(["--gpus", str(n), "--rehearse-one-gpu"] + common)
    assert many["n_gpus"] == n and many["config"]["world_size"] == n and many["config"]["backend"] == "gloo"
    assert many["metric"].startswith("rehearsal")
    assert one["framebuffer_sha256_16"] == many["framebuffer_sha256_16"]


def _bench_line_env(args, extra):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra)
    res = subprocess.run([sys.executable, "-u", "bench.py"] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("env,kind", [({"RTX_SIM_BANDS": "3"}, "device copies"), ({"RTX_SIM_BANDS": "8"}, "device copies"),
                                      ({"RTX_FORCE_RCCL": "1"}, "rccl")])
def test_in_process_leg_on_one_gpu(env, kind):
    """`bench.py --in-process`: one process timing rtx_render(n_gpus) — the C-ABI's own N-device path
    (bands, gather to device 0, de-interleave, copy to the host) that rank 0 of an N-GPU run also times
    after its ranks' steps.  On one GPU: RTX_SIM_BANDS=3 renders three bands on device 0 and assembles
    them as the gather does; RTX_FORCE_RCCL=1 runs the ncclGather as a 1-rank gather.  Same framebuffer as
    the one-rank bench, the gather timed."""
    common = ["--width", "192", "--spp", "8", "--steps", "2", "--warmup", "1", "--no-cpu"]
    one = _bench_line(["--gpus", "1"] + common)
    got = _bench_line_env(["--in-process", "--gpus", "1"] + common, env)
    assert got["gather_kind"] == kind and got["gather_ms_avg"] > 0
    assert got["framebuffer_sha256_16"] == one["framebuffer_sha256_16"]
    assert got["value"] > 0 and got["kernel_ms_max_band_avg"] > 0


@pytest.mark.gpu
def test_shard_run_renders_its_rows():
    """`bench.py --shard 1/3`: rank 1's rows of a 3-way run rendered alone (its PMC profile's workload):
    the metric says so, and the roofline looks up that shard's own profile."""
    got = _bench_line(["--shard", "1/3", "--width", "192", "--spp", "8", "--steps", "1", "--warmup", "0", "--no-cpu"])
    assert got["metric"].startswith("shard 1/3")
    assert got["roofline"]["workload"].endswith("/rows1of3") and "rank 1's kernel" in got["roofline"]["scope"]
