#!/usr/bin/env python3
"""Headline benchmark: Mray/s on 1920x1080x500spp random-spheres (BASELINE.json configs[1])
on N MI355X, with the roofline of the megakernel and the CPU oracle timed on the host beside it.

A step = one render of the whole image of randSpheres (main.go:227-289, seeded),
row-interleaved over the N ranks (one process per GPU), plus the RCCL gather of the shards
to rank 0 when N > 1.  Scene tables are uploaded to HBM before timing.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--spp S]
  --spp 2000 is configs[2] (1920x1080x2000, meant for 8 GPUs).
  N > 1 either under torch.distributed.run (RANK/WORLD_SIZE in the environment), or plain
  `python bench.py --gpus N`: the process then starts N rank processes itself (before any
  GPU call) and exits with their status.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "raytracer-go_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
SIMDS = 1024  # 256 CUs x 4 SIMD-32
CLOCK_MAX_GHZ = 2.4
# VALU issue peak: one wave64 instruction per 2 cycles per SIMD (MI355X_MICROARCH.md, wave scheduling)
VALU_PEAK_GINST = SIMDS * CLOCK_MAX_GHZ / 2.0
LDS_READ_PEAK_GBS = 150000.0  # ds_read_b128 aggregate with every CU streaming (MI355X_MICROARCH.md §LDS)
CPU_SHARE_PER_GPU = 16  # the host's cores per GPU (gpurun: "size worker pools to the box's CPU share")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--scene", default="random_spheres")
    ap.add_argument("--scene-seed", type=int, default=1)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--cpu-target-s", type=float, default=15.0, help="CPU baseline budget (seconds)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: the host's CPU share per GPU")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-hash", action="store_true", help="skip the framebuffer hash")
    ap.add_argument("--no-verify", action="store_true",
                    help="one rank: skip the untimed render with the library's stats and error check after the timed "
                         "steps (PMC profiles count every dispatch of the bench kernel: scripts/gpu_profiles.sh)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_r06.jsonl"),
                    help="PMC HBM-traffic summaries (scripts/pmc_traffic.py): a .json, or a .jsonl of one per workload")
    ap.add_argument("--valu", default=os.path.join(ROOT, "profiles", "valu_r06.jsonl"),
                    help="PMC VALU summaries (scripts/pmc_valu.py): a .json, or a .jsonl of one per workload")
    ap.add_argument("--stripe", type=int, default=1, help="rows per stripe of the shards, a power of two (1: single "
                    "rows interleaved, the fastest slowest-rank at N = 4 and 8, profiles/r05_stripe_sweep.jsonl)")
    ap.add_argument("--shard", default="", help="R/N: one process renders only rank R's rows of N (a rank's "
                    "workload of the N-GPU run, for its PMC profile); not a scaling number")
    ap.add_argument("--in-process", action="store_true",
                    help="one process drives --gpus N devices through rtx_render(n_gpus = N): the C-ABI's own "
                         "band render + ncclGather + de-interleave + copy into a host buffer (what a Go host calls)")
    ap.add_argument("--no-in-process", action="store_true",
                    help="N > 1 under torch.distributed: skip rank 0's in-process leg after the timed steps")
    # launcher self-test on the CPU (tests/test_bench_launcher.py): gloo, no GPU, shards filled
    # with a known function of the global pixel instead of rendered
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N > 1 rank processes all on cuda:0 with a gloo gather (host copies): the multi-rank "
                         "render path on a one-GPU box; not a scaling number")
    ap.add_argument("--selftest-gloo", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--selftest-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    # test hook (tests/test_bench_check.py): with RTX_LIB = librtx_dbgclaim.so, timed step i (0-based) alone enters
    # the unit-queue claim with half the wave; the error check after the timed region must fail the bench
    ap.add_argument("--debug-partial-step", type=int, default=-1, help=argparse.SUPPRESS)
    return ap.parse_args()


# ---- launcher: N rank processes without torchrun ------------------------------------------
def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """Start n copies of this script as ranks 0..n-1 (torch.distributed env contract) and
    wait for them; if one fails, stop the others.  Touches no GPU itself."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:  # a failed rank leaves the others waiting in a collective
                    q.terminate()
        time.sleep(0.05)
    return rc


# ---- measurement helpers -----------------------------------------------------------------
def alg_bytes(st: dict, pixels: int) -> float:
    """32 B per node visit, 20 B per primitive test (16 B sphere +
    4 B material id), 20 B per hit (material record), 4 B per texel fetch, plus the
    12 B float32 RGB write per pixel."""
    return (32.0 * st["node_visits"] + 20.0 * st["prim_tests"] + 20.0 * st["hits"] + 4.0 * st["texel_fetches"]
            + 12.0 * pixels)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cgroup_cpus():
    """The CPUs the cgroup's quota allows this process (cgroup v2 cpu.max "quota period"), or None when unlimited:
    the GPU box shares its host, so sched_getaffinity can list more CPUs than the process may use at once."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(scene, cam, seed: int, target_s: float, threads: int, stride: int = 0) -> dict:
    """The oracle (oracle/liboracle.so, a scalar C restatement) on host threads over a
    bounded sample of the same workload: full-width rows at a fixed stride, all spp.
    stride > 0: that sample (the full-host leg reuses the headline leg's rows), no calibration."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_binding as ob
    import rtx

    logical = len(os.sched_getaffinity(0))
    if threads <= 0:
        threads = min(CPU_SHARE_PER_GPU, logical)
    H = cam.image_height
    if stride <= 0:
        # Calibrate on 2 rows per thread (every thread busy), then size the sample to
        # ~target_s of wall time on those threads.
        cal_rows = min(H, 2 * threads)
        stride = max(1, H // cal_rows)
        t0 = time.perf_counter()
        ob.render(scene.desc, cam, seed, rtx.Region(0, 0, cam.image_width, H, 0, stride), ob.ORDER_REFERENCE, threads)
        dt = time.perf_counter() - t0
        rows_per_s = ((H + stride - 1) // stride) / max(dt, 1e-6)
        rows = max(2, min(H, int(rows_per_s * target_s)))
        stride = max(1, H // rows)
    reg = rtx.Region(0, 0, cam.image_width, H, 0, stride)
    t0 = time.perf_counter()
    _, c = ob.render(scene.desc, cam, seed, reg, ob.ORDER_REFERENCE, threads)
    dt = time.perf_counter() - t0
    nrows = (H + stride - 1) // stride
    who = (f"one GPU's share of the host's {logical} logical CPUs" if threads < logical else
           f"every logical CPU this process may run on (os.sched_getaffinity), as the reference sizes its pool to "
           f"runtime.NumCPU() (camera.go:167)")
    return {
        "value": c["segments"] / dt / 1e6,
        "unit": "Mray/s",
        "cores": threads,
        "kind": "port",
        "samples_per_s": c["samples"] / dt,
        "seconds": dt,
        "stride": stride,
        "cpu_model": cpu_model(),
        "host_logical_cpus": logical,
        "cgroup_cpu_quota": cgroup_cpus(),
        "sample": f"{nrows} full-width rows (every {stride}th) of the same {cam.image_width}x{H}x{cam.samples_per_pixel} "
                  f"render, {c['samples']} samples, C oracle on {threads} threads = {who} (Go absent on the host: the "
                  "C restatement stands in for the Go reference)",
    }


def schedule(st: dict) -> dict:
    """Wave-schedule counters of rank 0's untimed counting launch (same decisions as the timed
    kernel): traversal active-lane fraction, lanes idle for want of work, shading's share of
    wave cycles and, for scenes too big for the LDS copy, the LDS-cache hit rate."""
    out = {}
    if st.get("wave_iters"):
        it = 64.0 * st["wave_iters"]
        out["trav_lane_util"] = round(st["lane_steps"] / it, 4)
        out["idle_lane_frac"] = round(st["idle_lanes"] / it, 4)
        out["parked_lane_frac"] = round(st.get("parked_lanes", 0) / it, 4)  # waiting to shade
        out["deferred_lane_frac"] = round(st.get("deferred_lanes", 0) / it, 4)  # other entry kind
        cyc = st["trav_cycles"] + st["shade_cycles"]
        out["shade_cycle_share"] = round(st["shade_cycles"] / cyc, 4) if cyc else None
        sp = st.get("shade_split_cycles")
        if cyc and sp:  # shares of all wave cycles: scatter sampling, shading, claims + camera rays, trav_begin
            out["shade_split"] = {k: round(v / cyc, 4) for k, v in zip(("scatter", "shade", "claim_camera", "begin"), sp)}
    reads = st.get("node_visits", 0) + st.get("prim_tests", 0)
    if st.get("cache_hits") and reads:
        out["lds_cache_hit_frac"] = round(st["cache_hits"] / reads, 4)
    return out


def lib_sha16() -> str:
    """sha256 prefix of the librtx.so this process renders with (rtx.load(): RTX_LIB or the in-tree build)."""
    import rtx

    path = os.environ.get("RTX_LIB") or rtx.lib_path("librtx.so")
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def load_profile(path: str, workload: str, lib: str):
    """A committed PMC summary, if it was measured on this workload with this very library
    (pmc_valu.py / pmc_traffic.py record the library's hash); else (None, why)."""
    if not os.path.exists(path):
        return None, f"{os.path.relpath(path, ROOT)} missing"
    with open(path) as f:
        if path.endswith(".jsonl"):
            entries = [json.loads(ln) for ln in f if ln.strip()]
        else:
            entries = [json.load(f)]
    same = [d for d in entries if d.get("workload") == workload]
    if not same:
        return None, f"{os.path.relpath(path, ROOT)} has no profile of {workload}"
    for d in same:
        if d.get("librtx_sha256_16") == lib:
            return d, None
    return None, (f"{os.path.relpath(path, ROOT)} profiled {workload} on librtx "
                  f"{', '.join(sorted({str(d.get('librtx_sha256_16')) for d in same}))}, this run loads {lib}: "
                  "stale, frac not derived")


def served_from(st: dict) -> str:
    """Where the walk's entry reads come from (rtx_stats.scene_placement)."""
    import rtx

    reads = st.get("node_visits", 0) + st.get("prim_tests", 0)
    if st.get("scene_placement") == rtx.RTX_SCENE_IN_LDS:
        return "LDS (whole scene + material table copied per workgroup)"
    if st.get("scene_placement") == rtx.RTX_SCENE_LDS_CACHE and reads:
        h = st["cache_hits"] / reads
        return f"LDS cache of the top levels {h:.1%} of entry reads, the other {1 - h:.1%} L2/MALL/HBM"
    return "L2/MALL/HBM (scene in HBM, no LDS cache)"


def roofline(st: dict, pixels: int, kernel_s: float, workload: str, traffic_path: str, valu_path: str) -> dict:
    """The render kernel's roof is VALU issue: its scene and materials are
    LDS-resident, HBM carries only the sample scratch.  achieved = the committed PMC pass's VALU
    wave-instructions per launch (same kernel, same workload, same librtx.so by hash) / this run's
    HIP-event time of the launch; peak = 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction.
    A profile of another library build leaves achieved / frac null (stale).  The SURVEY §8(d)
    algorithmic bytes and the measured HBM bytes are reported beside it."""
    launch_bytes = alg_bytes(st, pixels)
    lib = lib_sha16()
    tr, tr_why = load_profile(traffic_path, workload, lib)
    vr, vr_why = load_profile(valu_path, workload, lib)
    out = {"bound": "valu", "achieved": None, "peak": round(VALU_PEAK_GINST, 1), "unit": "Gwave-inst/s",
           "frac": None, "traffic": tr.get("hbm_bytes_per_launch") if tr else None, "librtx_sha256_16": lib,
           "workload": workload}
    if vr:
        achieved = vr["valu_insts_per_launch"] / kernel_s / 1e9
        out.update(achieved=round(achieved, 1), frac=round(achieved / VALU_PEAK_GINST, 4),
                   lane_frac=vr["valu_lane_frac"], pmc_issue_frac=vr["valu_issue_frac"],
                   valu_insts_per_launch=vr["valu_insts_per_launch"], source=os.path.relpath(valu_path, ROOT))
    else:
        out["stale"] = vr_why
    src = served_from(st)
    lds_scene = src.startswith("LDS (whole")
    out["alg_bytes"] = {
        "per_launch": launch_bytes,
        "achieved_gbs": round(launch_bytes / kernel_s / 1e9, 1),
        "served_from": src,
    }
    if lds_scene:
        out["alg_bytes"]["frac_of_lds_read_peak"] = round(launch_bytes / kernel_s / 1e9 / LDS_READ_PEAK_GBS, 4)
    if tr:
        out["hbm"] = {"bytes_per_launch": tr["hbm_bytes_per_launch"],
                      "achieved_gbs": round(tr["hbm_bytes_per_launch"] / kernel_s / 1e9, 1),
                      "frac": round(tr["hbm_bytes_per_launch"] / kernel_s / 1e9 / HBM_PEAK_GBS, 4),
                      "source": os.path.relpath(traffic_path, ROOT)}
    else:
        out["hbm"] = {"stale": tr_why}
    return out


def walk_desc(st, skips, near_skips, cam) -> str:
    """The walked layout(s) of a render, from its stats and the plans' skip masks."""
    import rtx

    lay = st.get("walk_layout", 0)
    tiered = bool(lay & rtx.RTX_LAYOUT_TIERED)
    lay &= ~rtx.RTX_LAYOUT_TIERED

    def col(m):
        return f"collapsed: {int(m.sum())} of {len(m)} node tests left out" if m.any() else "every box test"

    if tiered:
        far = "the caller's tree" if lay == rtx.RTX_LAYOUT_REFERENCE else "guarded tree"
        return (f"tiered: near tree ({col(near_skips)}), {far} for {st.get('deferred_paths', 0)} deferred "
                f"paths ({col(skips)}), camera octant {rtx.camera_octant(cam)}")
    if lay == rtx.RTX_LAYOUT_REFERENCE:
        return "reference tree, " + col(skips)
    return f"rebuilt tree, camera octant {lay}, " + col(skips)


def framebuffer_hash(img) -> str:
    import numpy as np

    a = np.ascontiguousarray(img.detach().cpu().numpy(), dtype=np.float32)
    return hashlib.sha256(a.tobytes()).hexdigest()[:16]


# ---- the run -------------------------------------------------------------------------------
def main():
    args = parse()
    if args.in_process:
        return main_in_process(args)
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(launch_ranks(args.gpus))  # before anything touches a GPU
    import torch
    import torch.distributed as dist

    from dist import gather_image, max_shard_rows

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.selftest_gloo:
        return selftest_gloo(args, rank, world)

    import rtx

    shared = args.rehearse_one_gpu and world > 1  # every rank on cuda:0 (RCCL needs one GPU per rank)
    torch.cuda.set_device(0 if shared else local_rank)
    backend = None
    if shared:
        backend = "gloo"
        dist.init_process_group(backend)
    elif world > 1:
        backend = "nccl"  # RCCL on ROCm
        dist.init_process_group(backend, device_id=torch.device("cuda", local_rank))

    scene = rtx.HostScene(args.scene, seed=args.scene_seed)
    cam = scene.camera(width=args.width, spp=args.spp, depth=args.depth)
    W, H, S = cam.image_width, cam.image_height, cam.samples_per_pixel
    dev = rtx.DeviceScene(scene.desc)  # one-time upload to this rank's HBM
    skips = dev.walk_skip(cam)  # the walk's plan for this camera (rtx_collapse.h), made before timing
    near_skips = dev.near_skip(cam) if dev.near_region(cam)[1] else None  # the tiered walk's near tree (§14)
    # the rows this process renders: its rank's of the world, or (--shard R/N) one rank's of N alone
    srank, sworld = (int(v) for v in args.shard.split("/")) if args.shard else (rank, world)
    if world > 1 and args.shard:
        raise SystemExit("--shard is a one-process run")
    stripe = max(args.stripe, 1)  # rows per stripe
    reg = rtx.Region(0, 0, W, H, srank, sworld, stripe)
    R = max_shard_rows(H, sworld, stripe)
    shard = torch.zeros((R, W, 3), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # Untimed counting pass (separate kernel instantiation): the work units of a step.
    st = dev.render_region(cam, args.seed, reg, shard.data_ptr(), stream, counters=True, timed=True).as_dict()
    my_rows = rtx.region_rows(reg)
    keys = ["samples", "segments", "node_visits", "prim_tests", "hits", "texel_fetches", "rng_draws"]
    counts = torch.tensor([st[k] for k in keys], dtype=torch.float64, device="cpu" if shared else "cuda")
    if world > 1:
        dist.all_reduce(counts)
    tot = dict(zip(keys, counts.tolist()))

    def step(times, gathers):
        s = dev.render_region(cam, args.seed, reg, shard.data_ptr(), stream, counters=False, timed=True)
        times.append(s.kernel_ms)
        g0 = time.perf_counter()  # (render_region waited for this rank's kernel)
        out = shard[:rtx.region_rows(reg)] if args.shard else gather_image(shard.cpu() if shared else shard, H, rank,
                                                                                world, stripe=stripe)
        if world > 1 and out is not None and not shared:
            torch.cuda.synchronize()
        gathers.append((time.perf_counter() - g0) * 1e3)
        return out

    for _ in range(args.warmup):
        step([], [])
    barrier()
    # The K steps are enqueued back to back on the stream (no stats read between them, so the GPU does not idle for
    # a host round trip per step): per step the render, then (N > 1) the RCCL gather of the shards and rank 0's
    # de-interleave, each bracketed by events on that stream — the kernel time and the gather time per step.  (An
    # RCCL collective on torch's NCCL stream waits for this stream's render and makes this stream wait for it, so
    # the next render does not overwrite the shard before it is sent.)  Nothing of the library's stats is read in
    # the timed region: its sticky error word is checked once after it, for all K renders.
    # (A rehearsal on one GPU runs the same loop; its gloo gather takes host copies, which wait on the host.)
    timed_img = None
    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i, (e0, e1, e2) in enumerate(evs):
        if i == args.debug_partial_step:  # (test hook: the debug library's partial-wave claim in this step only)
            os.environ["RTX_DEBUG_PARTIAL_SITE"] = "3"
        e0.record()
        dev.render_region(cam, args.seed, reg, shard.data_ptr(), stream, counters=False, timed=False)
        e1.record()
        os.environ.pop("RTX_DEBUG_PARTIAL_SITE", None)
        timed_img = shard[:rtx.region_rows(reg)] if args.shard else gather_image(shard.cpu() if shared else shard, H,
                                                                                 rank, world, stripe=stripe)
        e2.record()
    barrier()
    elapsed = time.perf_counter() - t0
    # Every timed render's kernel ran without a watchdog stop or a partial-wave claim, or the bench fails here
    # (rtx_device_check reads the error word no render clears: one check covers all K).
    rtx.device_check(torch.cuda.current_device())
    # the frame the last timed step produced (rank 0: the gathered image), hashed before anything renders again
    timed_hash = framebuffer_hash(timed_img) if rank == 0 and not args.no_hash else None
    kms = [e0.elapsed_time(e1) for e0, e1, _ in evs]
    gms = [e1.elapsed_time(e2) for _, e1, e2 in evs]
    img = timed_img
    if not args.no_verify:
        img = step([], [])  # (untimed: the frame once more, with the library's stats and error check)
    t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if shared else "cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    # per-rank kernel time (HIP events on this rank's stream), to tell imbalance from gather cost
    mine = torch.tensor([sum(kms) / len(kms)], dtype=torch.float64, device="cpu" if shared else "cuda")
    per_rank = [mine]
    if world > 1:
        per_rank = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(per_rank, mine)
    rank_kms = [float(x.item()) for x in per_rank]

    if rank == 0:
        assert img is not None and tuple(img.shape) == ((rtx.region_rows(reg), W, 3) if args.shard else (H, W, 3))
        ms_step = elapsed / args.steps * 1e3
        mray = tot["segments"] * args.steps / elapsed / 1e6
        samples_s = tot["samples"] * args.steps / elapsed
        avg_kernel_s = sum(kms) / len(kms) / 1e3
        headline = args.scene == "random_spheres" and (W, H, S) == (1920, 1080, 500)
        c3 = args.scene == "random_spheres" and (W, H, S) == (1920, 1080, 2000)
        metric = ("Mray/s on 1920x1080x500spp random-spheres; achieved HBM GB/s vs peak" if headline else
                  f"Mray/s on {W}x{H}x{S}spp {args.scene}" + (" (configs[2])" if c3 else " (not the headline config)"))
        tag = " (configs[1])" if headline else (" (configs[2])" if c3 else "")
        if shared:
            metric = f"rehearsal: {world} ranks sharing one GPU, gloo gather (not a scaling number); " + metric
        if args.shard:
            metric = f"shard {srank}/{sworld} alone (rank {srank}'s rows of an {sworld}-GPU run; not a scaling number); " + metric
        # the PMC profile of this process's own workload: the frame, or its rank's rows of an N-way run
        # (profiled alone with --shard R/N)
        profile_workload = f"{args.scene}:{W}x{H}x{S}" + (f"/rows{srank}of{sworld}" if sworld > 1 else "") + (
            f"/stripe{stripe}" if stripe > 1 else "")
        out = {
            "metric": metric,
            "value": round(mray, 3),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (seeded {args.scene} scene built by the host mirror of main.go; "
                    "RNG contract Philox4x32-10)",
            "config": {
                "workload": f"{args.scene} {W}x{H}x{S}spp depth {cam.max_depth}{tag}",
                "scene_seed": args.scene_seed,
                "render_seed": args.seed,
                "parallelism": f"row-interleave x{world}" + (" + gloo gather on one GPU" if shared else
                                                               (" + RCCL gather" if world > 1 else "")),
                "world_size": dist.get_world_size() if world > 1 else 1,
                "backend": backend,
            },
            "samples_per_s": round(samples_s, 1),
            "gsamples_per_s": round(samples_s / 1e9, 4),
            "segments_per_sample": round(tot["segments"] / tot["samples"], 4),
            "node_visits_per_segment": round(tot["node_visits"] / tot["segments"], 3),
            "kernel_ms_avg": round(avg_kernel_s * 1e3, 3),
            "walk_layout": walk_desc(st, skips, near_skips, cam),
            "prim_tests_per_segment": round(tot["prim_tests"] / tot["segments"], 3),
            "schedule": schedule(st),
            "roofline": roofline(st, my_rows * W, avg_kernel_s, profile_workload, args.traffic, args.valu),
        }
        if sworld > 1:
            out["roofline"]["scope"] = (f"rank {srank}'s kernel on its own rows ({my_rows} of {H}), against the PMC "
                                        f"profile of that shard rendered alone (bench.py --shard {srank}/{sworld})")
        if world > 1:  # rank 0's wall time in the gather (incl. waiting for the slowest rank)
            out["gather_ms_avg"] = round(sum(gms) / len(gms), 3)
            out["kernel_ms_per_rank"] = {"min": round(min(rank_kms), 3), "max": round(max(rank_kms), 3),
                                         "all": [round(x, 3) for x in rank_kms]}
        if not args.no_hash:
            out["framebuffer_sha256_16"] = framebuffer_hash(img)  # bitwise-comparable across N
            # the last timed step's own frame: equal to the checked frame, or the timed region rendered something else
            out["timed_frames_hash"] = timed_hash
            out["timed_frames_checked"] = (f"rtx_device_check after the {args.steps} timed renders: no watchdog stop, "
                                           "no partial-wave claim; the last timed frame's hash "
                                           + ("equals the verify render's" if not args.no_verify else
                                              "(no verify render: --no-verify)"))
            if not args.no_verify and timed_hash != out["framebuffer_sha256_16"]:
                print(json.dumps(out), flush=True)
                raise SystemExit(f"the last timed frame ({timed_hash}) differs from the verify render "
                                 f"({out['framebuffer_sha256_16']})")
        if world == 1 and not args.no_cpu and not args.shard:
            out["cpu_baseline"] = cpu_baseline(scene, cam, args.seed, args.cpu_target_s, args.cpu_threads)
            # the same rows on every CPU the process may use: the reference's own concurrency (runtime.NumCPU()
            # workers, camera.go:167); the one-GPU share above stays the headline baseline
            if len(os.sched_getaffinity(0)) > out["cpu_baseline"]["cores"]:
                out["cpu_baseline_full_host"] = cpu_baseline(scene, cam, args.seed, args.cpu_target_s,
                                                             len(os.sched_getaffinity(0)),
                                                             stride=out["cpu_baseline"]["stride"])
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        if world > 1 and not shared and not args.no_in_process:
            out["in_process"] = in_process_leg(args, world)
        print(json.dumps(out), flush=True)


def in_process_leg(args, n: int) -> dict:
    """Rank 0, after the ranks' timed steps: the same workload through the C-ABI's own N-device path
    (rtx_render(n_gpus = N): bands on devices 0..N-1, one ncclGather to device 0, the de-interleave
    kernel, the copy into a host buffer) in a child process with a time limit — the path a Go host
    takes, timed by the same driver run."""
    keep = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "MASTER_ADDR",
            "MASTER_PORT", "TORCHELASTIC_RUN_ID")
    env = {k: v for k, v in os.environ.items() if k not in keep}
    cmd = [sys.executable, os.path.abspath(__file__), "--in-process", "--gpus", str(n), "--steps", str(args.steps),
           "--warmup", str(max(1, args.warmup)), "--width", str(args.width), "--spp", str(args.spp), "--depth",
           str(args.depth), "--scene", args.scene, "--scene-seed", str(args.scene_seed), "--seed", str(args.seed)]
    try:
        res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
        if res.returncode != 0 or not lines:
            return {"error": f"exit {res.returncode}: {(res.stderr or res.stdout)[-400:]}"}
        return json.loads(lines[-1])
    except subprocess.TimeoutExpired:
        return {"error": "timed out after 600 s"}


def main_in_process(args):
    """--in-process: one process, --gpus N devices, rtx_render(n_gpus = N) timed per step (render of
    every band + RCCL gather + de-interleave + copy into this process's host buffer).  Counts come from
    one untimed rtx_render_ex(RTX_FLAG_COUNTERS) over the same devices."""
    import numpy as np
    import torch  # (before librtx.so: one HIP runtime per process)

    import rtx

    n = args.gpus
    assert torch.cuda.device_count() >= n, f"--in-process --gpus {n}: {torch.cuda.device_count()} devices visible"
    scene = rtx.HostScene(args.scene, seed=args.scene_seed)
    cam = scene.camera(width=args.width, spp=args.spp, depth=args.depth)
    W, H, S = cam.image_width, cam.image_height, cam.samples_per_pixel
    dev = rtx.DeviceScene(scene.desc)
    buf = np.zeros((H, W, 3), dtype=np.float32)
    _, st = dev.render_host(cam, args.seed, n_gpus=n, counters=True, out=buf)
    for _ in range(args.warmup):
        dev.render_host(cam, args.seed, n_gpus=n, stats=True, out=buf)
    kms, gms = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        _, s = dev.render_host(cam, args.seed, n_gpus=n, stats=True, out=buf)
        kms.append(s.kernel_ms)
        gms.append(s.gather_ms)
    elapsed = time.perf_counter() - t0
    out = {
        "metric": f"Mray/s on {W}x{H}x{S}spp {args.scene}, one process driving {n} GPUs (rtx_render)",
        "value": round(st.segments * args.steps / elapsed / 1e6, 3),
        "unit": "Mray/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "gsamples_per_s": round(st.samples * args.steps / elapsed / 1e9, 4),
        "kernel_ms_max_band_avg": round(sum(kms) / len(kms), 3),
        "gather_ms_avg": round(sum(gms) / len(gms), 3),
        "gather_kind": {rtx.RTX_GATHER_NONE: "none", rtx.RTX_GATHER_RCCL: "rccl", rtx.RTX_GATHER_HOST: "host copies",
                        rtx.RTX_GATHER_DEVICE: "device copies"}.get(s.gather_kind, str(s.gather_kind)),
        "step": "every band's render on its device + ncclGather to device 0 + de-interleave + copy to the host "
                "buffer (24.9 MB at 1920x1080 over PCIe)",
        "framebuffer_sha256_16": hashlib.sha256(np.ascontiguousarray(buf).tobytes()).hexdigest()[:16],
    }
    print(json.dumps(out), flush=True)


def selftest_gloo(args, rank: int, world: int) -> None:
    """The multi-rank plumbing of main() on the CPU: gloo process group, striped shards
    of a width x height image (height from the scene's 16:9 aspect), each filled with its global
    pixel index instead of a render, the same gather + de-interleave, and rank 0's JSON line
    with the framebuffer hash (tests/test_bench_launcher.py recomputes it)."""
    import torch
    import torch.distributed as dist

    from dist import gather_image, max_shard_rows, shard_rows

    if rank == args.selftest_fail_rank:
        raise SystemExit(f"rank {rank}: failing on purpose (--selftest-fail-rank)")
    if world > 1:
        dist.init_process_group("gloo")
    W = args.width
    H = int(W * 9 // 16)
    S = max(args.stripe, 1)  # main()'s stripes
    R = max_shard_rows(H, world, S)
    shard = torch.zeros((R, W, 3), dtype=torch.float32)
    for i in range(shard_rows(H, rank, world, S)):
        y = ((i // S) * world + rank) * S + i % S  # rtx_region_row
        idx = torch.arange(W, dtype=torch.float32) + float(y * W)
        shard[i] = idx[:, None].expand(W, 3)
    img = gather_image(shard, H, rank, world, stripe=S)
    if rank == 0:
        print(json.dumps({"selftest": True, "n_gpus": world, "world_size": dist.get_world_size() if world > 1 else 1,
                          "backend": "gloo" if world > 1 else None, "height": H,
                          "framebuffer_sha256_16": framebuffer_hash(img)}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
