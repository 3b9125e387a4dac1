"""Shared GPU-vs-oracle checks (test infrastructure, imported by the -m gpu tests).

Every GPU check renders its region TWICE through the C-ABI (rtx_render_region_device):
  - with the timed kernel (counters off: the instantiation bench.py measures, with the
    assembly walk), and
  - with the counting kernel (RTX_FLAG_COUNTERS: the C++ walk plus work counters),
and holds both to the oracle (oracle/oracle.c):
  1. bit-identical to the oracle's iterative colour order walking the tree the scene walks
     (rtx_scene_topology: the library's rebuilt tree, or the caller's) with the box tests the
     scene's collapsed walk leaves out left out too (rtx_scene_walk_skip), and the counting
     kernel's counters equal to the oracle's on that walk — every box test, sphere test, hit,
     texel fetch and RNG draw; the oracle's full walk of the same tree gives the same image and
     paths (leaving a box test out changes nothing else: rtx_collapse.h);
  2. when the scene walks a rebuilt tree: the oracle on the rebuilt tree bit-identical to the
     oracle on the caller's (the reference's) tree, with the same segments, hits, texel fetches
     and draws — the tree changes the work, not a single path;
  3. within the north-star bar, |delta| <= 1e-4 per channel, of the oracle in the reference's
     own (recursive) colour order on the caller's tree.
A render that walks in two tiers (rtx_stats.walk_layout & RTX_LAYOUT_TIERED) is
held to the oracle's tiered walk (oracle_tier): the near tree with its skips for segments that
start in the near region, the guarded tree with its skips for the others; check 2 then holds
that walk to the caller's tree as well.
"""
from __future__ import annotations

import numpy as np

import oracle_binding as ob
import rtx

TOL = 1e-4  # north_star: per-channel RGB |delta| <= 1e-4 vs the seeded reference
PATH_KEYS = ("samples", "segments", "hits", "texel_fetches", "rng_draws")
WORK_KEYS = PATH_KEYS + ("node_visits", "prim_tests")


def gpu_region(torch, dev, cam, seed, reg, counters=True, flags=0):
    """One region render on cuda:0 (NaN-filled output), waited for; (image, stats)."""
    rows = rtx.region_rows(reg)
    out = torch.full((max(rows, 1), max(reg.width, 1), 3), float("nan"), dtype=torch.float32, device="cuda")
    st = dev.render_region(cam, seed, reg, out.data_ptr(), torch.cuda.current_stream().cuda_stream,
                           counters=counters, timed=True, flags=flags)
    torch.cuda.synchronize()
    return out[:rows, : reg.width].cpu().numpy(), st


def assert_counters_equal(st, cnt, keys=WORK_KEYS):
    for k in keys:
        assert getattr(st, k) == cnt[k], (k, getattr(st, k), cnt[k])


def walk_of(dev, desc, cam):
    """(the tree the scene walks for cam, its per-node skips for the oracle's walk hooks)."""
    walk = dev.walk_desc(desc, cam)
    return walk, rtx.node_skip(walk, dev.walk_skip(cam))


def tier_of(dev, desc, cam):
    """(near tree description, its skips, (near box, guarded tree, its skips)) of a scene that walks
    in two tiers for cam, or None."""
    box, active = dev.near_region(cam)
    if not active:
        return None
    near = dev.near_desc(desc, cam)
    far, fskip = walk_of(dev, desc, cam)
    return near, rtx.node_skip(near, dev.near_skip(cam)), (box, far, fskip)


def oracle_checks(desc, walk, cam, seed, reg, skip=None, tier=None):
    """(iterative image on the walked tree with its skips, its counters, reference-order image on
    the caller's tree); asserts check 2 and the collapsed walk's own check."""
    rank = ob.sphere_ranks(desc) if walk is not desc else None  # the walk's tie rule (sphere_test RANKED)
    it, cnt = ob.render(walk, cam, seed, reg, ob.ORDER_ITERATIVE, skip=skip, tier=tier, rank=rank)
    if walk is not desc or (skip is not None and skip.any()):
        it0, cnt0 = ob.render(desc, cam, seed, reg, ob.ORDER_ITERATIVE)
        assert np.array_equal(it, it0), f"walked tree changes the image: max {np.abs(it - it0).max()}"
        assert cnt["prim_tests"] == cnt0["prim_tests"] or walk is not desc
        for k in PATH_KEYS:
            assert cnt[k] == cnt0[k], (k, cnt[k], cnt0[k])
    ref, _ = ob.render(desc, cam, seed, reg, ob.ORDER_REFERENCE)
    return it, cnt, ref


def check_scene(torch, dev, desc, cam, seed, reg, flags=0, kernels=("timed", "counting")):
    """Checks 1-3 for both kernels on one region; returns (timed image, counting stats, oracle counters)."""
    tier = tier_of(dev, desc, cam)
    if tier is not None:
        walk, skip, tw = tier
    else:
        (walk, skip), tw = walk_of(dev, desc, cam), None
    it, cnt, ref = oracle_checks(desc, walk, cam, seed, reg, skip, tw)
    img = st = None
    for k in kernels:
        gpu, s = gpu_region(torch, dev, cam, seed, reg, counters=(k == "counting"), flags=flags)
        assert np.isfinite(gpu).all(), k
        assert np.array_equal(gpu, it), f"{k} kernel not bit-identical to the oracle: max {np.abs(gpu - it).max()}"
        d = float(np.abs(gpu - ref).max()) if gpu.size else 0.0
        assert d <= TOL, f"{k} kernel: max |delta| = {d} > {TOL} vs the reference-order oracle"
        far = tw[1] if tier is not None else walk  # the tree the walk falls back on: rebuilt, or the caller's
        want = rtx.camera_octant(cam) if far is not desc else rtx.RTX_LAYOUT_REFERENCE
        if tier is not None:
            want |= rtx.RTX_LAYOUT_TIERED
        assert s.walk_layout == want, (k, s.walk_layout, want)
        assert s.redo_chunks == 0, (k, s.redo_chunks)
        if k == "counting":
            assert_counters_equal(s, cnt)
            st = s
        else:
            img = gpu
    return (img if img is not None else it), st, cnt
