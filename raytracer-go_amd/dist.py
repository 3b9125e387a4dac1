"""Image sharding across ranks (one process per GPU) and the framebuffer gather.

Rows are dealt in stripes: rank r renders the stripes r, r + N, r + 2N, ... of S rows
each (sky at the top and spheres at the bottom cost very differently, so contiguous
bands would be unbalanced; S = 8 keeps a rank's 8x8 work tiles compact in the image,
S = 1 interleaves single rows).  Every pixel's value is keyed by its global index, so the assembled
image is bitwise independent of N.  Assembly is ONE gather of the equal-sized shard
buffers to rank 0 (RCCL over xGMI with the "nccl" backend; gloo in the CPU tests),
then a de-interleave copy on rank 0.
"""
from __future__ import annotations


def shard_rows(height: int, rank: int, world: int, stripe: int = 1) -> int:
    """Rows of a shard (rtx_region_rows): the rows of stripes rank, rank + world, ... of `stripe` rows each
    (ceil((H - rank) / N) for single rows)."""
    S = max(stripe, 1)
    nst = (height + S - 1) // S
    if world <= 0 or rank >= world or rank >= nst:
        return 0
    rows = (nst - rank + world - 1) // world * S
    if (nst - 1) % world == rank and height % S:
        rows -= S - height % S
    return rows


def max_shard_rows(height: int, world: int, stripe: int = 1) -> int:
    """The padded size every shard buffer has: shard 0's rows rounded up to whole stripes."""
    S = max(stripe, 1)
    return (shard_rows(height, 0, world, S) + S - 1) // S * S


def deinterleave(stacked, height: int, stripe: int = 1):
    """stacked: [N, R, W, 3] (R a multiple of the stripe; shard d's row q*S + o = image row (q*N + d)*S + o)
    -> [H, W, 3]."""
    n, r, w, c = stacked.shape
    S = max(stripe, 1)
    full = stacked.reshape(n, r // S, S, w, c).permute(1, 0, 2, 3, 4).reshape(n * r, w, c)
    return full[:height]


def gather_image(shard, height: int, rank: int, world: int, dist=None, stripe: int = 1):
    """Gather padded shards [R, W, 3] (R = max_shard_rows) to rank 0 and return the
    full image there (None on other ranks).  With world == 1 the shard is the image."""
    if world == 1:
        return shard[:height]
    if dist is None:
        import torch.distributed as dist
    import torch

    if rank == 0:
        stacked = torch.empty((world,) + tuple(shard.shape), dtype=shard.dtype, device=shard.device)
        dist.gather(shard, gather_list=list(stacked.unbind(0)), dst=0)  # straight into one buffer
        return deinterleave(stacked, height, stripe)
    dist.gather(shard, gather_list=None, dst=0)
    return None
