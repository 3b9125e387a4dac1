"""Image sharding across ranks (one process per GPU) and the framebuffer gather.

Rows are interleaved: rank r renders rows y = r, r + N, r + 2N, ... (sky at the top
and spheres at the bottom cost very differently, so contiguous bands would be
unbalanced).  Every pixel's value is keyed by its global index, so the assembled
image is bitwise independent of N.  Assembly is ONE gather of the equal-sized shard
buffers to rank 0 (RCCL over xGMI with the "nccl" backend; gloo in the CPU tests),
then a de-interleave copy on rank 0.
"""
from __future__ import annotations


def shard_rows(height: int, rank: int, world: int) -> int:
    """Rows of a shard: ceil((H - rank) / N) (rtx_region_rows)."""
    if world <= 0 or rank >= world or height <= rank:
        return 0
    return (height - rank + world - 1) // world


def max_shard_rows(height: int, world: int) -> int:
    return shard_rows(height, 0, world)


def deinterleave(stacked, height: int):
    """stacked: [N, R, W, 3] (shard r row i = image row r + i*N) -> [H, W, 3]."""
    n, r, w, c = stacked.shape
    full = stacked.permute(1, 0, 2, 3).reshape(n * r, w, c)
    return full[:height]


def gather_image(shard, height: int, rank: int, world: int, dist=None):
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
        return deinterleave(stacked, height)
    dist.gather(shard, gather_list=None, dst=0)
    return None
