"""Multi-rank path of bench.py on the CPU: one process per rank (gloo), row-interleaved
shards (rtx_region rank/world), gathered to rank 0 with dist.gather and de-interleaved
by raytracer-go_amd/dist.py.  On MI355X the same code runs with the "nccl" (RCCL)
backend; here each shard is rendered by the CPU oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import dist as rdist
import oracle_binding as ob
import rtx

W, SPP = 40, 3


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, out_path, stripe=1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene = ob.OracleScene(1)
    cam = ob.rand_spheres_camera(W, SPP, 50)
    H = cam.image_height
    reg = rtx.Region(0, 0, W, H, rank, world, stripe)
    rows = rdist.shard_rows(H, rank, world, stripe)
    assert rows == ob.region_rows(reg)
    R = rdist.max_shard_rows(H, world, stripe)
    shard = torch.zeros((R, W, 3), dtype=torch.float32)
    if rows:
        img, _ = ob.render(scene.desc, cam, 11, reg, ob.ORDER_ITERATIVE, threads=2)
        shard[:rows] = torch.from_numpy(img)
    full = rdist.gather_image(shard, H, rank, world, stripe=stripe)
    if rank == 0:
        np.save(out_path, full.numpy())
    else:
        assert full is None
    dist.barrier()
    dist.destroy_process_group()


# world 8: the driver's one-node scaling run (C3); stripe 8: rtx_render's and bench.py's bands (H = 22: 3 stripes,
# the last one partial, so ranks 3..7 hold no row), stripe 4 over 3 ranks: ragged
@pytest.mark.parametrize("world,stripe", [(2, 1), (3, 1), (8, 1), (2, 8), (8, 8), (3, 4)])
def test_sharded_gather_equals_single_render(built, tmp_path, world, stripe):
    out = str(tmp_path / "full.npy")
    mp.start_processes(worker, args=(world, free_port(), out, stripe), nprocs=world, join=True, start_method="spawn")
    got = np.load(out)
    scene = ob.OracleScene(1)
    cam = ob.rand_spheres_camera(W, SPP, 50)
    want, _ = ob.render(scene.desc, cam, 11, rtx.Region(0, 0, W, cam.image_height, 0, 1), ob.ORDER_ITERATIVE)
    assert got.shape == want.shape
    assert np.array_equal(got, want)


@pytest.mark.parametrize("H,world,stripe", [(7, 3, 1), (7, 3, 2), (1080, 8, 8), (1080, 8, 1), (37, 4, 8), (5, 8, 8),
                                            (2160, 8, 16)])
def test_deinterleave_layout(H, world, stripe):
    """Every image row exactly once: shard d's row i is image row rtx_region_row (stripes of `stripe` rows dealt
    round-robin); the row counts agree with the library's rtx_region_rows and the oracle's."""
    R = rdist.max_shard_rows(H, world, stripe)
    stacked = torch.full((world, R, 1, 1), -1.0)
    total = 0
    for r in range(world):
        reg = rtx.Region(0, 0, 1, H, r, world, stripe)
        n = rdist.shard_rows(H, r, world, stripe)
        assert n == rtx.region_rows(reg) == ob.region_rows(reg)
        total += n
        for i in range(n):
            S = max(stripe, 1)
            stacked[r, i] = float(((i // S) * world + r) * S + i % S)  # value = image row index
    assert total == H
    full = rdist.deinterleave(stacked, H, stripe)
    assert full[:, 0, 0].tolist() == [float(y) for y in range(H)]
