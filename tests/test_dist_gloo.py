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


def worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene = ob.OracleScene(1)
    cam = ob.rand_spheres_camera(W, SPP, 50)
    H = cam.image_height
    reg = rtx.Region(0, 0, W, H, rank, world)
    rows = rdist.shard_rows(H, rank, world)
    assert rows == ob.region_rows(reg)
    R = rdist.max_shard_rows(H, world)
    shard = torch.zeros((R, W, 3), dtype=torch.float32)
    if rows:
        img, _ = ob.render(scene.desc, cam, 11, reg, ob.ORDER_ITERATIVE, threads=2)
        shard[:rows] = torch.from_numpy(img)
    full = rdist.gather_image(shard, H, rank, world)
    if rank == 0:
        np.save(out_path, full.numpy())
    else:
        assert full is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])  # 8: the driver's one-node scaling run (C3)
def test_sharded_gather_equals_single_render(built, tmp_path, world):
    out = str(tmp_path / "full.npy")
    mp.start_processes(worker, args=(world, free_port(), out), nprocs=world, join=True, start_method="spawn")
    got = np.load(out)
    scene = ob.OracleScene(1)
    cam = ob.rand_spheres_camera(W, SPP, 50)
    want, _ = ob.render(scene.desc, cam, 11, rtx.Region(0, 0, W, cam.image_height, 0, 1), ob.ORDER_ITERATIVE)
    assert got.shape == want.shape
    assert np.array_equal(got, want)


def test_deinterleave_layout():
    H, world = 7, 3
    R = rdist.max_shard_rows(H, world)
    stacked = torch.full((world, R, 1, 1), -1.0)
    for r in range(world):
        for i in range(rdist.shard_rows(H, r, world)):
            stacked[r, i] = float(r + i * world)  # value = image row index
    full = rdist.deinterleave(stacked, H)
    assert full[:, 0, 0].tolist() == [float(y) for y in range(H)]
