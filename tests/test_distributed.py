"""Row-interleaved sharding + all_gather (go_raytracer_amd/shard.py) on 2 gloo
ranks: the assembled image equals the single-rank render bitwise.  The per-rank
tiles come from the CPU oracle here (no GPU); on the GPU box bench.py runs the
same code path over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import go_raytracer_amd as rt
    from go_raytracer_amd import shard
    from oracle import pyoracle
    t, cam, w, l = rt.demo_scene("cornell")
    cam.Width = 20
    cam.SamplesPerPixel = 4
    d = cam.derived()
    part, _ = pyoracle.render(t, w, l, cam, seed=9, threads=2, rank=rank, nranks=world)
    tile = torch.zeros((shard.tile_rows(d.height, world), d.width, 3))
    tile[: part.shape[0]] = torch.from_numpy(part)
    img = shard.gather_image(tile, d.height)
    if rank == 0:
        full, _ = pyoracle.render(t, w, l, cam, seed=9, threads=2)
        q.put(bool(np.array_equal(img.numpy(), full)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_assembles_bitwise(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


def test_assemble_unit():
    from go_raytracer_amd import shard
    H, n = 7, 3
    rp = shard.tile_rows(H, n)
    g = torch.full((n * rp, 1, 1), -1.0)
    for r in range(n):
        for i, row in enumerate(shard.rows_of_rank(H, r, n)):
            g[r * rp + i] = row
    out = shard.assemble(g, H, n)
    assert out[:, 0, 0].tolist() == list(range(H))
