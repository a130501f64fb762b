"""Row-interleaved sharding + gather (go_raytracer_amd/shard.py) on 2-3 gloo
ranks: the assembled image equals the single-rank render bitwise.  The CPU tests
render the per-rank tiles with the oracle; the GPU test renders them with the HIP
path (every rank on cuda:0, one process per rank as torchrun starts them) and
gathers over gloo; bench.py runs the same gather over RCCL."""
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


def _worker(rank, world, port, q, backend, collective):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import go_raytracer_amd as rt
    from go_raytracer_amd import shard
    t, cam, w, l = rt.demo_scene("cornell")
    cam.Width = 20 if backend == "oracle" else 64
    cam.SamplesPerPixel = 4 if backend == "oracle" else 16
    d = cam.derived()
    if backend == "oracle":
        from oracle import pyoracle
        part, _ = pyoracle.render(t, w, l, cam, seed=9, threads=2, rank=rank, nranks=world)
    else:  # the HIP path: this rank's rows on cuda:0
        with rt.Scene(t, w, l) as sc:
            part, st = sc.render(cam, seed=9, rank=rank, nranks=world)
        assert st["rows"] == part.shape[0]
    tile = torch.zeros((shard.tile_rows(d.height, world), d.width, 3))
    tile[: part.shape[0]] = torch.from_numpy(part)
    if collective == "all_gather":
        img = shard.gather_image(tile, d.height)
    else:
        img = shard.gather_to_root(tile, d.height)
        assert (img is None) == (rank != 0)
    if rank == 0:
        if backend == "oracle":
            full, _ = pyoracle.render(t, w, l, cam, seed=9, threads=2)
        else:
            with rt.Scene(t, w, l) as sc:
                full, _ = sc.render(cam, seed=9)
        q.put(bool(np.array_equal(img.numpy(), full)))
    dist.barrier()
    dist.destroy_process_group()


def _run(world, backend, collective):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, backend, collective))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


@pytest.mark.parametrize("collective", ["all_gather", "gather"])
@pytest.mark.parametrize("world", [2, 3])
def test_gather_assembles_bitwise(world, collective):
    _run(world, "oracle", collective)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_hip_ranks_gather_bitwise(world):
    """One process per rank (torchrun's layout) rendering its rows through the HIP
    path, gathered to rank 0: bit-equal to a one-process render (camera.go:119-130)."""
    _run(world, "hip", "gather")


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
