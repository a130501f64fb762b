"""Image-space sharding across ranks.

Row r of the image belongs to rank r % nranks (row-interleaved: cost varies
strongly by row, e.g. the Cornell light region, so interleaving balances it).
Each rank renders its rows with the GLOBAL pixel index in the RNG key, so the
assembled image is bitwise independent of the rank count.  The per-rank tiles
are exchanged with one gather to rank 0 (RCCL over xGMI for the "nccl" backend,
gloo on CPU; the reference collects its row buffers in one place too,
camera.go:119-130) and de-interleaved there; gather_image keeps the all_gather
form for callers that want the image on every rank.
"""
import torch
import torch.distributed as dist


def rows_of_rank(height, rank, nranks):
    return range(rank, height, nranks)


def tile_rows(height, nranks):
    """rows per rank, padded to the maximum so every rank sends the same size."""
    return (height + nranks - 1) // nranks


def assemble(gathered, height, nranks):
    """gathered: [nranks * tile_rows, W, C] (rank-major) -> [height, W, C]."""
    rp = tile_rows(height, nranks)
    out = torch.empty((height,) + tuple(gathered.shape[1:]), dtype=gathered.dtype,
                      device=gathered.device)
    for r in range(nranks):
        rows = torch.arange(r, height, nranks, device=gathered.device)
        out[rows] = gathered[r * rp: r * rp + len(rows)]
    return out


def gather_image(tile, height, group=None):
    """All ranks' [tile_rows, W, C] tiles -> the full [height, W, C] image on every rank."""
    nranks = dist.get_world_size(group)
    gathered = torch.empty((nranks * tile.shape[0],) + tuple(tile.shape[1:]), dtype=tile.dtype,
                           device=tile.device)
    dist.all_gather_into_tensor(gathered, tile.contiguous(), group=group)
    return assemble(gathered, height, nranks)


def gather_to_root(tile, height, gathered=None, dst=0, group=None):
    """All ranks' [tile_rows, W, C] tiles -> the full [height, W, C] image on rank
    `dst` (None elsewhere): one gather, so only the destination receives the image.
    `gathered` ([nranks * tile_rows, W, C] on dst) may be passed to reuse a buffer."""
    nranks = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if rank == dst:
        if gathered is None:
            gathered = torch.empty((nranks * tile.shape[0],) + tuple(tile.shape[1:]),
                                   dtype=tile.dtype, device=tile.device)
        parts = list(gathered.split(tile.shape[0]))
        dist.gather(tile.contiguous(), parts, dst=dst, group=group)
        return assemble(gathered, height, nranks)
    dist.gather(tile.contiguous(), None, dst=dst, group=group)
    return None
