"""Pixel sharding across GPUs: one process per GPU, rows y % world == rank, one gather at the end.

The reference renders on one GPU (PT/src/pathtrace.cu:437-525); SURVEY.md §8e: pixels are
independent, so rank r owns the rows y with y % world == r (row-interleaved for load balance:
the light and the open front make per-row cost uneven), scene data is replicated, and the only
collective is ONE gather of the float accumulators to rank 0 when the image is saved.  Message
per rank: ceil(H / world) * W * 12 bytes.

The device side of the partition lives in pt_kernels.hip (TileDev: global pixel index of a tile
row); this module is the host side: row bookkeeping, padding and the gather.  It is backend
agnostic — RCCL ("nccl") on the GPU box, gloo in the CPU tests.
"""
from __future__ import annotations

import numpy as np


def shard_rows(height: int, rank: int, world: int) -> int:
    """Number of image rows rank `rank` owns (rows y with y % world == rank)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad shard rank={rank} world={world}")
    return max(0, (height - rank + world - 1) // world)


def max_shard_rows(height: int, world: int) -> int:
    return (height + world - 1) // world


def row_of(tile_row: int, rank: int, world: int) -> int:
    """Global image row of local tile row `tile_row`."""
    return tile_row * world + rank


def assemble(tiles, height: int, world: int) -> np.ndarray:
    """Interleave per-rank tiles ((>= rows_r, W, 3) arrays, rank order) into the (H, W, 3) image."""
    if len(tiles) != world:
        raise ValueError(f"expected {world} tiles, got {len(tiles)}")
    width = np.asarray(tiles[0]).shape[1]
    full = np.zeros((height, width, 3), np.float32)
    for r, t in enumerate(tiles):
        rows = shard_rows(height, r, world)
        full[r::world] = np.asarray(t)[:rows]
    return full


def gather_tiles(torch, dist, tile, height: int, group=None):
    """ONE gather of every rank's (rows_r, W, 3) float32 tile to rank 0.  Returns the list of
    padded tiles (device tensors, rank order) on rank 0 and None elsewhere.  `tile` lives on the
    collective's device (cuda for RCCL, cpu for gloo).  Tiles are padded to ceil(H / world) rows
    so a single fixed-size gather suffices."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if dist.get_backend(group) == "gloo" and tile.is_cuda:   # gloo gathers host tensors
        tile = tile.cpu()
    rows = shard_rows(height, rank, world)
    if tile.dim() != 3 or tile.shape[0] < rows or tile.shape[2] != 3:
        raise ValueError(f"tile shape {tuple(tile.shape)} does not hold {rows} rows of RGB")
    send = torch.zeros((max_shard_rows(height, world), tile.shape[1], 3), dtype=torch.float32, device=tile.device)
    send[:rows] = tile[:rows]
    recv = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
    dist.gather(send, recv, dst=0, group=group)
    return recv if rank == 0 else None


def gather_image(torch, dist, tile, height: int, group=None):
    """gather_tiles + assemble: the (H, W, 3) numpy image on rank 0, None elsewhere."""
    tiles = gather_tiles(torch, dist, tile, height, group)
    if tiles is None:
        return None
    return assemble([t.cpu().numpy() for t in tiles], height, len(tiles))


def _coll_device(torch, dist, device):
    return torch.device("cpu") if dist.get_backend() == "gloo" else device


def max_over_ranks(torch, dist, seconds: float, device) -> float:
    """Wall time of the slowest rank (the bench's timed region ends when every rank is done)."""
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=_coll_device(torch, dist, device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(torch, dist, count: int, device) -> int:
    """Units (traced segments) processed by all ranks together."""
    t = torch.tensor([int(count)], dtype=torch.int64, device=_coll_device(torch, dist, device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def per_rank(torch, dist, values, device) -> list:
    """Every rank's `values` (a short list of numbers), in rank order, on every rank (one
    all_gather): the bench's per-rank elapsed time and segments, so an imbalanced N-GPU line can be
    diagnosed from the line itself."""
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=_coll_device(torch, dist, device))
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[float(x) for x in o.tolist()] for o in out]


def rank_spread(rows) -> dict:
    """Summary of per_rank((elapsed_s, segments)) rows: per-rank lists, min / max, and the spread of
    the elapsed time (max / min - 1) and of the segments (max / min - 1)."""
    el = [r[0] for r in rows]
    sg = [int(r[1]) for r in rows]
    return {"elapsed_s": el, "segments": sg,
            "elapsed_min_s": min(el), "elapsed_max_s": max(el),
            "elapsed_spread": max(el) / min(el) - 1.0 if min(el) > 0 else None,
            "segments_min": min(sg), "segments_max": max(sg),
            "segments_spread": max(sg) / min(sg) - 1.0 if min(sg) > 0 else None,
            "slowest_rank": int(max(range(len(el)), key=lambda i: el[i]))}
