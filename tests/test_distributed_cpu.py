"""Multi-process pixel sharding on the CPU with gloo (world_size 2 and 3), the same code path the
bench uses over RCCL: rank r renders rows y % world == r, one gather assembles the image on rank 0
(SURVEY.md §8e).  Each rank's shard is computed by the oracle (the GPU box runs the same
distributed.py with libpt_amd.so tiles); rank 0 checks the gathered image against shards
rendered in a single process, plus the max/sum reductions used for the bench's value.
"""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    from oracle import binding as O
    sc = O.OracleScene.from_json(ROOT / "tests" / "scenes" / "cornell.json")
    sc.cam = O.camera((24, 17), 45.0, (0.0, 5.0, 10.5), (0.0, 5.0, 0.0), (0.0, 1.0, 0.0))
    return sc


def _worker(rank, world, port, out_dir):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from cuda_pathtracer_amd import distributed as D
    from oracle import binding as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = _scene()
        W, H = sc.cam.res[0], sc.cam.res[1]
        fl = O.flags()
        tile = None
        for it in (1, 2):   # two passes accumulate into the tile
            tile, _ = O.render_pass(sc, fl, iter_first=it, rank=rank, world=world, image=tile)
        assert tile.shape == (D.shard_rows(H, rank, world), W, 3)
        # bench.py's own calls: one gather_tiles of the rank's tile, then assemble on rank 0
        tiles = D.gather_tiles(torch, dist, torch.from_numpy(tile), H)
        img = D.assemble([t.cpu().numpy() for t in tiles], H, world) if tiles is not None else None
        t = D.max_over_ranks(torch, dist, 1.0 + rank, torch.device("cpu"))
        n = D.sum_over_ranks(torch, dist, 10 * (rank + 1), torch.device("cpu"))
        # bench.py's N > 1 diagnostics: every rank's (elapsed, segments), rank order, on every rank
        rows = D.per_rank(torch, dist, (1.0 + rank, 10 * (rank + 1)), torch.device("cpu"))
        assert rows == [[1.0 + r, 10.0 * (r + 1)] for r in range(world)]
        sp = D.rank_spread(rows)
        assert sp["elapsed_max_s"] == t and sum(sp["segments"]) == n and sp["slowest_rank"] == world - 1
        assert abs(sp["elapsed_spread"] - world + 1) < 1e-12 and sp["segments_min"] == 10
        if rank == 0:
            np.save(Path(out_dir) / "gathered.npy", img)
            np.save(Path(out_dir) / "reduce.npy", np.array([t, n], np.float64))
        else:
            assert img is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_shard_and_gather(tmp_path, world):
    import torch.multiprocessing as mp
    from cuda_pathtracer_amd import distributed as D
    from oracle import binding as O
    O.lib()                       # build the oracle once before forking ranks
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    img = np.load(tmp_path / "gathered.npy")
    sc = _scene()
    H = sc.cam.res[1]
    parts = []
    for r in range(world):
        tile = None
        for it in (1, 2):
            tile, _ = O.render_pass(sc, O.flags(), iter_first=it, rank=r, world=world, image=tile)
        parts.append(tile)
    np.testing.assert_array_equal(img, D.assemble(parts, H, world))
    assert img.shape == (H, sc.cam.res[0], 3) and img.sum() > 0
    t, n = np.load(tmp_path / "reduce.npy")
    assert t == float(world) and n == 10 * world * (world + 1) // 2


def test_shard_rows_cover_image():
    from cuda_pathtracer_amd import distributed as D
    for H in (1, 7, 800, 1080, 2160):
        for world in (1, 2, 3, 4, 8):
            rows = [D.shard_rows(H, r, world) for r in range(world)]
            assert sum(rows) == H and max(rows) == D.max_shard_rows(H, world)
            owned = sorted(D.row_of(i, r, world) for r in range(world) for i in range(rows[r]))
            assert owned == list(range(H))
    with pytest.raises(ValueError):
        D.shard_rows(10, 2, 2)
