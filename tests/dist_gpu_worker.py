"""One rank of tests/test_distributed_gpu.py (a child process; env: RANK, WORLD_SIZE, MASTER_ADDR,
MASTER_PORT, PT_DIST_BACKEND, PT_DIST_OUT).  The bench's N > 1 data path on one GPU: render this
rank's rows (rows y % world == rank) with the shard-invariant shading key, copy the tile into a
device tensor, ONE gather_tiles to rank 0, plus the max/sum reductions of the bench's timing."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main() -> None:
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    backend = os.environ["PT_DIST_BACKEND"]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import cuda_pathtracer_amd as P
        from cuda_pathtracer_amd import distributed as D
        s = P.Scene(str(ROOT / "tests" / "scenes" / "cornell.json"))
        s.set_camera((40, 37), 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
        s.finalize()
        g = P.GuiDataContainer()
        g.rngKeyPixel = True
        pt = P.PathTracer(s, g, rank=rank, world=world, spp=2)
        stream = torch.cuda.current_stream()
        for it in (1, 3):
            pt.render_pass(it, stream)
        tile = torch.empty((pt.rows, pt.width, 3), dtype=torch.float32, device=dev)
        pt.copy_image_to(tile.data_ptr(), stream)
        torch.cuda.synchronize()
        tiles = D.gather_tiles(torch, dist, tile, 37)
        t = D.max_over_ranks(torch, dist, 1.0 + rank, dev)
        n = D.sum_over_ranks(torch, dist, 10 * (rank + 1), dev)
        pt.free()
        if rank == 0:
            assert all(x.is_cuda == (backend == "nccl") for x in tiles)
            img = D.assemble([x.cpu().numpy() for x in tiles], 37, world)
            out = Path(os.environ["PT_DIST_OUT"])
            np.save(out / "gathered.npy", img)
            np.save(out / "reduce.npy", np.array([t, n], np.float64))
        else:
            assert tiles is None
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
