"""The bench's multi-GPU data path on one GPU (8-GPU runs are the driver's): rank
processes render their row shards with libpt_amd.so, copy the tiles into device tensors and gather
them to rank 0 through cuda_pathtracer_amd.distributed.gather_tiles —
  * over RCCL (the "nccl" backend) in a world-size-1 group: the device-tensor branch the bench
    takes at N > 1 (two RCCL ranks cannot share one GPU);
  * over gloo with two ranks on the same GPU (gather_tiles moves the device tiles to the host).
With the shard-invariant shading key (rngKeyPixel) the assembled image equals a 1-GPU render bit
for bit.  Each rank is a child process (tests/dist_gpu_worker.py) under its own time limit."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _reference():
    from cuda_pathtracer_amd import GuiDataContainer, PathTracer, Scene
    s = Scene(str(ROOT / "tests" / "scenes" / "cornell.json"))
    s.set_camera((40, 37), 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    s.finalize()
    g = GuiDataContainer()
    g.rngKeyPixel = True
    pt = PathTracer(s, g, spp=2)
    for it in (1, 3):
        pt.render_pass(it)
    img = pt.image()
    pt.free()
    return img


@pytest.mark.parametrize("backend,world", [("nccl", 1), ("gloo", 2)])
def test_gather_tiles_on_device(gpu_device, tmp_path, backend, world):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PT_DIST_BACKEND=backend, PT_DIST_OUT=str(tmp_path))
        procs.append(subprocess.Popen([sys.executable, str(ROOT / "tests" / "dist_gpu_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=150)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    img = np.load(tmp_path / "gathered.npy")
    ref = _reference()
    assert img.shape == ref.shape and ref.sum() > 0
    np.testing.assert_array_equal(img, ref)
    t, n = np.load(tmp_path / "reduce.npy")
    assert t == float(world) and n == 10 * world * (world + 1) // 2
