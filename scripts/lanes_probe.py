"""Probe: throughput of L independent contexts (spp/L iterations each) rendering concurrently on
L streams of one GPU, against one context with spp iterations per pass (same paths per step)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import cuda_pathtracer_amd as P  # noqa: E402

scene = P.Scene(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tests", "scenes", "cornell.json"))
SPP, STEPS = 32, 30
for L in (1, 2, 4):
    pts = [P.PathTracer(scene, P.GuiDataContainer(), spp=SPP // L) for _ in range(L)]
    sts = [torch.cuda.Stream() for _ in range(L)]
    it = 1
    for _ in range(3):
        for p, s in zip(pts, sts):
            p.render_pass(it, s)
        it += SPP
    torch.cuda.synchronize()
    s0 = sum(p.stats()["segments"] for p in pts)
    t0 = time.perf_counter()
    for _ in range(STEPS):
        for k, (p, s) in enumerate(zip(pts, sts)):
            p.render_pass(it + k * (SPP // L), s)
        it += SPP
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    seg = sum(p.stats()["segments"] for p in pts) - s0
    print(f"lanes={L} {seg / dt / 1e6:.1f} Mray/s {dt / STEPS * 1e3:.3f} ms/step", flush=True)
    for p in pts:
        p.free()
