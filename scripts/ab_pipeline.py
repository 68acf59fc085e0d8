"""A/B the fused vs split bounce pipelines in ONE process (guide rule 24): interleaved rounds."""
import os, sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import torch
import cuda_pathtracer_amd as P
scene = P.Scene(str(ROOT / "tests" / "scenes" / "cornell.json"))
ctx = {}
for name in ("fused", "split"):
    os.environ["PT_PIPELINE"] = name
    ctx[name] = P.PathTracer(scene, P.GuiDataContainer())
res = {k: [] for k in ctx}
it = 1
for rnd in range(6):
    for name, pt in ctx.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            pt.render_pass(it)
            it += 1
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) / 50 * 1e3)
for k, v in res.items():
    v = sorted(v)
    seg = ctx[k].stats()["segments"] / ctx[k].stats()["passes"]
    print(f"{k}: ms/pass median {v[len(v)//2]:.4f} min {v[0]:.4f}  Mray/s {seg / (v[len(v)//2] * 1e-3) / 1e6:.1f}")
