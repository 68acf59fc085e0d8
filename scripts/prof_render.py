"""Render-only workload for rocprofv3 (no torch kernels, no scan): N passes of a scene,
`spp=K` iterations per pass (default 32, like bench.py).

usage: prof_render.py N [sort] [spp=K] [scene=PATH] [bvhcull]   (default scene: cornell.json)"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
os.environ.setdefault("PT_AMD_NO_TORCH", "1")
import cuda_pathtracer_amd as P  # noqa: E402

passes = int(sys.argv[1]) if len(sys.argv) > 1 else 20
opts = sys.argv[2:]
sort = "sort" in opts
spp = next((int(a[4:]) for a in opts if a.startswith("spp=")), 32)   # bench.py's default batch
scene = next((a[6:] for a in opts if a.startswith("scene=")), str(ROOT / "tests" / "scenes" / "cornell.json"))
s = P.Scene(scene)
g = P.GuiDataContainer()
g.sortbyMaterial = sort
g.bvhCull = "bvhcull" in opts
pt = P.PathTracer(s, g, spp=spp)
for k in range(passes):
    pt.render_pass(1 + k * spp)
st = pt.stats()
print(st["segments"], st["bounce_live"])
pt.free()
