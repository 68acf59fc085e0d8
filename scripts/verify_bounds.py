"""GPU check of the bounded closest-hit pass: every ray of many render passes is
intersected twice — bounded pass and the plain per-geom loop — and any difference in t, material
or normal bits is counted (PT_AMD_VERIFY_BOUNDS=1, split pipeline, whose rays are the fused
kernel's).  Scenes: cornell.json, config 4's multi-object room at reduced size, and randomized
stress scenes (rotated, thin, overlapping cubes and spheres, glass).  Exit status 1 on any mismatch.

usage: python scripts/verify_bounds.py [passes] [random scenes] [iterations per pass]
"""
import os
import sys
from pathlib import Path

os.environ["PT_AMD_VERIFY_BOUNDS"] = "1"
os.environ["PT_PIPELINE"] = "split"
os.environ.setdefault("PT_AMD_NO_TORCH", "1")
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import cuda_pathtracer_amd as P  # noqa: E402
from cuda_pathtracer_amd import scenes as SG  # noqa: E402

passes = int(sys.argv[1]) if len(sys.argv) > 1 else 8
out = ROOT / "gpurun_out" / "verify_scenes"
cases = [("cornell", str(ROOT / "tests" / "scenes" / "cornell.json"), None, False),
         ("cornell_sorted", str(ROOT / "tests" / "scenes" / "cornell.json"), None, True),
         ("multi_object", SG.multi_object(out, res=(960, 540)), None, False)]
nrand = int(sys.argv[2]) if len(sys.argv) > 2 else 6
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 4
cases += [(f"random_primitives_{s}", SG.random_primitives(out, seed=s), None, s % 2 == 1) for s in range(1, nrand + 1)]
bad = tot = 0
for name, path, _, sort in cases:
    sc = P.Scene(path)
    g = P.GuiDataContainer()
    g.sortbyMaterial = sort
    pt = P.PathTracer(sc, g, spp=spp)
    for k in range(passes):
        pt.render_pass(1 + spp * k)
    st = pt.stats()
    pt.free()
    bad += st["bound_mismatch"]
    tot += st["segments"]
    print(f"{name:24s} sorted={int(sort)} segments={st['segments']:>12d} mismatches={st['bound_mismatch']}", flush=True)
print(f"TOTAL segments {tot} mismatches {bad}")
sys.exit(1 if bad else 0)
