"""BVH traversal counters of k_traverse (diagnostic library built with -DPT_TRAV_STATS):
rays, pair fetches and triangle tests per ray, and the SIMD efficiency of the walk
(lane steps / (waves x 64 x longest lane's steps)).  Usage: trav_stats.py [scene.json] [spp]."""
import ctypes as C
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
os.environ["PT_AMD_LIB"] = str(ROOT / "cuda_pathtracer_amd" / "build" / "libpt_amd_trav.so")
os.environ.setdefault("PT_AMD_NO_TORCH", "1")
sys.path.insert(0, str(ROOT))
import cuda_pathtracer_amd as P  # noqa: E402
from cuda_pathtracer_amd._native import lib  # noqa: E402

scene = sys.argv[1]
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 1
pt = P.PathTracer(P.Scene(scene), P.GuiDataContainer(), spp=spp)
buf = (C.c_ulonglong * 5)()
pt.render_pass(1)
lib().pt_debug_trav(buf, 1)
pt.render_pass(1 + spp)
lib().pt_debug_trav(buf, 0)
rays, pairs, tris, wmax, waves = (int(buf[k]) for k in range(5))
print(f"rays={rays} pairs/ray={pairs / max(rays, 1):.1f} tris/ray={tris / max(rays, 1):.1f} "
      f"lanes/wave={rays / max(waves, 1):.1f} simd_eff={(pairs + tris) / max(64 * wmax, 1):.3f} "
      f"(active-lane eff={(pairs + tris) / max(wmax * rays / max(waves, 1), 1):.3f})")
pt.free()
