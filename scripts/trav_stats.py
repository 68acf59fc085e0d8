"""BVH traversal counters of k_traverse / k_traverse4 (diagnostic library built with -DPT_TRAV_STATS,
cuda_pathtracer_amd/build.py build_trav_stats): rays, interior fetches and triangle tests per ray, and how many lanes of
the wave do useful work.  Usage: trav_stats.py scene.json [spp] (PT_AMD_TRAV=pairs: round 2's walk).

Definitions (one 'trip' = one iteration of the walk loop by one wave with at least one ray):
  trips_per_ray = lane-trips holding a ray / rays: the trips a ray spends in the walk [k_traverse4]
  busy       = lane-trips holding a ray / (64 x trips)                      [k_traverse4]
  inner_eff  = interior steps / (64 x trips that ran the interior branch)   [k_traverse4]
  task_eff   = triangle tests / (64 x K x trips that ran the triangle branch), K triangle tasks
               per lane                                                       [k_traverse4]
  lane_eff   = useful lane-steps / (64 x branch executions), the two branches weighted by their
               VALU cost (interior step = 1, triangle test = 1): the fraction of the lanes issued
               in the walk's two branches that carried work.  For k_traverse (both branches every
               trip, one step per lane) this is (pairs + tris) / (64 x 2 x trips).
  r02_metric = round 2's printed 'active-lane eff' formula, (pairs + tris) / (trips x rays/waves):
               kept for continuity; it scales with rays per wave and is not a lane fraction."""
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
buf = (C.c_ulonglong * 8)()
pt.render_pass(1)
lib().pt_debug_trav(buf, 1)
pt.render_pass(1 + spp)
lib().pt_debug_trav(buf, 0)
rays, inner, tris, trips, waves, busy, t_leaf, t_inner = (int(buf[k]) for k in range(8))
R = max(rays, 1)
quad = busy > 0
out = {"walk": "k_traverse4 (quads, leaf tasks)" if quad else "k_traverse (pairs)",
       "rays": rays, "interior_per_ray": round(inner / R, 1), "tris_per_ray": round(tris / R, 1),
       "trips_per_wave": round(trips / max(waves, 1), 1),
       "r02_metric": round((inner + tris) / max(trips * rays / max(waves, 1), 1), 3)}
if quad:
    # triangle tasks per lane: 2, or 1 where the exact t-cull is on (PT_AMD_WALK_TASKS forces it)
    K = int(os.environ.get("PT_AMD_WALK_TASKS") or (1 if pt.walk_info()["tcull"] else 2))
    out.update({"tasks_per_lane": K, "trips_per_ray": round(busy / R, 1),
                "busy": round(busy / max(64 * trips, 1), 3),
                "inner_eff": round(inner / max(64 * t_inner, 1), 3),
                "task_eff": round(tris / max(64 * K * t_leaf, 1), 3),
                "lane_eff": round((inner + tris) / max(64 * (t_inner + t_leaf), 1), 3)})
else:
    out.update({"simd_eff": round((inner + tris) / max(64 * trips, 1), 3),
                "lane_eff": round((inner + tris) / max(64 * 2 * trips, 1), 3)})
print(" ".join(f"{k}={v}" for k, v in out.items()))
pt.free()
