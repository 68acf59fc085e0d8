"""The exact t-cull forced on (PT_AMD_TCULL=1; TCULL=auto: each scene's default walk) with the device re-walk verification
(PT_AMD_VERIFY_BOUNDS=1: every mesh ray's record is compared with the reference's node-at-a-time
BVHIntersectionTest) over >= 1 G segments of config 5 at its benched 3840x2160, then the tessellated
workload (cull on by default there).  Prints segments and mismatches per pass."""
import os
import sys
import tempfile
import time
from pathlib import Path
os.environ["PT_AMD_VERIFY_BOUNDS"] = "1"
# TCULL=auto: the walk each scene gets by default (config 5: no cull, two triangle tasks per lane)
if os.environ.get("TCULL", "1") != "auto":
    os.environ["PT_AMD_TCULL"] = os.environ.get("TCULL", "1")
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import cuda_pathtracer_amd as P  # noqa: E402
from cuda_pathtracer_amd import scenes  # noqa: E402

d = tempfile.mkdtemp()
for name, path, spp, target, tmax in (("config 5 3840x2160", scenes.random_triangles(d), 16, 1_000_000_000, 600),
                                      ("tessellated 1920x1080", scenes.tessellated_meshes(d), 32, 500_000_000, 200)):
    s = P.Scene(path)
    pt = P.PathTracer(s, P.GuiDataContainer(), spp=spp)
    print(name, pt.walk_info(), flush=True)
    t0, it, seg, mism = time.time(), 1, 0, 0
    while seg < target and time.time() - t0 < tmax:
        pt.render_pass(it)
        it += spp
        st = pt.stats()
        seg, mism = st["segments"], st["bound_mismatch"]
        print(f"  iterations {it - 1}: segments {seg:,}  mismatches {mism}  device_error {st['device_error']}  "
              f"{time.time() - t0:.0f} s", flush=True)
        if mism or st["device_error"]:
            break
    pt.free()
    print(f"{name}: {seg:,} segments verified, {mism} mismatches", flush=True)
    if mism:
        sys.exit(1)
