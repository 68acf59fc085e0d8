"""Worker of tests/test_render_gpu.py::test_context_synchronisation_is_scoped, run in a fresh process so
that the only streams on the device are the two contexts' own (HIP maps a process's streams onto
GPU_MAX_HW_QUEUES = 4 hardware queues; streams beyond that share queues and run in submission order,
and a pytest process has made many streams by then).  Prints one JSON line."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> None:
    import numpy as np
    import torch
    from cuda_pathtracer_amd import GuiDataContainer, PathTracer, Scene
    from oracle import binding as O
    cornell = str(ROOT / "tests" / "scenes" / "cornell.json")
    s = Scene(cornell)
    s.set_camera((32, 24), 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    s.finalize()
    o = O.OracleScene.from_json(cornell)
    o.set_camera((32, 24), 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    small = PathTracer(s, GuiDataContainer())
    small.render_pass(1)
    ref, _ = O.render_pass(o, O.flags(), 1)
    first_ok = bool(np.array_equal(small.image(), ref))
    os.environ["PT_AMD_LANES"] = "1"
    big = PathTracer(Scene(cornell), GuiDataContainer(), spp=64)
    os.environ.pop("PT_AMD_LANES", None)
    big.render_pass(1)                    # warm-up pass (first launches, code objects)
    big.stats()
    ev = torch.cuda.Event()
    t0 = time.perf_counter()
    for k in range(1, 9):                 # 8 x 64 iterations of 800x800: tens of ms of GPU work
        big.render_pass(1 + 64 * k)
    ev.record()
    img = small.image()
    st = small.stats()
    t_small = time.perf_counter() - t0
    running = not ev.query()
    torch.cuda.synchronize()
    t_big = time.perf_counter() - t0
    bst = big.stats()
    out = {"first_ok": first_ok, "second_ok": bool(np.array_equal(img, ref)), "running": running,
           "t_small_ms": t_small * 1e3, "t_big_ms": t_big * 1e3, "small_live0": st["bounce_live"][0],
           "small_err": st["device_error"], "big_live0": bst["bounce_live"][0], "big_err": bst["device_error"]}
    big.free()
    small.free()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
