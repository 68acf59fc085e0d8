"""Regenerate the committed golden fixtures in tests/golden/ (test infrastructure).

Inputs follow the shape of the reference's own self-check (stream_compaction/src/main.cpp:14-146:
POT and NPOT sizes, last element forced to 0, values in [0,50) for scan and [0,4) for compaction)
and its scene files (path_tracer/scenes/cornell.json).  The reference run is time-seeded and its
renderer could not be run here, so the expected outputs come from the CPU
restatement in oracle/ — pinned independently by the known-answer tests in
tests/test_oracle_cpu.py (INSTRUCTION.md:262-302 vectors, numpy cumsum, the C++ standard's
minstd_rand check value).  The fixtures freeze that pinned behaviour so later changes to the
oracle or to the product cannot drift silently.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))

from oracle import binding as O  # noqa: E402

SEED = 0x5EED


def gen(n: int, maxval: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    a = rng.integers(0, maxval, size=n, dtype=np.int32)
    if n:
        a[-1] = 0
    return a


def scan_compact() -> dict:
    out = {}
    for tag, n in (("pot", 1 << 12), ("npot", (1 << 12) - 3), ("small", 7)):
        a = gen(n, 50, SEED + n)
        b = gen(n, 4, SEED + 2 * n)
        out[f"{tag}_scan_in"] = a
        out[f"{tag}_scan_out"] = O.scan(a)
        out[f"{tag}_compact_in"] = b
        out[f"{tag}_compact_out"] = O.compact_without_scan(b)
        perm, live = O.partition_indices(b)
        out[f"{tag}_partition_perm"] = perm
        out[f"{tag}_partition_live"] = np.array([live], np.int64)
    return out


RNG_KEYS = [(1, 0, 0), (1, 12345, 0), (7, 639999, 3), (5000, 77, 7), (1, 0, 63)]


def rng() -> dict:
    return {"keys": np.array(RNG_KEYS, np.int32),
            "u01": np.stack([O.u01_sequence(i, x, d, 16) for i, x, d in RNG_KEYS])}


SINCOS_X = np.array([0.0, 1e-6, 0.5, 1.0, 1.5707964, 3.1415927, 4.0, 6.2831855, -2.5, 100.0, 1000.5],
                    np.float32)


def sincos() -> dict:
    sc = np.array([O.sincos(float(x)) for x in SINCOS_X], np.float32)
    return {"x": SINCOS_X, "sin": sc[:, 0], "cos": sc[:, 1]}


def scene_small(res=32):
    sc = O.OracleScene.from_json(ROOT / "tests" / "scenes" / "cornell.json")
    c = sc.cam
    # same orbit camera at a smaller resolution (main.cpp:117-136 recompute is in oracle.camera)
    sc.cam = O.camera((res, res), 45.0, (0.0, 5.0, 10.5), (0.0, 5.0, 0.0), (0.0, 1.0, 0.0))
    del c
    return sc


RENDER_CASES = {
    "default": dict(),
    "nossaa_nodof_sort": dict(ssaa=False, dof=False, sort_by_material=True),
    "no_rr": dict(russian_roulette=False),
}


def render() -> dict:
    out = {}
    sc = scene_small()
    for name, kw in RENDER_CASES.items():
        img, live = O.render_pass(sc, O.flags(**kw), iter_first=1)
        img2, live2 = O.render_pass(sc, O.flags(**kw), iter_first=2, image=img.copy())
        out[f"{name}_image_1"] = img
        out[f"{name}_live_1"] = np.array(live, np.int64)
        out[f"{name}_image_2"] = img2
        out[f"{name}_live_2"] = np.array(live2, np.int64)
        out[f"{name}_tonemap_2"] = O.tonemap(img2, 2.0)
    return out


def transforms() -> dict:
    cases = np.array([[[0, 0, 0], [0, 0, 0], [1, 1, 1]],
                      [[0, 10, 0], [0, 0, 0], [10, .3, 10]],
                      [[-1, 4, -1], [0, 45, 0], [3, 3, 3]],
                      [[1.5, -2.25, 3], [30, -60, 90], [0.5, 2, 4]]], np.float32)
    T, I, IT = zip(*(O.build_transform(t, r, s) for t, r, s in cases))
    return {"trs": cases, "transform": np.stack(T), "inverse": np.stack(I), "inv_transpose": np.stack(IT)}


def main() -> None:
    for name, fn in (("scan_compact", scan_compact), ("rng", rng), ("sincos", sincos),
                     ("render_cornell32", render), ("transforms", transforms)):
        path = HERE / f"{name}.npz"
        np.savez_compressed(path, **fn())
        print(f"wrote {path.relative_to(ROOT)} ({path.stat().st_size} bytes)")


if __name__ == "__main__":
    main()

# REFERENCE_cornell.5000samp.png is the reference's course render (path_tracer/img/), copied
# verbatim as expected-output DATA for tests/test_render_gpu.py (the GPU box has no
# /root/reference); it is not generated here.
