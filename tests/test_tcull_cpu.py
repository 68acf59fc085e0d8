"""Why the 4-wide walk has no t-cull, checked on the CPU.

BVHIntersectionTest (intersections.cu:170-224) tests every triangle of every leaf whose box the ray
line crosses and keeps the first-found minimum of glm::intersectRayTriangle's computed t
(gtx/intersect.inl:37-74: one-sided, a < FLT_EPSILON rejected, t = f * dot(e2, q)).  A walk may skip
a subtree only if every triangle under it has computed t >= the best t found so far.  For a grazing
ray the computed t is far from the geometric one: a stays above FLT_EPSILON while its rounding error
is a sizeable fraction of it, and the error of t scales with |o - v0|.  This file pins one such ray
on config 5's own geometry (scenes.random_triangles, seed 5): triangle 65409 (|e1||e2| = 0.62, the
largest of the 100k) reports t = 0.75 for a ray that enters the triangle's own bounding box — and so
every BVH box holding it — only at t = 1.636.  Any cull of boxes entered beyond k x best with
k < 2.18 would drop this hit; a cull margin that is provable for every ray is therefore a large
multiple of best for config 5's triangles and removes little of the walk.

The arithmetic is glm's in float32 numpy (each operation correctly rounded, no FMA: the evaluation
contract of the kernels and the oracle, -ffp-contract=off), on the triangle as the product's loader
stores it (pt_scene_get_triangles).
"""
from __future__ import annotations

import numpy as np

import cuda_pathtracer_amd as P
from cuda_pathtracer_amd import _native as N
from cuda_pathtracer_amd import scenes

f32 = np.float32


def _cross(a, b):
    return np.array([f32(f32(a[1] * b[2]) - f32(a[2] * b[1])), f32(f32(a[2] * b[0]) - f32(a[0] * b[2])),
                     f32(f32(a[0] * b[1]) - f32(a[1] * b[0]))], f32)


def _dot(a, b):
    return f32(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2]))


def _ray_tri(v0, v1, v2, o, d):
    """glm::intersectRayTriangle (gtx/intersect.inl:37-74); oracle/pt_oracle.cpp ray_tri."""
    e1, e2 = (v1 - v0).astype(f32), (v2 - v0).astype(f32)
    p = _cross(d, e2)
    a = _dot(e1, p)
    if a < np.finfo(f32).eps:
        return None
    fi = f32(f32(1) / a)
    s = (o - v0).astype(f32)
    bx = f32(fi * _dot(s, p))
    if bx < 0 or bx > 1:
        return None
    q = _cross(s, e1)
    by = f32(fi * _dot(d, q))
    if by < 0 or f32(by + bx) > 1:
        return None
    bz = f32(fi * _dot(e2, q))
    return (bx, by, bz) if bz >= 0 else None


def test_grazing_ray_computed_t_far_before_the_box(tmp_path):
    path = scenes.random_triangles(tmp_path, n=100_000, res=(64, 36), depth=32)
    s = P.Scene(path)
    nt = s.counts()[2]
    arr = (N.Triangle * nt)()
    assert N.lib().pt_scene_get_triangles(s.handle, arr, nt) == nt
    tr = next(t for t in arr if t.id == 65409)
    v = np.array([list(tr.v[k]) for k in range(3)], f32)
    e1 = np.linalg.norm((v[1] - v[0]).astype(np.float64))
    e2 = np.linalg.norm((v[2] - v[0]).astype(np.float64))
    assert e1 * e2 > 0.6
    o = np.array([-0.8385278582572937, 5.838564872741699, -3.015523672103882], f32)
    d = np.array([-0.504230260848999, -0.8464691042900085, 0.17100246250629425], f32)
    assert abs(np.linalg.norm(d.astype(np.float64)) - 1.0) < 1e-6   # a normalized direction
    hit = _ray_tri(v[0], v[1], v[2], o, d)
    assert hit is not None and hit[2] == f32(0.75)
    # the exact entry parameter of the triangle's own box (any BVH box holding it contains it)
    lo, hi = v.astype(np.float64).min(0), v.astype(np.float64).max(0)
    inv = 1.0 / d.astype(np.float64)
    t1, t2 = (lo - o) * inv, (hi - o) * inv
    entry, exit_ = np.max(np.minimum(t1, t2)), np.min(np.maximum(t1, t2))
    assert entry <= exit_ and entry > 1.63
    assert float(hit[2]) / entry < 0.46
    # the geometric intersection of the ray line with the triangle's plane is near the box, not at 0.75
    n = np.cross((v[1] - v[0]).astype(np.float64), (v[2] - v[0]).astype(np.float64))
    t_geo = np.dot(v[0].astype(np.float64) - o, n) / np.dot(d.astype(np.float64), n)
    assert t_geo > 1.2


def _tcull_tables(path):
    import ctypes as C
    s = P.Scene(path)
    fr = C.c_double()
    n = N.lib().pt_scene_bvh_tcull(s.handle, None, 0, C.byref(fr))
    words = (C.c_uint32 * n)()
    assert N.lib().pt_scene_bvh_tcull(s.handle, words, n, C.byref(fr)) == n
    w = np.frombuffer(bytes(words), np.uint32).reshape(-1, 4)
    nq = N.lib().pt_scene_bvh_quads(s.handle, None, 0, None, None)
    buf = (C.c_uint8 * (128 * nq))()
    assert N.lib().pt_scene_bvh_quads(s.handle, buf, nq, None, None) == nq == len(w)
    q = np.frombuffer(bytes(buf), np.dtype([("b", "<f4", (6, 4)), ("code", "<i4", 4), ("meta", "<i4", 4)]))
    nt = s.counts()[2]
    arr = (N.Triangle * nt)()
    assert N.lib().pt_scene_get_triangles(s.handle, arr, nt) == nt
    tv = np.array([[list(t.v[k]) for k in range(3)] for t in arr], f32)   # BVH order
    return s, fr.value, w, q, tv


def _leaf_range(code):
    c = -int(code) - 1
    return c >> 8, (c >> 8) + (c & 255)


import pytest   # noqa: E402


@pytest.mark.parametrize("scene", ["tessellated", "config5"])
def test_tcull_margins_only_skip_worse_hits(tmp_path, scene):
    """The walk's exact t-cull (pt_kernels.hip k_traverse4; margins from build_qcull, DESIGN.md
    §4.3) enters no slot whose margin says A * tau_lo > B + best.  For leaf slots of the tessellated
    scene (the cull's case) and of config 5 (whose large triangles mostly get no margin), rays aimed
    at the leaf's triangles — a third of them grazing the triangle's plane at the FLT_EPSILON
    threshold — must give every computed glm t at or above the largest `best` the slot would be
    culled at: (A tau_lo)(1 - 2^-20) / (1 + 2^-20) - B, with tau_lo computed as the kernel does."""
    path = (scenes.tessellated_meshes(tmp_path, res=(64, 36)) if scene == "tessellated"
            else scenes.random_triangles(tmp_path, n=100_000, res=(64, 36), depth=32))
    _, frac, w, q, tv = _tcull_tables(path)
    assert (frac >= 0.25) == (scene == "tessellated")
    rng = np.random.default_rng(7)
    leaf_slots = [(qi, k) for qi in range(len(q)) for k in range(4)
                  if (q["meta"][qi, 0] >> k) & 1 and q["code"][qi, k] < 0 and (w[qi, k] & 0xffff) != 0]
    assert len(leaf_slots) > 100
    checked = hits = 0
    for idx in rng.choice(len(leaf_slots), size=min(400, len(leaf_slots)), replace=False):
        qi, k = leaf_slots[idx]
        A = float(np.array([w[qi, k] & 0xffff], np.uint16).view(np.float16)[0])
        B = float(np.array([w[qi, k] >> 16], np.uint16).view(np.float16)[0])
        lo_b = np.array([q["b"][qi, 0, k], q["b"][qi, 2, k], q["b"][qi, 4, k]], f32)
        hi_b = np.array([q["b"][qi, 1, k], q["b"][qi, 3, k], q["b"][qi, 5, k]], f32)
        t0, t1 = _leaf_range(q["code"][qi, k])
        for _ in range(12):
            ti = rng.integers(t0, t1)
            v = tv[ti].astype(np.float64)
            a_, b_ = rng.uniform(0, 1, 2)
            if a_ + b_ > 1:
                a_, b_ = 1 - a_, 1 - b_
            P_ = v[0] + a_ * (v[1] - v[0]) + b_ * (v[2] - v[0])
            n = np.cross(v[1] - v[0], v[2] - v[0])
            nn = np.linalg.norm(n)
            if nn == 0:
                continue
            nh = n / nn
            wv = rng.normal(size=3)
            wv -= wv.dot(nh) * nh
            wv /= np.linalg.norm(wv)
            sn = rng.uniform(0.05, 3.0) * 1.19e-7 / nn if rng.random() < 1 / 3 else rng.uniform(0.0, 1.0)
            sn = min(sn, 1.0)
            dd = wv * np.sqrt(1 - sn * sn) + nh * sn * (1 if rng.random() < 0.5 else -1)
            o = (P_ - rng.uniform(0.05, 10.0) * dd).astype(f32)
            d = dd.astype(f32)
            dsq = float(_dot(d, d))
            if not (1 - 2.0**-18 + 2.0**-22 <= dsq <= 1 + 2.0**-18 - 2.0**-22):
                continue
            # tau_lo as the kernel computes it (float32)
            s_ = np.where(d < 0, hi_b, lo_b).astype(f32)
            t = ((s_ - o).astype(f32) * d).astype(f32)
            tm = f32(f32(t[0] + t[1]) + t[2])
            sl = f32(f32(abs(t[0]) + abs(t[1])) + abs(t[2]))
            lo = f32(tm - f32(sl * f32(2.0**-20)))
            if lo <= 0:
                continue
            thr = (A * float(lo)) * (1 - 2.0**-20) / (1 + 2.0**-20) - B
            checked += 1
            for tj in range(t0, t1):
                h = _ray_tri(tv[tj][0], tv[tj][1], tv[tj][2], o, d)
                if h is not None:
                    hits += 1
                    assert float(h[2]) >= thr, (qi, k, tj, float(h[2]), thr)
    assert checked > 1000 and hits > 300


def test_tcull_words_follow_the_triangle_sizes(tmp_path):
    """build_qcull's words: binary16 A in [0, 1) and B >= 0 per valid slot; A is positive exactly
    where c = 9 max|e1||e2| (the subtree's largest triangle) stays below 1, and slots holding config
    5's largest triangles (|e1||e2| up to 0.62) get A = 0, B = inf — never culled."""
    path = scenes.tessellated_meshes(tmp_path / "t", res=(64, 36))
    _, frac, w, q, tv = _tcull_tables(path)
    A = (w & 0xffff).astype(np.uint16).view(np.float16).astype(np.float64)
    B = (w >> 16).astype(np.uint16).view(np.float16).astype(np.float64)
    valid = np.array([[(int(q["meta"][i, 0]) >> k) & 1 for k in range(4)] for i in range(len(q))], bool)
    assert frac == 1.0 and (A[valid] > 0.9).all() and (A[valid] < 1).all() and (B[valid] >= 0).all()
    path5 = scenes.random_triangles(tmp_path / "c", n=100_000, res=(64, 36), depth=32)
    _, frac5, w5, q5, tv5 = _tcull_tables(path5)
    A5 = (w5 & 0xffff).astype(np.uint16).view(np.float16).astype(np.float64)
    B5 = (w5 >> 16).astype(np.uint16).view(np.float16).astype(np.float64)
    e1 = np.linalg.norm((tv5[:, 1] - tv5[:, 0]).astype(np.float64), axis=1)
    e2 = np.linalg.norm((tv5[:, 2] - tv5[:, 0]).astype(np.float64), axis=1)
    big = int(np.argmax(e1 * e2))
    assert e1[big] * e2[big] > 0.6 and frac5 < 0.25
    # the leaf slot holding the largest triangle: no margin
    found = 0
    for i in range(len(q5)):
        for k in range(4):
            c = int(q5["code"][i, k])
            if (int(q5["meta"][i, 0]) >> k) & 1 and c < 0:
                t0, t1 = _leaf_range(c)
                if t0 <= big < t1:
                    assert A5[i, k] == 0 and np.isinf(B5[i, k])
                    found += 1
    assert found == 1
