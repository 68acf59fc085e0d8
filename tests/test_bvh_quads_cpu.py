"""The 4-wide BVH layout k_traverse4 walks (pt_kernels.hip DQuad, built by the product's host code
and read back through pt_scene_bvh_quads) against the reference's binary walk, on the CPU.

BVHIntersectionTest (intersections.cu:170-224; BoundingBox::intersect boundingbox.h:73-92) visits
the nodes whose boxes the ray hits, near child first by `dir_neg[axis]`, and tests the triangles of
every leaf it reaches in order; the closest hit's first-found tie-break makes that ORDER part of
the result.  Both walks are restated here in float32 numpy arithmetic, the binary one from the
flattened node array (pt_scene_get_bvh, byte-equal to the oracle's tree in test_mesh_cpu.py) and
the 4-wide one from the quad table, and the sequence of leaves reached must be identical for
every ray.  Also checks the layout's structure: codes in range, each leaf reachable once, the
nesting of collapsed children and the stack bound.  (No GPU: this guards the table the kernel
indexes before any GPU run.)
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import cuda_pathtracer_amd as P
from cuda_pathtracer_amd import _native as N
from oracle import binding as O

IDX_MASK = (1 << 21) - 1   # interior code = quad index | meta << 21
QUAD_DTYPE = np.dtype([("lox", "<f4", 4), ("hix", "<f4", 4), ("loy", "<f4", 4), ("hiy", "<f4", 4),
                       ("loz", "<f4", 4), ("hiz", "<f4", 4), ("code", "<i4", 4), ("meta", "<i4", 4)])
assert QUAD_DTYPE.itemsize == 128
f32 = np.float32


def _tables(s):
    nn = s.counts()[3]
    nodes = (N.BvhNode * max(nn, 1))()
    assert N.lib().pt_scene_get_bvh(s.handle, nodes, nn) == nn
    pn = np.frombuffer(bytes(nodes), O.NODE_DTYPE)[:nn]
    root, bound = C.c_int32(), C.c_int32()
    nq = N.lib().pt_scene_bvh_quads(s.handle, None, 0, C.byref(root), C.byref(bound))
    assert nq > 0
    buf = (C.c_uint8 * (128 * nq))()
    assert N.lib().pt_scene_bvh_quads(s.handle, buf, nq, C.byref(root), C.byref(bound)) == nq
    return pn, np.frombuffer(bytes(buf), QUAD_DTYPE), root.value, bound.value


def _slab(bmin, bmax, o, inv, finite):
    """BoundingBox::intersect's hit test in float32: glm's ternary min/max (reference) or
    fminf/fmaxf (the kernels' form for finite o and 1/d)."""
    m = (bmin - o) * inv
    M = (bmax - o) * inv
    if finite:
        lo = np.max(np.minimum(m, M))
        hi = np.min(np.maximum(m, M))
    else:
        mn = [m[a] if m[a] < M[a] else M[a] for a in range(3)]
        mx = [m[a] if m[a] > M[a] else M[a] for a in range(3)]
        lo = mn[0] if mn[0] > mn[1] else mn[1]
        lo = lo if lo > mn[2] else mn[2]
        hi = mx[0] if mx[0] < mx[1] else mx[1]
        hi = hi if hi < mx[2] else mx[2]
    return not (hi < 0) and not (lo > hi)


def _walk_binary(pn, o, d):
    """The reference's walk: leaves reached, in order, as (first triangle, count)."""
    inv = (f32(1) / d).astype(f32)
    neg = d < 0
    out, stack, cur = [], [], 0
    while True:
        n = pn[cur]
        if _slab(n["bmin"], n["bmax"], o, inv, False):
            if n["sub_areas"] > 0:
                out.append((int(n["first_area_idx"]), int(n["sub_areas"])))
                if not stack:
                    break
                cur = stack.pop()
            else:
                assert len(stack) < 64
                if neg[n["axis"]]:
                    stack.append(cur + 1)
                    cur = int(n["rchild_idx"])
                else:
                    stack.append(int(n["rchild_idx"]))
                    cur = cur + 1
        else:
            if not stack:
                break
            cur = stack.pop()
    return out


def _walk_quads(pn, Q, root_code, o, d, max_stack):
    """k_traverse4's walk (finite rays): root box, then quads; the same leaves, as (first, count)."""
    inv = (f32(1) / d).astype(f32)
    negm = int(d[0] < 0) | (int(d[1] < 0) << 1) | (int(d[2] < 0) << 2)
    out = []
    if not _slab(pn[0]["bmin"], pn[0]["bmax"], o, inv, True):
        return out, 0
    stack, code, deepest = [], root_code, 0
    while True:
        if code < 0:
            c = -code - 1
            out.append((c >> 8, c & 255))
            if not stack:
                break
            code = stack.pop()
            continue
        q = Q[code & IDX_MASK]
        meta = (code >> 21) & 1023   # the code carries its quad's meta (k_traverse4 reads it there)
        assert meta == int(q["meta"][0])
        hm = 0
        for k in range(4):
            lo = np.array([q["lox"][k], q["loy"][k], q["loz"][k]], f32)
            hi = np.array([q["hix"][k], q["hiy"][k], q["hiz"][k]], f32)
            if (meta >> k) & 1 and _slab(lo, hi, o, inv, True):
                hm |= 1 << k
        c = [int(x) for x in q["code"]]
        if (negm >> ((meta >> 6) & 3)) & 1:
            c[0], c[1] = c[1], c[0]
            hm = (hm & 12) | ((hm & 1) << 1) | ((hm >> 1) & 1)
        if (negm >> ((meta >> 8) & 3)) & 1:
            c[2], c[3] = c[3], c[2]
            hm = (hm & 3) | ((hm & 4) << 1) | ((hm >> 1) & 4)
        if (negm >> ((meta >> 4) & 3)) & 1:
            c = [c[2], c[3], c[0], c[1]]
            hm = ((hm & 3) << 2) | (hm >> 2)
        hits = [c[k] for k in range(4) if (hm >> k) & 1]
        if hits:
            stack.extend(reversed(hits[1:]))
            deepest = max(deepest, len(stack))
            code = hits[0]
        else:
            if not stack:
                break
            code = stack.pop()
    assert deepest <= max_stack
    return out, deepest


def _rays(pn, n, seed):
    rng = np.random.default_rng(seed)
    lo, hi = pn[0]["bmin"].astype(np.float64), pn[0]["bmax"].astype(np.float64)
    ext = hi - lo
    o = rng.uniform(lo - 0.3 * ext, hi + 0.3 * ext, size=(n, 3)).astype(f32)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o, d.astype(f32)


def _check_structure(pn, Q, root, bound):
    nq = len(Q)
    leaves = set()
    for q in Q:
        meta = int(q["meta"][0])
        valid = meta & 15
        assert valid in (5, 7, 13, 15), "each group has its first slot"
        for k in range(4):
            if not (valid >> k) & 1:
                continue
            cd = int(q["code"][k])
            if cd >= 0:
                assert (cd & IDX_MASK) < nq and (cd >> 21) == int(Q[cd & IDX_MASK]["meta"][0])
            else:
                c = -cd - 1
                leaves.add((c >> 8, c & 255))
    real = {(int(x["first_area_idx"]), int(x["sub_areas"])) for x in pn if x["sub_areas"] > 0}
    assert leaves == real, "every leaf is a slot of exactly the quads that reach it"
    assert (root & IDX_MASK) == 0 and (root >> 21) == int(Q[0]["meta"][0]) and 0 < bound <= 64


@pytest.mark.parametrize("which", ["room", "tri3000", "tri20000"])
def test_quad_walk_reaches_the_reference_leaves_in_order(tmp_path, which):
    from pathlib import Path
    from cuda_pathtracer_amd import scenes
    if which == "room":
        path = Path(__file__).resolve().parent / "scenes" / "room.json"
        nrays = 300
    else:
        path = scenes.random_triangles(tmp_path, n=int(which[3:]), res=(16, 9), depth=8)
        nrays = 150
    s = P.Scene(path)
    pn, Q, root, bound = _tables(s)
    _check_structure(pn, Q, root, bound)
    o, d = _rays(pn, nrays, seed=len(which))
    for i in range(nrays):
        a = _walk_binary(pn, o[i], d[i])
        b, _ = _walk_quads(pn, Q, root, o[i], d[i], bound)
        assert a == b, f"ray {i}: leaf sequences differ"


def test_quad_layout_is_smaller_and_shallower(tmp_path):
    """The collapse halves the interior fetches: about half as many entries as interior nodes."""
    from cuda_pathtracer_amd import scenes
    path = scenes.random_triangles(tmp_path, n=20000, res=(16, 9), depth=8)
    pn, Q, root, bound = _tables(P.Scene(path))
    interior = int((pn["sub_areas"] == 0).sum())
    assert len(Q) < 0.6 * interior
