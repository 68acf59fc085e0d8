"""Mesh host path on the CPU: OBJ loading (tinyobjloader 1.0.6 semantics), world-space transform and
the SAH BVH, product (cuda_pathtracer_amd/csrc/pt_mesh.cpp) against the oracle's independent
restatement (oracle/mesh_oracle.cpp, which uses this toolchain's real libstdc++ nth_element /
partition like the reference's BVH_tree.cpp).  Reference: scene.cpp:94-173, BVH_tree.cpp:27-181,
boundingbox.h, tiny_obj_loader.h:425-723,890-944.
"""
from __future__ import annotations

import ctypes as C
import json
from pathlib import Path

import numpy as np
import pytest

import cuda_pathtracer_amd as P
from cuda_pathtracer_amd import _native as N
from oracle import binding as O

SCENES = Path(__file__).resolve().parent / "scenes"


def _product_tables(s):
    ng, nm, nt, nn, ntex = s.counts()
    tris = (N.Triangle * max(nt, 1))()
    nodes = (N.BvhNode * max(nn, 1))()
    assert N.lib().pt_scene_get_triangles(s.handle, tris, nt) == nt
    assert N.lib().pt_scene_get_bvh(s.handle, nodes, nn) == nn
    pt = np.frombuffer(bytes(tris), O.TRI_DTYPE)[:nt]
    pn = np.frombuffer(bytes(nodes), O.NODE_DTYPE)[:nn]
    return pt, pn


def _assert_same(scene_path):
    s = P.Scene(scene_path)
    o = O.OracleScene.from_json(scene_path)
    pt, pn = _product_tables(s)
    assert len(pt) == len(o.tris) and len(pn) == len(o.nodes)
    assert pt.tobytes() == o.tris.tobytes(), "triangles differ (order, ids or bits)"
    assert pn.tobytes() == o.nodes.tobytes(), "BVH nodes differ"
    for g, og in zip(s.geoms(), o.geoms):
        assert (g.type, g.material_id, g.tri_start, g.tri_end) == (og.type, og.materialid, og.tri_start, og.tri_end)
        assert list(g.min_bound) == list(og.min_bound) and list(g.max_bound) == list(og.max_bound)
    return s, o, pt, pn


def test_room_scene_matches_oracle():
    s, o, pt, pn = _assert_same(SCENES / "room.json")
    assert len(pt) == 2810 and s.counts()[4] == 2           # chair x3 + fan-triangulated wall, 2 JPEGs
    # every triangle appears once; ids are load-order indices; leaves cover the array exactly
    assert sorted(pt["id"].tolist()) == list(range(len(pt)))
    leaves = pn[pn["sub_areas"] > 0]
    assert int(leaves["sub_areas"].sum()) == len(pt)
    assert sorted(leaves["first_area_idx"].tolist()) == sorted(set(leaves["first_area_idx"].tolist()))
    inner = pn[pn["sub_areas"] == 0]
    assert (inner["rchild_idx"] > 0).all() and (inner["axis"] >= 0).all()


def test_geom_bound_keeps_flt_min_quirk():
    """scene.cpp:117: the max bound starts at FLT_MIN (smallest positive float), so a mesh lying
    entirely at z < 0 still reports max z = FLT_MIN."""
    s = P.Scene(SCENES / "room.json")
    wall = [g for g in s.geoms() if g.type == P.MESH][0]
    assert wall.max_bound[2] == np.float32(1.1754943508222875e-38)


OBJ_EDGE = """# edge cases of tinyobjloader 1.0.6's parser
v 1 2 3
v -1.5e0 2.25E+1 .5
v +0.125 -7e-3 4.000000001
v 1.0000000000001 2.5e-2 -3
v 10 20 30 1.0
vt 0.5 0.25
vt 1 0
vn 0 0 1
vn 0 1 0
g first
usemtl m
f 1 2 3
f 1/1 2/2 3/1
f 1//1 2//2 3//1 4//2
f -4/-2/-2 -3/-1/-1 -2/-2/-2 -1/-1/-1 1/1/1
o second
f 5 4 3 2 1\r
"""


def test_obj_parser_edge_cases(tmp_path):
    (tmp_path / "Models").mkdir()
    (tmp_path / "Models" / "edge.obj").write_bytes(OBJ_EDGE.encode())
    scene = {
        "Materials": {"white": {"RGB": [0.9, 0.9, 0.9]}, "light": {"RGB": [1, 1, 1], "EMITTANCE": 5.0}},
        "Camera": {"RES": [16, 16], "FOVY": 45.0, "ITERATIONS": 1, "DEPTH": 4, "FILE": "edge",
                   "EYE": [0.0, 5.0, 10.5], "LOOKAT": [0.0, 5.0, 0.0], "UP": [0.0, 1.0, 0.0]},
        "Objects": [
            {"TYPE": "mesh", "MATERIAL": "white", "OBJ_FILE": "edge.obj", "TRANS": [0.5, 1, -2],
             "ROTAT": [10, 20, 30], "SCALE": [1, 2, 0.5]},
            {"TYPE": "cube", "MATERIAL": "light", "TRANS": [0, 10, 0], "ROTAT": [0, 0, 0], "SCALE": [3, 0.3, 3]},
            {"TYPE": "mesh", "MATERIAL": "white", "OBJ_FILE": "edge.obj", "TRANS": [0, 0, 0],
             "ROTAT": [0, 0, 0], "SCALE": [1, 1, 1]},
        ],
    }
    path = tmp_path / "edge.json"
    path.write_text(json.dumps(scene))
    s, o, pt, pn = _assert_same(path)
    # 1 + 1 + 2 + 3 + 3 fan triangles per mesh, two meshes
    assert len(pt) == 2 * 10
    # untransformed second copy: parsed values (tinyobj arithmetic, then float).  ".5" has no
    # integer digit, which tinyobj's tryParseDouble rejects, so parseReal's default 0 is used.
    second = pt[pt["id"] >= 10]
    first_tri = second[second["id"] == 10][0]
    np.testing.assert_array_equal(first_tri["v"], np.array([[1, 2, 3], [-1.5, 22.5, 0.0], [0.125, -7e-3, 4.0]],
                                                           np.float32))


def test_programmatic_mesh_equals_obj(tmp_path):
    """pt_scene_add_mesh (the same fan triangulation from arrays) == the OBJ loader's result."""
    (tmp_path / "Models").mkdir()
    obj = "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nv 0.5 1.5 0\nvn 0 0 1\nvt 0 0\nvt 1 0\nvt 1 1\n" \
          "f 1/1/1 2/2/1 3/3/1 5/3/1 4/2/1\n"
    (tmp_path / "Models" / "p.obj").write_text(obj)
    scene = {"Materials": {"a": {"RGB": [1, 1, 1]}},
             "Camera": {"RES": [8, 8], "FOVY": 45.0, "ITERATIONS": 1, "DEPTH": 2, "FILE": "p",
                        "EYE": [0.0, 0.5, 3.0], "LOOKAT": [0.0, 0.5, 0.0], "UP": [0.0, 1.0, 0.0]},
             "Objects": [{"TYPE": "mesh", "MATERIAL": "a", "OBJ_FILE": "p.obj", "TRANS": [1, 2, 3],
                          "ROTAT": [0, 45, 0], "SCALE": [2, 2, 2]}]}
    (tmp_path / "p.json").write_text(json.dumps(scene))
    ref = P.Scene(tmp_path / "p.json")
    sc = P.Scene()
    m = sc.add_material(rgb=(1, 1, 1))
    pos = np.array([0, 0, 0, 1, 0, 0, 1, 1, 0, 0, 1, 0, 0.5, 1.5, 0], np.float32)
    nrm = np.array([0, 0, 1], np.float32)
    uv = np.array([0, 0, 1, 0, 1, 1], np.float32)
    fs = np.array([5], np.int32)
    ip = np.array([0, 1, 2, 4, 3], np.int32)
    inn = np.zeros(5, np.int32)
    it = np.array([0, 1, 2, 2, 1], np.int32)
    gid = C.c_int32()
    f3 = lambda v: (C.c_float * 3)(*v)  # noqa: E731
    rc = N.lib().pt_scene_add_mesh(sc.handle, m, f3([1, 2, 3]), f3([0, 45, 0]), f3([2, 2, 2]),
                                   pos.ctypes.data_as(N._FP), 5, nrm.ctypes.data_as(N._FP), 1,
                                   uv.ctypes.data_as(N._FP), 3, fs.ctypes.data_as(N._IP), 1,
                                   ip.ctypes.data_as(N._IP), inn.ctypes.data_as(N._IP), it.ctypes.data_as(N._IP),
                                   C.byref(gid))
    assert rc == 0 and gid.value == 0
    sc.set_camera((8, 8), 45.0, (0, 0.5, 3), (0, 0.5, 0))
    sc.finalize()
    a, _ = _product_tables(sc)
    b, _ = _product_tables(ref)
    assert len(a) == 3 and a.tobytes() == b.tobytes()
    bad = (C.c_int32 * 3)(0, 1, 9)
    assert N.lib().pt_scene_add_mesh(sc.handle, m, f3([0, 0, 0]), f3([0, 0, 0]), f3([1, 1, 1]),
                                     pos.ctypes.data_as(N._FP), 5, None, 0, None, 0,
                                     (C.c_int32 * 1)(3), 1, bad, None, None, None) != 0


def test_missing_obj_is_an_error(tmp_path):
    scene = {"Materials": {"a": {"RGB": [1, 1, 1]}},
             "Camera": {"RES": [8, 8], "FOVY": 45.0, "ITERATIONS": 1, "DEPTH": 2, "FILE": "p",
                        "EYE": [0.0, 0.5, 3.0], "LOOKAT": [0.0, 0.5, 0.0], "UP": [0.0, 1.0, 0.0]},
             "Objects": [{"TYPE": "mesh", "MATERIAL": "a", "OBJ_FILE": "none.obj", "TRANS": [0, 0, 0],
                          "ROTAT": [0, 0, 0], "SCALE": [1, 1, 1]}]}
    (tmp_path / "m.json").write_text(json.dumps(scene))
    with pytest.raises(N.PtError, match="OBJ"):
        P.Scene(tmp_path / "m.json")


def test_random_triangles_100k_bvh_matches_oracle(tmp_path):
    """Config 5's scene at full size: 100k triangles, product BVH == oracle BVH byte for byte."""
    from cuda_pathtracer_amd import scenes
    path = scenes.random_triangles(tmp_path, n=100_000)
    s, o, pt, pn = _assert_same(path)
    assert len(pt) == 100_000
    assert int(pn[pn["sub_areas"] > 0]["sub_areas"].sum()) == 100_000


@pytest.mark.parametrize("value", [np.nan, np.inf, 3e38])
def test_non_finite_mesh_vertices_are_rejected(value):
    """A world vertex that is not finite or beyond 2^126 would give the SAH build NaN or infinite
    centres and extents, every triangle in one bucket and an unbounded recursion (the reference's
    build has no defined result there); pt_scene_add_mesh refuses it with PT_ERR_ARG and leaves the
    scene unchanged."""
    sc = P.Scene()
    m = sc.add_material(rgb=(1, 1, 1))
    pos = np.array([0, 0, 0, 1, 0, 0, 0, 1, value], np.float32)
    f3 = lambda v: (C.c_float * 3)(*v)  # noqa: E731
    rc = N.lib().pt_scene_add_mesh(sc.handle, m, f3([0, 0, 0]), f3([0, 0, 0]), f3([1, 1, 1]),
                                   pos.ctypes.data_as(N._FP), 3, None, 0, None, 0, (C.c_int32 * 1)(3), 1,
                                   (C.c_int32 * 3)(0, 1, 2), None, None, None)
    assert rc == 1   # PT_ERR_ARG (include/pt_amd.h)
    assert sc.counts()[0] == 0 and sc.counts()[2] == 0
