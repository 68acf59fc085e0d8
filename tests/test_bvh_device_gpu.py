"""the BVH built on the device (cuda_pathtracer_amd/csrc/bvh_build.hip) is the
host build's tree — flattened nodes and reordered triangles byte for byte — for the bundled room
scene, config 5's 100k-triangle scene and adversarial meshes (duplicated triangles, all-zero boxes
at the origin, coplanar slivers, sizes around the one-thread subtree threshold).  Reference:
BVH_tree.cpp:27-181 (build_bvh, traverse_bvh, build_bvh_tree); the host restatement is pinned to
the oracle's (libstdc++ partition) in test_mesh_cpu.py.  Both build times are printed."""
import ctypes as C
import json
from pathlib import Path

import numpy as np
import pytest

from cuda_pathtracer_amd import _native as N

pytestmark = pytest.mark.gpu

SCENES = Path(__file__).resolve().parent / "scenes"


def _tables(s):
    _, _, nt, nn, _ = s.counts()
    tris = (N.Triangle * max(nt, 1))()
    nodes = (N.BvhNode * max(nn, 1))()
    assert N.lib().pt_scene_get_triangles(s.handle, tris, nt) == nt
    assert N.lib().pt_scene_get_bvh(s.handle, nodes, nn) == nn
    return bytes(tris)[:nt * C.sizeof(N.Triangle)], bytes(nodes)[:nn * C.sizeof(N.BvhNode)], nn


def _both(path):
    from cuda_pathtracer_amd import Scene
    h = Scene(path)
    d = Scene(path, device_bvh=True)
    on_h, ms_h = h.bvh_build_info()
    on_d, ms_d = d.bvh_build_info()
    assert not on_h and on_d, "device build did not run on the device"
    th, nh, kh = _tables(h)
    td, nd, kd = _tables(d)
    return (th, nh, kh), (td, nd, kd), ms_h, ms_d


def _assert_same(path, what):
    (th, nh, kh), (td, nd, kd), ms_h, ms_d = _both(path)
    assert kh == kd, f"{what}: {kh} host nodes vs {kd} device nodes"
    if nh != nd:
        a = np.frombuffer(nh, np.uint8).reshape(kh, -1)
        b = np.frombuffer(nd, np.uint8).reshape(kd, -1)
        first = int(np.argwhere((a != b).any(axis=1))[0][0])
        fh = np.frombuffer(a[first].tobytes(), np.float32)[:6]
        fd = np.frombuffer(b[first].tobytes(), np.float32)[:6]
        ih = np.frombuffer(a[first].tobytes(), np.int32)[6:]
        idv = np.frombuffer(b[first].tobytes(), np.int32)[6:]
        raise AssertionError(f"{what}: first differing node {first}: host {fh} {ih} device {fd} {idv}")
    assert th == td, f"{what}: triangle order differs"
    print(f"{what}: {kh} nodes; host build {ms_h:.1f} ms, device build {ms_d:.1f} ms")
    return ms_h, ms_d


def test_room_device_bvh_equals_host(gpu_device):
    _assert_same(SCENES / "room.json", "room.json")


def test_100k_device_bvh_equals_host(gpu_device, tmp_path):
    from cuda_pathtracer_amd import scenes
    path = scenes.random_triangles(tmp_path, n=100_000)
    _assert_same(path, "random_triangles 100k")


def _mesh_scene(tmp_path, verts, name):
    (tmp_path / "Models").mkdir(exist_ok=True)
    lines = [f"v {x:.9g} {y:.9g} {z:.9g}" for x, y, z in verts.reshape(-1, 3)]
    lines += [f"f {3 * i + 1} {3 * i + 2} {3 * i + 3}" for i in range(len(verts))]
    (tmp_path / "Models" / f"{name}.obj").write_text("\n".join(lines) + "\n")
    scene = {"Materials": {"w": {"RGB": [0.9, 0.9, 0.9]}, "l": {"RGB": [1, 1, 1], "EMITTANCE": 5.0}},
             "Camera": {"RES": [16, 16], "FOVY": 45.0, "ITERATIONS": 1, "DEPTH": 4, "FILE": name,
                        "EYE": [0.0, 5.0, 10.5], "LOOKAT": [0.0, 5.0, 0.0], "UP": [0.0, 1.0, 0.0]},
             "Objects": [{"TYPE": "mesh", "MATERIAL": "w", "OBJ_FILE": f"{name}.obj", "TRANS": [0, 0, 0],
                          "ROTAT": [0, 0, 0], "SCALE": [1, 1, 1]},
                         {"TYPE": "cube", "MATERIAL": "l", "TRANS": [0, 10, 0], "ROTAT": [0, 0, 0],
                          "SCALE": [3, 0.3, 3]}]}
    p = tmp_path / f"{name}.json"
    p.write_text(json.dumps(scene))
    return p


@pytest.mark.parametrize("n,seed", [(1, 0), (2, 1), (3, 2), (9, 3), (128, 4), (129, 5), (300, 6), (5000, 7)])
def test_adversarial_meshes_device_bvh_equals_host(gpu_device, tmp_path, n, seed):
    """Random triangles mixed with exact duplicates (equal centres: leaves by the centre-box test),
    triangles collapsed to the origin (all-zero boxes: the `||` quirk's dropped leading boxes),
    axis-aligned slivers (zero-width boxes) and repeated coordinates (ties in the min/max folds)."""
    rng = np.random.default_rng(seed)
    v = rng.uniform(-3, 3, size=(n, 3, 3)).astype(np.float32)
    if n >= 3:
        k = max(1, n // 7)
        v[rng.choice(n, k, replace=False)] = v[0]                       # duplicates of triangle 0
        v[rng.choice(n, k, replace=False)] = 0.0                        # all-zero boxes at the origin
        s = rng.choice(n, k, replace=False)
        v[s, :, 1] = v[s, :1, 1]                                        # y-flat slivers
        v[rng.choice(n, k, replace=False), :, 0] = np.float32(1.25)     # shared x coordinate (ties)
    _assert_same(_mesh_scene(tmp_path, v, f"adv{n}_{seed}"), f"adversarial n={n}")


def test_render_with_device_bvh_equals_oracle(gpu_device):
    """A render on the device-built tree equals the oracle (the tree is the host one, so the
    traversal order and the first-found tie-break are the reference's)."""
    from oracle import binding as O
    from cuda_pathtracer_amd import GuiDataContainer, PathTracer, Scene
    room_path = str(SCENES / "room.json")
    s = Scene(room_path, device_bvh=True)
    s.set_camera((40, 40), 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    s.finalize()
    assert s.bvh_build_info()[0]
    pt = PathTracer(s, GuiDataContainer(), spp=2)
    pt.render_pass(1)
    img = pt.image()
    pt.free()
    o = O.OracleScene.from_json(room_path)
    o.set_camera((40, 40), 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    ref = O.render_pass(o, O.flags(), 1, spp=2)[0]
    assert np.array_equal(img, ref)


def _api_mesh_scene(verts, device):
    """The same triangles through pt_scene_add_mesh (the OBJ parser, like tinyobj's, reads no
    'nan'), the BVH built on the host or the device."""
    from cuda_pathtracer_amd import Scene
    sc = Scene()
    m = sc.add_material(rgb=(0.9, 0.9, 0.9))
    pos = np.ascontiguousarray(verts.reshape(-1), np.float32)
    n = len(verts)
    fs = np.full(n, 3, np.int32)
    ip = np.arange(3 * n, dtype=np.int32)
    gid = C.c_int32()
    f3 = lambda v: (C.c_float * 3)(*v)  # noqa: E731
    assert N.lib().pt_scene_add_mesh(sc.handle, m, f3([0, 0, 0]), f3([0, 0, 0]), f3([1, 1, 1]),
                                     pos.ctypes.data_as(N._FP), 3 * n, None, 0, None, 0,
                                     fs.ctypes.data_as(N._IP), n, ip.ctypes.data_as(N._IP), None, None,
                                     C.byref(gid)) == 0
    sc.set_camera((16, 16), 45.0, (0, 0, 10), (0, 0, 0))
    sc.set_bvh_builder(device)
    sc.finalize()
    return sc


@pytest.mark.parametrize("value", [1e30, -2e37])
def test_large_coordinates_device_bvh_equals_host(gpu_device, value):
    """Coordinates far from the rest (the loader accepts up to 2^126): bucket offsets of the
    other centres collapse towards 0 and the SAH splits peel the far triangles off; both builds
    agree."""
    rng = np.random.default_rng(11)
    v = rng.uniform(-3, 3, size=(300, 3, 3)).astype(np.float32)
    v[17, :, 2] = value
    v[200, 1, 0] = -value
    h = _api_mesh_scene(v, False)
    d = _api_mesh_scene(v, True)
    assert not h.bvh_build_info()[0] and d.bvh_build_info()[0]
    assert _tables(h) == _tables(d)
