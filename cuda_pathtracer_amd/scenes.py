"""Synthetic workload scenes in the reference's JSON scene format (BASELINE.json configs 3-5).

Each generator writes a scene file (and, for meshes, an OBJ under Models/) into a directory and
returns its path; generation is deterministic for a given seed.  The files use only the keys the
reference loader reads (scene.cpp:33-219), plus the REFRACTIVE / IOR extension for config 4
(the reference loader ignores those keys — SURVEY.md §2 quirk 1 — so refraction is parity-unpinned
against the reference itself; the CPU oracle restates the build's refraction).  Scenes with glass
opt in with the top-level "Extensions": {"REFRACTION": true} (pt_scene_load_json_ex); without it
the loaders ignore the keys, as the reference's does.

  cornell_hd        config 3: cornell.json geometry, 1920x1080, DEPTH 16 (run with material sort on)
  multi_object      config 4: Cornell-style room with a grid of spheres and boxes — diffuse,
                    mirror and refractive materials — 3840x2160, DEPTH 8
  random_triangles  config 5: N random triangles (one OBJ mesh through the BVH path) in a lit
                    box, 3840x2160, DEPTH 32
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent

CORNELL_MATERIALS = {
    "light": {"TYPE": "Emitting", "RGB": [1.0, 1.0, 1.0], "EMITTANCE": 5.0},
    "diffuse_white": {"TYPE": "Diffuse", "RGB": [0.98, 0.98, 0.98]},
    "diffuse_red": {"TYPE": "Diffuse", "RGB": [0.85, 0.35, 0.35]},
    "diffuse_green": {"TYPE": "Diffuse", "RGB": [0.35, 0.85, 0.35]},
    "specular_white": {"TYPE": "Specular", "RGB": [0.98, 0.98, 0.98], "SPECRGB": [0.98, 0.98, 0.98],
                       "REFLECTIVE": 1.0},
}


def _room(light_scale=(3.0, 0.3, 3.0)):
    """The Cornell box shell of cornell.json: light, floor, ceiling, back, left, right walls."""
    def cube(mat, t, r, s):
        return {"TYPE": "cube", "MATERIAL": mat, "TRANS": list(t), "ROTAT": list(r), "SCALE": list(s)}
    return [
        cube("light", (0.0, 10.0, 0.0), (0, 0, 0), light_scale),
        cube("diffuse_white", (0.0, 0.0, 0.0), (0, 0, 0), (10.0, 0.01, 10.0)),
        cube("diffuse_white", (0.0, 10.0, 0.0), (0, 0, 90), (0.01, 10.0, 10.0)),
        cube("diffuse_white", (0.0, 5.0, -5.0), (0, 90, 0), (0.01, 10.0, 10.0)),
        cube("diffuse_red", (-5.0, 5.0, 0.0), (0, 0, 0), (0.01, 10.0, 10.0)),
        cube("diffuse_green", (5.0, 5.0, 0.0), (0, 0, 0), (0.01, 10.0, 10.0)),
    ]


def _camera(res, depth, iterations, name):
    return {"RES": list(res), "FOVY": 45.0, "ITERATIONS": iterations, "DEPTH": depth, "FILE": name,
            "EYE": [0.0, 5.0, 10.5], "LOOKAT": [0.0, 5.0, 0.0], "UP": [0.0, 1.0, 0.0]}


def _write(out_dir, name, scene) -> str:
    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    path = out / f"{name}.json"
    path.write_text(json.dumps(scene, indent=1))
    return str(path)


def cornell_hd(out_dir, res=(1920, 1080), depth=16) -> str:
    """Config 3: the bundled Cornell scene at a different resolution and depth."""
    scene = json.loads((_HERE.parent / "tests" / "scenes" / "cornell.json").read_text())
    scene["Camera"]["RES"] = list(res)
    scene["Camera"]["DEPTH"] = int(depth)
    scene["Camera"]["FILE"] = "cornell_hd"
    return _write(out_dir, "cornell_hd", scene)


def multi_object(out_dir, res=(3840, 2160), depth=8, grid=(4, 3), seed=4) -> str:
    """Config 4: spheres and boxes on a grid inside the box; materials cycle through diffuse,
    mirror and glass (REFRACTIVE/IOR extension)."""
    rng = np.random.default_rng(seed)
    mats = dict(CORNELL_MATERIALS)
    mats["glass"] = {"TYPE": "Refractive", "RGB": [0.98, 0.98, 0.98], "SPECRGB": [0.98, 0.98, 0.98],
                     "REFRACTIVE": 1.0, "IOR": 1.5}
    mats["mirror_gold"] = {"TYPE": "Specular", "RGB": [0.95, 0.8, 0.4], "SPECRGB": [0.95, 0.8, 0.4],
                           "REFLECTIVE": 1.0}
    mats["diffuse_blue"] = {"TYPE": "Diffuse", "RGB": [0.35, 0.35, 0.85]}
    cycle = ["diffuse_blue", "glass", "specular_white", "mirror_gold", "diffuse_white", "glass"]
    objs = _room()
    nx, nz = grid
    k = 0
    for iz in range(nz):
        for ix in range(nx):
            x = -3.0 + 6.0 * ix / max(nx - 1, 1)
            z = -2.5 + 4.0 * iz / max(nz - 1, 1)
            size = float(rng.uniform(0.9, 1.6))
            mat = cycle[k % len(cycle)]
            if k % 2 == 0:
                objs.append({"TYPE": "sphere", "MATERIAL": mat, "TRANS": [x, size / 2 + 0.01, z],
                             "ROTAT": [0.0, 0.0, 0.0], "SCALE": [size, size, size]})
            else:
                objs.append({"TYPE": "cube", "MATERIAL": mat, "TRANS": [x, size / 2 + 0.01, z],
                             "ROTAT": [0.0, float(rng.uniform(0, 90)), 0.0], "SCALE": [size, size, size]})
            k += 1
    scene = {"Materials": mats, "Camera": _camera(res, depth, 5000, "multi_object"), "Objects": objs,
             "Extensions": {"REFRACTION": True}}
    return _write(out_dir, "multi_object", scene)


def random_triangles(out_dir, n=100_000, res=(3840, 2160), depth=32, seed=5) -> str:
    """Config 5: n random small triangles in the box volume as one OBJ mesh (BVH path)."""
    rng = np.random.default_rng(seed)
    out = Path(out_dir)
    (out / "Models").mkdir(parents=True, exist_ok=True)
    centers = rng.uniform((-4.0, 0.5, -4.0), (4.0, 8.5, 2.0), size=(n, 3))
    verts = centers[:, None, :] + rng.normal(0.0, 0.12, size=(n, 3, 3))
    normals = np.cross(verts[:, 1] - verts[:, 0], verts[:, 2] - verts[:, 0])
    normals /= np.maximum(np.linalg.norm(normals, axis=1, keepdims=True), 1e-12)
    lines = ["# random triangles (cuda_pathtracer_amd.scenes.random_triangles)"]
    lines += [f"v {x:.6f} {y:.6f} {z:.6f}" for x, y, z in verts.reshape(-1, 3)]
    lines += [f"vn {x:.6f} {y:.6f} {z:.6f}" for x, y, z in normals]
    lines += [f"f {3 * i + 1}//{i + 1} {3 * i + 2}//{i + 1} {3 * i + 3}//{i + 1}" for i in range(n)]
    name = f"tri{n}"
    (out / "Models" / f"{name}.obj").write_text("\n".join(lines) + "\n")
    objs = _room(light_scale=(4.0, 0.3, 4.0))
    objs.append({"TYPE": "mesh", "MATERIAL": "diffuse_white", "OBJ_FILE": f"{name}.obj",
                 "TRANS": [0.0, 0.0, 0.0], "ROTAT": [0.0, 0.0, 0.0], "SCALE": [1.0, 1.0, 1.0]})
    scene = {"Materials": dict(CORNELL_MATERIALS), "Camera": _camera(res, depth, 5000, name), "Objects": objs}
    return _write(out_dir, name, scene)


def _grid_mesh(pos, nu, nv, wrap_v):
    """Quads of a (nu x nv) parametric grid (u wraps; v wraps when wrap_v) split into triangles."""
    idx = lambda i, j: (i % nu) * nv + (j % nv)
    faces = []
    for i in range(nu):
        for j in range(nv if wrap_v else nv - 1):
            a, b, c, d = idx(i, j), idx(i + 1, j), idx(i + 1, j + 1), idx(i, j + 1)
            faces += [(a, b, c), (a, c, d)]
    return pos.reshape(-1, 3), faces


def tessellated_meshes(out_dir, res=(1920, 1080), depth=16) -> str:
    """Not a BASELINE workload: 100k small triangles on two closed surfaces (a UV sphere of 60k
    triangles and a torus of 40k) in the lit box — the shape of a real tessellated model, where the
    4-wide walk's exact t-cull pays, unlike config 5's large random triangles."""
    out = Path(out_dir)
    (out / "Models").mkdir(parents=True, exist_ok=True)
    nu, nv = 200, 151
    th = np.linspace(0.0, 2.0 * np.pi, nu, endpoint=False)[:, None]
    ph = np.linspace(0.0, np.pi, nv)[None, :]
    sph = np.stack([np.sin(ph) * np.cos(th), np.cos(ph) + 0.0 * th, np.sin(ph) * np.sin(th)], axis=-1)
    sph = sph * 2.2 + np.array([-1.5, 3.2, -1.0])
    v1, f1 = _grid_mesh(sph, nu, nv, False)
    mu, mv = 200, 100
    a = np.linspace(0.0, 2.0 * np.pi, mu, endpoint=False)[:, None]
    b = np.linspace(0.0, 2.0 * np.pi, mv, endpoint=False)[None, :]
    R, r = 1.6, 0.55
    tor = np.stack([(R + r * np.cos(b)) * np.cos(a), r * np.sin(b) + 0.0 * a, (R + r * np.cos(b)) * np.sin(a)], axis=-1)
    tor = tor + np.array([2.2, 1.2, 0.5])
    v2, f2 = _grid_mesh(tor, mu, mv, True)
    verts = np.concatenate([v1, v2])
    faces = f1 + [(x + len(v1), y + len(v1), z + len(v1)) for x, y, z in f2]
    fa = np.array(faces)
    nrm = np.cross(verts[fa[:, 1]] - verts[fa[:, 0]], verts[fa[:, 2]] - verts[fa[:, 0]])
    nrm /= np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-12)
    lines = ["# tessellated sphere + torus (cuda_pathtracer_amd.scenes.tessellated_meshes)"]
    lines += [f"v {x:.6f} {y:.6f} {z:.6f}" for x, y, z in verts]
    lines += [f"vn {x:.6f} {y:.6f} {z:.6f}" for x, y, z in nrm]
    lines += [f"f {x + 1}//{i + 1} {y + 1}//{i + 1} {z + 1}//{i + 1}" for i, (x, y, z) in enumerate(faces)]
    name = f"tess{len(faces)}"
    (out / "Models" / f"{name}.obj").write_text("\n".join(lines) + "\n")
    objs = _room()
    objs.append({"TYPE": "mesh", "MATERIAL": "diffuse_white", "OBJ_FILE": f"{name}.obj",
                 "TRANS": [0.0, 0.0, 0.0], "ROTAT": [0.0, 0.0, 0.0], "SCALE": [1.0, 1.0, 1.0]})
    scene = {"Materials": dict(CORNELL_MATERIALS), "Camera": _camera(res, depth, 5000, name), "Objects": objs}
    return _write(out_dir, name, scene)


def random_primitives(out_dir, n=24, res=(640, 480), depth=8, seed=7, extra_materials=0) -> str:
    """Stress scene for the bounded closest-hit pass (not a BASELINE workload): the Cornell shell
    plus n cubes and spheres with random rotations and strongly non-uniform scales (thin slabs,
    needles), overlapping each other and the walls; diffuse, mirror and glass materials.
    `extra_materials` adds that many diffuse/mirror materials used round-robin (material-sort width)."""
    rng = np.random.default_rng(seed)
    mats = dict(CORNELL_MATERIALS)
    mats["glass"] = {"TYPE": "Refractive", "RGB": [0.98, 0.98, 0.98], "SPECRGB": [0.98, 0.98, 0.98],
                     "REFRACTIVE": 1.0, "IOR": 1.5}
    cycle = ["diffuse_white", "specular_white", "glass", "diffuse_red", "diffuse_green"]
    for k in range(extra_materials):
        c = [float(v) for v in rng.uniform(0.2, 0.95, 3)]
        mats[f"m{k:03d}"] = ({"TYPE": "Diffuse", "RGB": c} if k % 3 else
                             {"TYPE": "Specular", "RGB": c, "SPECRGB": c, "REFLECTIVE": 0.5})
    if extra_materials:
        cycle = [f"m{k:03d}" for k in range(extra_materials)] + cycle
    objs = _room()
    for k in range(n):
        scale = np.exp(rng.uniform(np.log(0.02), np.log(4.0), 3))
        if k % 3 == 0:
            scale[:] = scale[0]
        objs.append({"TYPE": "sphere" if k % 2 else "cube", "MATERIAL": cycle[k % len(cycle)],
                     "TRANS": [float(v) for v in rng.uniform((-4.5, 0.0, -4.5), (4.5, 9.5, 3.0))],
                     "ROTAT": [float(v) for v in rng.uniform(0.0, 360.0, 3)],
                     "SCALE": [float(v) for v in scale]})
    scene = {"Materials": mats, "Camera": _camera(res, depth, 5000, "random_primitives"), "Objects": objs,
             "Extensions": {"REFRACTION": True}}
    return _write(out_dir, f"random_primitives_{seed}" + (f"_m{extra_materials}" if extra_materials else ""), scene)


CONFIGS = {
    "cornell": None,   # the bundled scene itself (configs[1])
    "cornell_hd_sorted": cornell_hd,
    "multi_object_4k": multi_object,
    "random_triangles_100k": random_triangles,
    "tessellated_meshes_100k": tessellated_meshes,   # (not a BASELINE workload: the exact t-cull's case)
}
