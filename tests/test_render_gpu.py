"""GPU renderer parity against the CPU restatement of the reference renderer (oracle/pt_oracle.cpp).

Under the evaluation contract the HIP kernels and the oracle perform identical
float32 operations, so the accumulated radiance must match BIT FOR BIT — a stronger bar than the
§8a tolerance (|d| <= 2/255 for 99% of pixels, mean luminance within 0.5%), which is also
asserted at full resolution as a backstop.
"""
import numpy as np
import pytest

from oracle import binding as O

pytestmark = pytest.mark.gpu


def _pair(cornell_path, res=(64, 64)):
    from cuda_pathtracer_amd import Scene
    s = Scene(cornell_path)
    s.set_camera(res, 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    s.finalize()
    o = O.OracleScene.from_json(cornell_path)
    o.set_camera(res, 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    return s, o


def _gui(**kw):
    from cuda_pathtracer_amd import GuiDataContainer
    g = GuiDataContainer()
    for k, v in kw.items():
        setattr(g, k, v)
    return g


def _oflags(g):
    return O.flags(g.russianRoulette, g.useBVHtree, g.useBBox, g.sortbyMaterial, g.useThrustPartition, g.SSAA,
                   g.DoF, g.aperture, g.focal_len, g.singleAlbedo, g.rngKeyPixel)


def _assert_bitexact(gpu, ref, what):
    g = np.asarray(gpu, np.float32)
    r = np.asarray(ref, np.float32)
    assert g.shape == r.shape, what
    same = (g == r) | (np.isnan(g) & np.isnan(r))
    bad = np.argwhere(~same)
    assert bad.size == 0, f"{what}: {len(bad)} mismatching values, first at {bad[:3].tolist()}: " \
                          f"gpu={g[tuple(bad[0])]!r} oracle={r[tuple(bad[0])]!r}"


def _run(scene, oscene, gui, iters, rank=0, world=1, spp=1):
    from cuda_pathtracer_amd import PathTracer
    pt = PathTracer(scene, gui, rank=rank, world=world, spp=spp)
    img = None
    live_ref = [0] * oscene.depth
    it = 1
    while it <= iters:
        pt.render_pass(it)
        img, live = O.render_pass(oscene, _oflags(gui), it, spp=spp, rank=rank, world=world, image=img)
        live_ref = [a + b for a, b in zip(live_ref, live)]
        it += spp
    gimg = pt.image()
    st = pt.stats()
    pt.free()
    return gimg, img, st, live_ref


def test_cornell_bitexact_default_flags(cornell_path):
    s, o = _pair(cornell_path)
    g, r, st, live = _run(s, o, _gui(), iters=3)
    _assert_bitexact(g, r, "cornell 64x64 x3")
    assert st["bounce_live"] == live
    assert st["segments"] == sum(live)
    assert r.sum() > 0


@pytest.mark.parametrize("kw", [
    dict(russianRoulette=False),
    dict(SSAA=False),
    dict(DoF=False),
    dict(SSAA=False, DoF=False, russianRoulette=False),
    dict(sortbyMaterial=True),
    dict(sortbyMaterial=True, russianRoulette=False),
    dict(useThrustPartition=True),
    dict(aperture=0.5, focal_len=7.0),
    dict(singleAlbedo=True),
    dict(singleAlbedo=True, sortbyMaterial=True),
    dict(sharedGPU=True),                          # claimed tile schedule, fused pipeline
    dict(sharedGPU=True, sortbyMaterial=True),     # claimed schedule in the sorted pipeline's compaction
    dict(rngKeyPixel=True),                        # shading RNG keyed by the global pixel
    dict(rngKeyPixel=True, sortbyMaterial=True),
])
def test_cornell_bitexact_flags(cornell_path, kw):
    s, o = _pair(cornell_path, (48, 40))
    g, r, st, live = _run(s, o, _gui(**kw), iters=2)
    _assert_bitexact(g, r, f"flags {kw}")
    assert st["bounce_live"] == live


def test_materials_reflective_refractive():
    """Mirror and (build-extension) refractive spheres; refraction reproduces glm 0.9.6.3 incl. NaN on TIR."""
    from cuda_pathtracer_amd import CUBE, SPHERE, Scene
    s, o = Scene(), O.OracleScene()
    for sc in (s, o):
        light = sc.add_material(rgb=(1, 1, 1), emittance=5.0)
        white = sc.add_material(rgb=(0.98, 0.98, 0.98))
        mirror = sc.add_material(rgb=(0.9, 0.9, 0.9), specrgb=(0.95, 0.95, 0.95), reflective=1.0)
        glass = sc.add_material(rgb=(0.95, 0.95, 0.95), refractive=1.0, ior=1.5)
        half = sc.add_material(rgb=(0.5, 0.7, 0.9), reflective=0.5)
        sc.add_geom(CUBE, light, (0, 10, 0), (0, 0, 0), (3, 0.3, 3))
        sc.add_geom(CUBE, white, (0, 0, 0), (0, 0, 0), (10, 0.01, 10))
        sc.add_geom(CUBE, white, (0, 5, -5), (0, 90, 0), (0.01, 10, 10))
        sc.add_geom(CUBE, half, (4, 2, -1), (30, 45, 10), (2, 2, 2))
        sc.add_geom(SPHERE, mirror, (-2, 3, -1), (0, 0, 0), (3, 3, 3))
        sc.add_geom(SPHERE, glass, (2, 4, 1), (0, 0, 0), (2.5, 2.5, 2.5))
        sc.set_camera((56, 48), 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    s.set_render(4, 8, "mat")
    s.finalize()
    o.depth = 8
    g, r, st, live = _run(s, o, _gui(), iters=3)
    _assert_bitexact(g, r, "reflective/refractive")
    assert st["bounce_live"] == live


def _coincident_scene():
    """Geoms whose bounds and exact distances tie: three identical axis-aligned cubes (world-box
    bounds) and two identical uniform spheres at the same place with different materials, a cube
    sharing a face with another, and the walls.  The reference keeps the first geom of equal t
    (`t < t_min`, pathtrace.cu:284-288), so a wrong tie-break changes the colours."""
    from cuda_pathtracer_amd import CUBE, SPHERE, Scene
    s, o = Scene(), O.OracleScene()
    for sc in (s, o):
        light = sc.add_material(rgb=(1, 1, 1), emittance=5.0)
        white = sc.add_material(rgb=(0.98, 0.98, 0.98))
        red = sc.add_material(rgb=(0.9, 0.2, 0.2))
        green = sc.add_material(rgb=(0.2, 0.9, 0.2))
        mirror = sc.add_material(rgb=(0.9, 0.9, 0.9), specrgb=(0.95, 0.95, 0.95), reflective=1.0)
        sc.add_geom(CUBE, light, (0, 10, 0), (0, 0, 0), (3, 0.3, 3))
        sc.add_geom(CUBE, white, (0, 0, 0), (0, 0, 0), (10, 0.01, 10))
        sc.add_geom(CUBE, white, (0, 5, -5), (0, 90, 0), (0.01, 10, 10))
        for m in (red, green, mirror):   # three coincident cubes
            sc.add_geom(CUBE, m, (-2.5, 2, -1), (0, 0, 0), (2, 2, 2))
        sc.add_geom(CUBE, green, (-0.5, 2, -1), (0, 0, 0), (2, 2, 2))   # shares the x = -1.5 face
        for m in (mirror, red):   # two coincident spheres
            sc.add_geom(SPHERE, m, (2.5, 3, 0), (0, 0, 0), (2.5, 2.5, 2.5))
        sc.set_camera((64, 48), 45.0, (0, 5, 10.5), (0, 3, 0), (0, 1, 0))
    s.set_render(4, 8, "tie")
    s.finalize()
    o.depth = 8
    return s, o


@pytest.mark.parametrize("kw", [dict(), dict(sortbyMaterial=True)])
def test_coincident_geoms_tie_break_bitexact(kw):
    """Exact ties between geoms (equal bounds, equal t): the bounded closest hit's tagged
    candidates (equal bounds differ only in their index bits) and its order-independent selection
    give the reference's first-geom choice — GPU == oracle bit for bit, fused and sorted."""
    s, o = _coincident_scene()
    g, r, st, live = _run(s, o, _gui(**kw), iters=3)
    _assert_bitexact(g, r, f"coincident geoms {kw}")
    assert st["bounce_live"] == live


def test_coincident_geoms_bounded_equals_plain_loop(monkeypatch):
    """The same scene under PT_AMD_VERIFY_BOUNDS=1: every ray's bounded hit equals the plain loop's."""
    from cuda_pathtracer_amd import PathTracer
    monkeypatch.setenv("PT_AMD_VERIFY_BOUNDS", "1")
    monkeypatch.setenv("PT_PIPELINE", "split")
    s, _ = _coincident_scene()
    pt = PathTracer(s, _gui(), spp=8)
    for k in range(2):
        pt.render_pass(1 + 8 * k)
    st = pt.stats()
    pt.free()
    assert st["bound_mismatch"] == 0
    assert st["segments"] > 10_000


@pytest.mark.parametrize("kw", [dict(), dict(sortbyMaterial=True)])
def test_glass_cubes_total_internal_reflection(kw):
    """Rotated glass cubes (config 4's glass objects are cubes): rays inside a cube meet its faces
    beyond the critical angle, glm::refract returns NaN (interactions.cu:70), and the next bounce's
    closest hit of those NaN rays is "no hit" without the per-geom loop (intersect_bounded's early
    return) — GPU == oracle bit for bit, batched and sorted."""
    from cuda_pathtracer_amd import CUBE, SPHERE, Scene
    s, o = Scene(), O.OracleScene()
    for sc in (s, o):
        light = sc.add_material(rgb=(1, 1, 1), emittance=5.0)
        white = sc.add_material(rgb=(0.98, 0.98, 0.98))
        glass = sc.add_material(rgb=(0.95, 0.95, 0.95), refractive=1.0, ior=1.5)
        dense = sc.add_material(rgb=(0.9, 0.95, 0.9), specrgb=(0.9, 0.9, 0.9), refractive=1.0, ior=2.4)
        sc.add_geom(CUBE, light, (0, 10, 0), (0, 0, 0), (3, 0.3, 3))
        sc.add_geom(CUBE, white, (0, 0, 0), (0, 0, 0), (10, 0.01, 10))
        sc.add_geom(CUBE, white, (0, 5, -5), (0, 90, 0), (0.01, 10, 10))
        for k in range(6):
            sc.add_geom(CUBE, glass if k % 2 else dense, (-4 + 1.6 * k, 1.5 + (k % 3), -1 + 0.4 * k),
                        (10.0 * k, 25 + 7.0 * k, 5.0 * k), (1.4, 1.4, 1.4))
        sc.add_geom(SPHERE, glass, (0, 6, 1), (0, 0, 0), (2.0, 2.0, 2.0))
        sc.set_camera((96, 72), 45.0, (0, 5, 10.5), (0, 3, 0), (0, 1, 0))
    s.set_render(4, 12, "glass")
    s.finalize()
    o.depth = 12
    g, r, st, live = _run(s, o, _gui(**kw), iters=2, spp=2)
    _assert_bitexact(g, r, f"glass cubes {kw}")
    assert st["bounce_live"] == live and r.sum() > 0


@pytest.mark.parametrize("rank,world,spp", [(0, 2, 1), (1, 2, 1), (0, 1, 2), (1, 3, 3), (2, 4, 4), (0, 1, 100),
                                             (3, 8, 256)])
def test_tiles_and_batched_samples(cornell_path, rank, world, spp):
    s, o = _pair(cornell_path, (40, 36))
    g, r, st, live = _run(s, o, _gui(), iters=spp * 2, rank=rank, world=world, spp=spp)
    _assert_bitexact(g, r, f"tile rank={rank} world={world} spp={spp}")
    assert st["bounce_live"] == live


@pytest.mark.parametrize("kw", [dict(), dict(sortbyMaterial=True)])
@pytest.mark.parametrize("pipeline", ["fused", "split"])
def test_batched_pass_equals_sequential_passes(cornell_path, monkeypatch, kw, pipeline):
    """On the device: one pass of 4 batched iterations == 4 one-iteration passes, bit for bit
    (per-iteration workgroup layout of k_bounce / k_iter_bases / (iteration, material) sort keys)."""
    from cuda_pathtracer_amd import PathTracer
    if pipeline == "split":
        monkeypatch.setenv("PT_PIPELINE", "split")
    s, o = _pair(cornell_path, (40, 36))
    pb = PathTracer(s, _gui(**kw), spp=4)
    pb.render_pass(3)
    gb, stb = pb.image(), pb.stats()
    pb.free()
    ps = PathTracer(s, _gui(**kw), spp=1)
    for it in (3, 4, 5, 6):
        ps.render_pass(it)
    gs, sts = ps.image(), ps.stats()
    ps.free()
    _assert_bitexact(gb, gs, f"batched vs sequential {kw} {pipeline}")
    assert stb["bounce_live"] == sts["bounce_live"]


def test_split_pipeline_back_to_back_batched_passes(cornell_path, monkeypatch):
    """The split (diagnostic) pipeline's look-back compaction while the previous pass's finalize still
    runs on its side stream: large batched passes back to back complete without a device error (its
    tiles are claimed, not statically co-resident, in batched passes) and equal the fused pipeline."""
    from cuda_pathtracer_amd import PathTracer
    s, _ = _pair(cornell_path, (320, 240))
    out = []
    for pipeline in ("split", "fused"):
        if pipeline == "split":
            monkeypatch.setenv("PT_PIPELINE", "split")
        else:
            monkeypatch.delenv("PT_PIPELINE", raising=False)
        pt = PathTracer(s, _gui(), spp=32)
        for k in range(4):
            pt.render_pass(1 + 32 * k)
        st = pt.stats()
        out.append((pt.image(), st["bounce_live"], st["device_error"]))
        pt.free()
    assert out[0][2] == 0 and out[1][2] == 0
    _assert_bitexact(out[0][0], out[1][0], "split vs fused, 4 x 32 iterations")
    assert out[0][1] == out[1][1]


def test_rng_key_pixel_shards_equal_single_gpu(cornell_path):
    """§8e's shard-invariant mode on the device: with rngKeyPixel the 3-way row shards, assembled,
    equal the 1-GPU image bit for bit — and so does the material-sorted pipeline."""
    from cuda_pathtracer_amd import PathTracer, distributed
    s, o = _pair(cornell_path, (40, 37))

    def render(rank, world, **kw):
        pt = PathTracer(s, _gui(rngKeyPixel=True, **kw), rank=rank, world=world, spp=2)
        for it in (1, 3):
            pt.render_pass(it)
        img = pt.image()
        pt.free()
        return img

    full = render(0, 1)
    assert full.sum() > 0
    parts = [render(r, 3) for r in range(3)]
    _assert_bitexact(distributed.assemble(parts, 37, 3), full, "assembled shards vs 1 GPU")
    _assert_bitexact(render(0, 1, sortbyMaterial=True), full, "sorted vs unsorted")


def test_preview_rgba_matches_sendImageToPBO(cornell_path, gpu_device):
    import torch
    from cuda_pathtracer_amd import PathTracer
    s, o = _pair(cornell_path, (32, 32))
    pt = PathTracer(s, _gui())
    for it in (1, 2):
        pt.render_pass(it)
    buf = torch.zeros(32 * 32 * 4, dtype=torch.uint8, device=gpu_device)
    pt.preview_rgba(2, buf.data_ptr())
    torch.cuda.synchronize()
    img = pt.image()
    ref = np.zeros(32 * 32 * 4, np.uint8)
    O.lib().oracle_preview(np.ascontiguousarray(img).ctypes.data, 32, 32, 2, ref.ctypes.data)
    np.testing.assert_array_equal(buf.cpu().numpy(), ref)
    pt.free()


def test_render_iteration_and_get_accum(cornell_path, gpu_device):
    """The §8b entry points: pt_render_iteration (pass + preview of iter + spp - 1 samples) and
    pt_get_accum give the same bits as pt_render_pass / pt_preview_rgba / pt_get_image."""
    import ctypes as C
    import torch
    from cuda_pathtracer_amd import PathTracer, lib
    s, o = _pair(cornell_path, (24, 20))
    pt = PathTracer(s, _gui(), spp=2)
    buf = torch.zeros(24 * 20 * 4, dtype=torch.uint8, device=gpu_device)
    for it in (1, 3):
        assert lib().pt_render_iteration(pt._h, it, C.c_void_p(buf.data_ptr()), None) == 0
    torch.cuda.synchronize()
    acc = np.zeros(24 * 20 * 3, np.float32)
    assert lib().pt_get_accum(pt._h, acc.ctypes.data) == 0
    pt.free()
    r = None
    for it in (1, 3):
        r, _ = O.render_pass(o, _oflags(_gui()), it, spp=2, image=r)
    _assert_bitexact(acc.reshape(r.shape), r, "pt_get_accum")
    ref = np.zeros(24 * 20 * 4, np.uint8)
    O.lib().oracle_preview(np.ascontiguousarray(r).ctypes.data, 24, 20, 4, ref.ctypes.data)
    np.testing.assert_array_equal(buf.cpu().numpy(), ref)


@pytest.mark.slow
def test_cornell_full_resolution(cornell_path):
    """The bundled scene as-is (800x800, DEPTH 8, default flags): bit-exact over 2 iterations, and the
    §8a tolerance as a backstop."""
    from cuda_pathtracer_amd import Scene, tonemap
    s = Scene(cornell_path)
    o = O.OracleScene.from_json(cornell_path)
    g, r, st, live = _run(s, o, _gui(), iters=2)
    _assert_bitexact(g, r, "cornell 800x800 x2")
    tg, tr = tonemap(g, 2).astype(int), O.tonemap(r, 2).astype(int)
    assert (np.abs(tg - tr) <= 2).mean() >= 0.99
    lum = lambda x: (x * np.array([0.2126, 0.7152, 0.0722], np.float32)).sum()  # noqa: E731
    assert abs(lum(g) - lum(r)) <= 0.005 * lum(r)


def test_cornell_256spp_tolerance(cornell_path):
    """§8a's stated radiance tolerance at >= 256 spp (16 passes of 16 batched samples, 128x128):
    per-pixel |d| <= 2/255 on the tone-mapped image for >= 99% of pixels and mean relative
    luminance within 0.5% — here the result is also bit-exact."""
    s, o = _pair(cornell_path, (128, 128))
    g, r, st, live = _run(s, o, _gui(), iters=256, spp=16)
    _assert_bitexact(g, r, "cornell 128x128 256spp")
    tg, tr = _tonemap_pair(g, r, 256)
    assert (np.abs(tg - tr) <= 2).mean() >= 0.99
    assert abs(_lum(g) - _lum(r)) <= 0.005 * _lum(r)


def _tonemap_pair(g, r, samples):
    from cuda_pathtracer_amd import tonemap
    return tonemap(g, samples).astype(int), O.tonemap(r, samples).astype(int)


def _lum(x):
    return float((np.asarray(x, np.float64) * np.array([0.2126, 0.7152, 0.0722])).sum())


def _course_render(cornell_path, single_albedo: bool):
    from cuda_pathtracer_amd import PathTracer, Scene, tonemap
    s = Scene(cornell_path)
    pt = PathTracer(s, _gui(singleAlbedo=single_albedo), spp=50)
    for it in range(1, 5001, 50):
        pt.render_pass(it)
    img = pt.image()
    pt.free()
    return tonemap(img, 5000).astype(np.int32)          # same x-mirror as the reference's PNG


@pytest.mark.slow
def test_statistical_match_with_reference_course_render(cornell_path):
    """The reference's only radiance artefact, path_tracer/img/REFERENCE_cornell.5000samp.png
    (800x800, 5000 samples; committed as a fixture under tests/golden/), against our render of
    cornell.json at 5000 samples.

    The reference CODE multiplies the path colour by the albedo twice (interactions.cu:60 and :83);
    its IMAGE matches the single-albedo model, which therefore pins camera, geometry, sampling,
    Russian roulette and tone mapping against the reference's own output.  The sample streams
    differ (the image came from an unknown build), so the match is statistical, not per pixel:
    §8a's mean relative luminance error <= 0.5%, every channel mean within 0.5%, 16x16 block means
    within 1/255 on average, per-pixel mean |d| < 3.5/255 (Monte Carlo noise at 5000 spp).  The
    reference-exact (double-albedo) model is ~25% darker, as that quirk predicts."""
    from pathlib import Path
    from PIL import Image
    ref = np.asarray(Image.open(Path(__file__).parent / "golden" / "REFERENCE_cornell.5000samp.png").convert("RGB"))
    ref = ref.astype(np.int32)
    ours1 = _course_render(cornell_path, True)
    d = np.abs(ours1 - ref)
    lum = lambda x: float((x * np.array([0.2126, 0.7152, 0.0722])).sum())  # noqa: E731
    rel_lum = abs(lum(ours1) - lum(ref)) / lum(ref)
    rel_ch = np.abs(ours1.mean(axis=(0, 1)) - ref.mean(axis=(0, 1))) / ref.mean(axis=(0, 1))
    blocks = lambda x: x.reshape(50, 16, 50, 16, 3).mean(axis=(1, 3))  # noqa: E731
    block_mad = float(np.abs(blocks(ours1) - blocks(ref)).mean())
    ours2 = _course_render(cornell_path, False)
    ratio2 = ours2.mean(axis=(0, 1)) / ref.mean(axis=(0, 1))
    print(f"course image: single-albedo rel_lum={rel_lum:.5f} rel_ch={rel_ch} block MAD={block_mad:.3f} "
          f"pixel mean|d|={float(d.mean()):.3f} <=2/255={float((d.max(axis=2) <= 2).mean()):.4f}; "
          f"reference-exact/course channel ratio {ratio2}")
    assert rel_lum <= 0.005 and (rel_ch <= 0.005).all()
    assert block_mad <= 1.0 and float(d.mean()) < 3.5
    assert ((ratio2 < 0.85) & (ratio2 > 0.6)).all()


@pytest.fixture(scope="module")
def room_path():
    from pathlib import Path
    return str(Path(__file__).parent / "scenes" / "room.json")


def _room_pair(room_path, res=(40, 40)):
    from cuda_pathtracer_amd import Scene
    s = Scene(room_path)
    s.set_camera(res, 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    s.finalize()
    o = O.OracleScene.from_json(room_path)
    o.set_camera(res, 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    return s, o


@pytest.mark.parametrize("kw", [
    dict(),                                       # BVH (default flags)
    dict(useBVHtree=False),                       # linear mesh loop + world-AABB cull
    dict(useBVHtree=False, useBBox=False),        # linear mesh loop, no cull
    dict(sortbyMaterial=True),
    dict(singleAlbedo=True, russianRoulette=False),
    dict(bvhCull=True),                           # extension: same image, fewer node visits
])
def test_room_meshes_textures_bitexact(room_path, kw):
    """room.json: three chairs (OBJ, fan-triangulated quads/octagons) + a textured wall mesh, one
    SAH BVH over all 2810 triangles, JPEG textures (scene.cpp:94-173, intersections.cu:119-224,
    sceneStructs.h:171-189) — GPU == oracle bit for bit."""
    s, o = _room_pair(room_path)
    g, r, st, live = _run(s, o, _gui(**kw), iters=2)
    _assert_bitexact(g, r, f"room {kw}")
    assert live[0] == 2 * 40 * 40 and r.sum() > 0


@pytest.fixture(scope="module")
def config_scenes(tmp_path_factory):
    """BASELINE.json configs 3-5 generated at parity-test sizes (cuda_pathtracer_amd.scenes)."""
    from cuda_pathtracer_amd import scenes
    d = tmp_path_factory.mktemp("configs")
    return {
        "cornell_hd": scenes.cornell_hd(d, res=(96, 54), depth=16),
        "multi_object": scenes.multi_object(d, res=(64, 36), depth=8),
        "random_triangles": scenes.random_triangles(d, n=3000, res=(48, 27), depth=32),
        "random_primitives_1": scenes.random_primitives(d, res=(64, 48), seed=1),
        "random_primitives_2": scenes.random_primitives(d, res=(64, 48), seed=2),
    }


@pytest.mark.parametrize("name,kw", [
    ("cornell_hd", dict(sortbyMaterial=True)),            # config 3: DEPTH 16, material-sorted shading
    ("multi_object", dict()),                             # config 4: diffuse + mirror + glass
    ("multi_object", dict(sortbyMaterial=True, SSAA=False)),
    ("random_triangles", dict()),                         # config 5: BVH over random triangles, DEPTH 32
    ("random_triangles", dict(useBVHtree=False)),
    ("random_triangles", dict(bvhCull=True)),
    ("random_primitives_1", dict()),                      # bounded closest hit: rotated, thin, overlapping
    ("random_primitives_2", dict(sortbyMaterial=True)),
])
def test_config_scenes_bitexact(config_scenes, name, kw):
    from cuda_pathtracer_amd import Scene
    path = config_scenes[name]
    g, r, st, live = _run(Scene(path), O.OracleScene.from_json(path), _gui(**kw), iters=2)
    _assert_bitexact(g, r, f"{name} {kw}")
    assert r.sum() > 0


@pytest.mark.parametrize("inline", [False, True])
@pytest.mark.parametrize("name,spp,kw", [
    ("room", 1, dict()),
    ("room", 3, dict()),                        # two lanes, each with its own k_traverse records
    ("room", 3, dict(bvhCull=True)),
    ("random_triangles", 2, dict()),
    ("random_triangles", 1, dict(SSAA=False, russianRoulette=False)),
])
def test_mesh_traversal_modes_bitexact(room_path, config_scenes, monkeypatch, inline, name, spp, kw):
    """Mesh scenes with the BVH on: the walk runs in k_traverse ahead of the bounce kernel, whose
    bounded closest hit takes the mesh hit as an evaluated candidate (default), or inside the bounce
    kernel (PT_AMD_MESH_INLINE=1).  Both equal the oracle bit for bit, one lane and two."""
    from cuda_pathtracer_amd import Scene
    if inline:
        monkeypatch.setenv("PT_AMD_MESH_INLINE", "1")
    if name == "room":
        s, o = _room_pair(room_path, (48, 36))
    else:
        s, o = Scene(config_scenes[name]), O.OracleScene.from_json(config_scenes[name])
    g, r, st, live = _run(s, o, _gui(**kw), iters=2, spp=spp)
    _assert_bitexact(g, r, f"{name} spp={spp} inline={inline} {kw}")
    assert r.sum() > 0


@pytest.mark.parametrize("nmat", [70, 200])
def test_sorted_many_materials_bitexact(tmp_path, nmat):
    """Material-sorted shading with more materials than a wave has lanes (the per-tile counts live
    in LDS rows of nmats entries): 70 and 200 materials over 120 objects, spp 1 and 3 (two lanes),
    bit-exact against the oracle's stable sort."""
    from cuda_pathtracer_amd import Scene, scenes
    path = scenes.random_primitives(tmp_path, n=120, res=(48, 36), seed=3, extra_materials=nmat)
    for spp in (1, 3):
        g, r, _, _ = _run(Scene(path), O.OracleScene.from_json(path), _gui(sortbyMaterial=True), iters=3, spp=spp)
        _assert_bitexact(g, r, f"{nmat} materials spp={spp}")
        assert r.sum() > 0


@pytest.mark.parametrize("nmat", [70, 200])
def test_fused_many_materials_bitexact(tmp_path, nmat):
    """The fused bounce kernel with the materials in its LDS table (70 + the scene's) and with more
    than the table holds (200: the analytic instantiation that reads them from global memory,
    k_bounce mode kAnalyticGM), spp 1 and 3, bit-exact against the oracle."""
    from cuda_pathtracer_amd import Scene, scenes
    path = scenes.random_primitives(tmp_path, n=120, res=(48, 36), seed=5, extra_materials=nmat)
    for spp in (1, 3):
        g, r, _, _ = _run(Scene(path), O.OracleScene.from_json(path), _gui(), iters=3, spp=spp)
        _assert_bitexact(g, r, f"fused, {nmat} materials, spp={spp}")
        assert r.sum() > 0


@pytest.mark.parametrize("rows", ["1", "3"])
def test_mesh_traversal_stack_spill_bitexact(room_path, config_scenes, monkeypatch, rows):
    """k_traverse keeps the first PT_AMD_STACK_ROWS stack entries per lane in LDS and the rest in
    scratch (HybStack): with 1 or 3 LDS rows nearly every push spills, and the images stay exact."""
    from cuda_pathtracer_amd import Scene
    monkeypatch.setenv("PT_AMD_STACK_ROWS", rows)
    s, o = _room_pair(room_path, (40, 30))
    g, r, _, _ = _run(s, o, _gui(), iters=2, spp=2)
    _assert_bitexact(g, r, f"room stack rows {rows}")
    path = config_scenes["random_triangles"]
    g, r, _, _ = _run(Scene(path), O.OracleScene.from_json(path), _gui(), iters=2, spp=2)
    _assert_bitexact(g, r, f"random triangles stack rows {rows}")


@pytest.mark.parametrize("spp,kw", [(4, dict()), (1, dict(sortbyMaterial=True)), (1, dict(useThrustPartition=True))])
def test_concurrent_contexts_on_two_streams(cornell_path, room_path, spp, kw):
    """Two render contexts in flight at once on separate streams (each bounce kernel sized to
    fill the GPU) with pt_flags.shared_gpu: both stay bit-exact and report no device error.  The
    split pipeline's look-back claims tiles in order; the sorted pipeline at spp=1 (one lane, which
    otherwise takes the single-pass library scan that needs its grid co-resident) scans its material
    histogram with the co-residency-free reduce/scan/apply kernels."""
    import os
    import torch
    from cuda_pathtracer_amd import PathTracer
    if kw.get("useThrustPartition"):
        os.environ["PT_PIPELINE"] = "split"
    try:
        s1, o1 = _pair(cornell_path, (96, 96))
        s2, o2 = _room_pair(room_path, (64, 64))
        p1 = PathTracer(s1, _gui(sharedGPU=True, **kw), spp=spp)
        p2 = PathTracer(s2, _gui(sharedGPU=True, **kw), spp=spp)
    finally:
        os.environ.pop("PT_PIPELINE", None)
    st1, st2 = torch.cuda.Stream(), torch.cuda.Stream()
    for k in range(3):
        p1.render_pass(1 + spp * k, st1)
        p2.render_pass(1 + spp * k, st2)
    torch.cuda.synchronize()
    g1, g2 = p1.image(), p2.image()
    assert p1.stats()["passes"] == 3 and p2.stats()["passes"] == 3   # pt_stats raises on a device error
    p1.free(); p2.free()
    r1 = r2 = None
    for k in range(3):
        r1, _ = O.render_pass(o1, _oflags(_gui(**kw)), 1 + spp * k, spp=spp, image=r1)
        r2, _ = O.render_pass(o2, _oflags(_gui(**kw)), 1 + spp * k, spp=spp, image=r2)
    _assert_bitexact(g1, r1, "cornell on stream 1")
    _assert_bitexact(g2, r2, "room on stream 2")


def test_camera_masks_verified_random_cameras(tmp_path, monkeypatch):
    """First-bounce geom masks under random cameras (inside and outside the scene, fov 20-110 deg,
    apertures up to 2, near and far focus, SSAA / DoF on and off) over stress scenes of rotated,
    thin and overlapping primitives: every camera ray's masked closest hit equals the plain loop
    over all geoms (PT_AMD_VERIFY_BOUNDS=1 in the material-sorted producer counts differences)."""
    from cuda_pathtracer_amd import PathTracer, Scene, scenes
    monkeypatch.setenv("PT_AMD_VERIFY_BOUNDS", "1")
    rng = np.random.default_rng(2024)
    rays = 0
    for k in range(8):
        s = Scene(scenes.random_primitives(tmp_path / f"s{k}", n=20, res=(48, 36), seed=100 + k))
        eye = rng.uniform((-4.5, 0.5, -4.5), (4.5, 9.5, 12.0))
        look = rng.uniform((-5, 0, -5), (5, 10, 5))
        s.set_camera((int(rng.integers(40, 90)), int(rng.integers(20, 60))), float(rng.uniform(20, 110)),
                     tuple(eye), tuple(look), (0, 1, 0))
        s.finalize()
        g = _gui(sortbyMaterial=True, SSAA=bool(k & 1), DoF=bool(k & 2) or k == 0,
                 aperture=float(rng.uniform(0.0, 2.0)), focal_len=float(rng.uniform(0.5, 15.0)))
        pt = PathTracer(s, g, spp=2)
        for it in (1, 3):
            pt.render_pass(it)
        st = pt.stats()
        pt.free()
        assert st["bound_mismatch"] == 0, (k, st["bound_mismatch"])
        rays += st["bounce_live"][0]
    assert rays > 20_000


def test_bounded_closest_hit_equals_plain_loop(config_scenes, monkeypatch):
    """The bounded closest-hit pass (pt_kernels.hip intersect_bounded) selects the same geom, t
    and normal bits as the plain per-geom loop for every ray of several passes of stress scenes
    (PT_AMD_VERIFY_BOUNDS=1 re-runs the plain loop on the device and counts differences)."""
    from cuda_pathtracer_amd import PathTracer, Scene
    monkeypatch.setenv("PT_AMD_VERIFY_BOUNDS", "1")
    monkeypatch.setenv("PT_PIPELINE", "split")
    total = 0
    for name in ("multi_object", "random_primitives_1", "random_primitives_2"):
        for sort in (False, True):
            pt = PathTracer(Scene(config_scenes[name]), _gui(sortbyMaterial=sort), spp=4)
            for k in range(3):
                pt.render_pass(1 + 4 * k)
            st = pt.stats()
            pt.free()
            assert st["bound_mismatch"] == 0, (name, sort, st["bound_mismatch"])
            total += st["segments"]
    assert total > 100_000


@pytest.mark.parametrize("walk", ["quad", "pairs"])
def test_bvh_walk_records_equal_reference_walk(room_path, config_scenes, tmp_path, monkeypatch, walk):
    """Every k_traverse4 (4-wide layout + leaf tasks; PT_AMD_TRAV=pairs: round 2's pair walk)
    record — closest triangle, t, barycentrics — equals the reference's node-at-a-time
    BVHIntersectionTest re-run on the device for the same ray (PT_AMD_VERIFY_BOUNDS=1 in the mesh
    bounce kernel counts differences): room (textured chairs), the 3000-triangle scene and config 5's
    100k-triangle tree, every bounce of several batched passes."""
    from cuda_pathtracer_amd import PathTracer, Scene, scenes
    monkeypatch.setenv("PT_AMD_VERIFY_BOUNDS", "1")
    if walk == "pairs":
        monkeypatch.setenv("PT_AMD_TRAV", "pairs")
    big = scenes.random_triangles(tmp_path, n=100_000, res=(320, 180), depth=32)
    total = 0
    for path, spp in ((room_path, 4), (config_scenes["random_triangles"], 4), (big, 2)):
        s = Scene(path)
        if path == room_path:
            s.set_camera((96, 72), 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
            s.finalize()
        pt = PathTracer(s, _gui(), spp=spp)
        for k in range(2):
            pt.render_pass(1 + spp * k)
        st = pt.stats()
        pt.free()
        assert st["bound_mismatch"] == 0, (path, st["bound_mismatch"])
        total += st["segments"]
    assert total > 200_000


@pytest.mark.parametrize("mode", ["auto", "forced"])
def test_exact_tcull_records_equal_reference_walk(room_path, config_scenes, tmp_path, monkeypatch, mode):
    """The 4-wide walk's exact t-cull changes no record: with PT_AMD_VERIFY_BOUNDS=1
    the mesh bounce kernel re-runs the reference's node-at-a-time BVHIntersectionTest for every ray
    and counts 0 differences in the closest triangle, t and barycentrics.  "auto": the cull is on
    where the margins pay (the tessellated scene's 100k small triangles, room.json) and off on
    config 5; "forced" (PT_AMD_TCULL=1): on everywhere, config 5's 100k large triangles included."""
    from cuda_pathtracer_amd import PathTracer, Scene, scenes
    monkeypatch.setenv("PT_AMD_VERIFY_BOUNDS", "1")
    if mode == "forced":
        monkeypatch.setenv("PT_AMD_TCULL", "1")
    tess = scenes.tessellated_meshes(tmp_path / "t", res=(200, 112), depth=16)
    big = scenes.random_triangles(tmp_path / "b", n=100_000, res=(320, 180), depth=32)
    total = 0
    for path, spp, expect in ((tess, 4, True), (room_path, 4, True), (config_scenes["random_triangles"], 4, None),
                              (big, 2, mode == "forced")):
        s = Scene(path)
        if path == room_path:
            s.set_camera((96, 72), 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
            s.finalize()
        pt = PathTracer(s, _gui(), spp=spp)
        info = pt.walk_info()
        assert info["quad_walk"]
        if expect is not None:
            assert info["tcull"] == expect, (path, info)
        for k in range(2):
            pt.render_pass(1 + spp * k)
        st = pt.stats()
        pt.free()
        assert st["bound_mismatch"] == 0, (path, st["bound_mismatch"])
        total += st["segments"]
    assert total > 400_000


@pytest.mark.parametrize("tasks", [None, "2"])
def test_tessellated_meshes_bitexact_with_tcull(tmp_path, monkeypatch, tasks):
    """The exact t-cull's own workload (100k small triangles on a sphere and a torus): the GPU image
    equals the oracle's (which walks the whole reference tree, no cull) bit for bit, batched and not;
    with the t-cull the walk deals one triangle task per lane, and two when forced (PT_AMD_WALK_TASKS)."""
    from cuda_pathtracer_amd import PathTracer, Scene, scenes
    if tasks is not None:
        monkeypatch.setenv("PT_AMD_WALK_TASKS", tasks)
    path = scenes.tessellated_meshes(tmp_path, res=(160, 90), depth=16)
    s = Scene(path)
    assert PathTracer(s, _gui()).walk_info()["tcull"]
    for spp in (1, 2):
        g, r, st, live = _run(Scene(path), O.OracleScene.from_json(path), _gui(), iters=2, spp=spp)
        _assert_bitexact(g, r, f"tessellated meshes spp={spp}")
        assert st["bounce_live"] == live and r.sum() > 0


def test_refraction_keys_render_like_bundled_scene(cornell_path, tmp_path):
    """A reference scene file carrying REFRACTIVE / IOR (keys scene.cpp:46-56 never reads) renders
    bit-identically to the bundled cornell.json when the loader extension is off (the default),
    and differently — with glass — when it is on (PT_LOAD_REFRACTION), against the oracle."""
    import json
    from cuda_pathtracer_amd import PathTracer, Scene
    scene = json.loads(open(cornell_path).read())
    scene["Materials"]["specular_white"]["REFRACTIVE"] = 1.0
    scene["Materials"]["specular_white"]["IOR"] = 1.5
    path = tmp_path / "cornell_refr.json"
    path.write_text(json.dumps(scene))
    def render(s):
        s.set_camera((64, 64), 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
        s.finalize()
        pt = PathTracer(s, _gui(), spp=2)
        pt.render_pass(1)
        img = pt.image()
        pt.free()
        return img
    base = render(Scene(cornell_path))
    assert np.array_equal(render(Scene(path)), base)
    glass = render(Scene(path, refraction=True))
    assert not np.array_equal(glass, base)
    o = O.OracleScene.from_json(path, refraction=True)
    o.set_camera((64, 64), 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    ref = O.render_pass(o, O.flags(), 1, spp=2)[0]
    _assert_bitexact(glass, ref, "cornell + REFRACTIVE/IOR, extension on")


def test_resume_from_checkpoint_is_bitexact(cornell_path, tmp_path):
    """Extension: checkpoint the float accumulator after 2 passes, resume in
    a fresh context at the next iteration index: identical to rendering the 4 passes in one go."""
    from cuda_pathtracer_amd import PathTracer
    s, o = _pair(cornell_path, (36, 30))
    ref = PathTracer(s, _gui(), spp=2)
    for it in (1, 3, 5, 7):
        ref.render_pass(it)
    full = ref.image()
    ref.free()
    a = PathTracer(s, _gui(), spp=2)
    for it in (1, 3):
        a.render_pass(it)
    ck = a.save_state(str(tmp_path / "ck.npz"), iterations_done=4)
    a.free()
    b = PathTracer(s, _gui(), spp=2)
    done = b.load_state(ck)
    assert done == 4
    for it in (done + 1, done + 3):
        b.render_pass(it)
    _assert_bitexact(b.image(), full, "resumed vs uninterrupted")
    b.free()


def test_full_size_cornell_batched_equals_sequential(cornell_path):
    """BASELINE configs[1] at full size (800x800, DEPTH 8): a 16-iteration pass equals 16
    one-iteration passes bit for bit, and the live-path counts agree (per-iteration keys and the
    segment layout against the reference's one-iteration pathtrace() calls; the bench's own pass of
    256 iterations is checked against two of 128 in test_benched_pass_size_equals_two_half_passes)."""
    from cuda_pathtracer_amd import PathTracer, Scene
    s = Scene(cornell_path)
    pb = PathTracer(s, _gui(), spp=16)
    pb.render_pass(1)
    gb, stb = pb.image(), pb.stats()
    pb.free()
    ps = PathTracer(s, _gui(), spp=1)
    for it in range(1, 17):
        ps.render_pass(it)
    gs, sts = ps.image(), ps.stats()
    ps.free()
    _assert_bitexact(gb, gs, "800x800: 16 batched vs 16 sequential")
    assert stb["bounce_live"] == sts["bounce_live"] and stb["bounce_live"][0] == 16 * 800 * 800
    assert all(b <= a for a, b in zip(stb["bounce_live"], stb["bounce_live"][1:]))


@pytest.mark.parametrize("spp", [0, 257])
def test_bad_batch_size_is_rejected(cornell_path, spp):
    from cuda_pathtracer_amd import PathTracer, PtError, Scene
    with pytest.raises(PtError):
        PathTracer(Scene(cornell_path), _gui(), spp=spp)


@pytest.mark.parametrize("kw", [dict(), dict(sortbyMaterial=True)])
def test_every_path_misses(cornell_path, kw):
    """Camera looking away from the scene: every camera ray misses at bounce 0, later bounces run
    with no live path (empty segment tables, idle workgroups) — zero image, no device error."""
    from cuda_pathtracer_amd import PathTracer, Scene
    s = Scene(cornell_path)
    s.set_camera((40, 30), 45.0, (0, 5, 10.5), (0, 5, 30.0), (0, 1, 0))
    s.finalize()
    o = O.OracleScene.from_json(cornell_path)
    o.set_camera((40, 30), 45.0, (0, 5, 10.5), (0, 5, 30.0), (0, 1, 0))
    g, r, st, live = _run(s, o, _gui(**kw), iters=6, spp=3)
    _assert_bitexact(g, r, f"all miss {kw}")
    assert st["bounce_live"][0] == 6 * 40 * 30 and st["bounce_live"][1] == 0 and not g.any()


@pytest.mark.parametrize("kw", [dict(), dict(sortbyMaterial=True)])
def test_max_batch_256_iterations(cornell_path, kw):
    """pt_shard.spp at its limit (256 = one thread of the bounce kernel's workgroup per iteration,
    the bench's 8-GPU pass): GPU == oracle bit for bit."""
    s, o = _pair(cornell_path, (12, 10))
    g, r, st, live = _run(s, o, _gui(**kw), iters=256, spp=256)
    _assert_bitexact(g, r, f"spp=256 {kw}")
    assert st["bounce_live"] == live


def test_deferred_finalize_is_ordered_with_image_calls(cornell_path):
    """Batched passes add their colours into the image on a side stream (pt_render_pass): the
    asynchronous image entry points on the caller's stream must see every finished pass, a reset
    must drop what came before it, and three passes in a row (both colour halves reused) must equal
    the same passes rendered with a read after each."""
    import torch
    from cuda_pathtracer_amd import PathTracer
    s, _ = _pair(cornell_path, (40, 32))
    st = torch.cuda.current_stream()
    a = PathTracer(s, _gui(), spp=3)
    for it in (1, 4, 7):
        a.render_pass(it, st)
    dev = torch.empty((a.rows, a.width, 3), dtype=torch.float32, device="cuda")
    a.copy_image_to(dev.data_ptr(), st)     # async on the caller's stream, no host sync before it
    torch.cuda.synchronize()
    b = PathTracer(s, _gui(), spp=3)
    for it in (1, 4, 7):
        b.render_pass(it, st)
        b.image()                           # synchronous read after every pass
    _assert_bitexact(dev.cpu().numpy(), b.image(), "async copy vs synchronous reads")
    # reset, then one more pass: only that pass's colours remain
    a.reset_image(st)
    a.render_pass(10, st)
    c = PathTracer(s, _gui(), spp=3)
    c.render_pass(10, st)
    _assert_bitexact(a.image(), c.image(), "reset then pass vs a fresh context")
    for p in (a, b, c):
        p.free()


@pytest.mark.parametrize("spp,lanes", [(2, "2"), (5, "2"), (32, "2"), (5, "3"), (7, "4"), (32, "4"), (3, "4")])
@pytest.mark.parametrize("sort", [False, True])
def test_two_lanes_equal_one_lane(cornell_path, monkeypatch, spp, lanes, sort):
    """Batched passes trace lanes of iterations on their own streams (pt_render_pass, 2-4 lanes,
    fused and material-sorted pipelines): image, live-path and emissive counts equal a one-lane
    context (PT_AMD_LANES=1) bit for bit, including uneven splits (5 = 3 + 2, 7 = 2 + 2 + 2 + 1) and
    more lanes than iterations (3 iterations, 4 lanes requested)."""
    from cuda_pathtracer_amd import PathTracer
    s, _ = _pair(cornell_path, (44, 30))
    out = []
    for n in (lanes, "1"):
        monkeypatch.setenv("PT_AMD_LANES", n)
        pt = PathTracer(s, _gui(sortbyMaterial=sort), spp=spp)
        for it in (1, 1 + spp):
            pt.render_pass(it)
        st = pt.stats()
        out.append((pt.image(), st["bounce_live"], st["bounce_emit"], st["passes"]))
        pt.free()
    _assert_bitexact(out[0][0], out[1][0], f"{lanes} lanes vs one, spp {spp} sort {sort}")
    assert out[0][1:] == out[1][1:]


@pytest.mark.parametrize("cam,kw,shard", [
    (((53, 37), 45.0, (0, 5, 10.5), (0, 5, 0)), dict(), (0, 1)),                         # 53 px rows: blocks span rows
    (((70, 30), 80.0, (3.5, 8.0, 4.0), (-2, 1, -3)), dict(aperture=1.5, focal_len=4.0, sortbyMaterial=True), (0, 1)),   # wide lens, near focus, sorted
    (((64, 48), 30.0, (0.5, 2.0, 3.0), (-1, 4, -1)), dict(SSAA=False, DoF=False), (1, 3)),   # inside the box, shard 1 of 3
    (((40, 40), 100.0, (-4.5, 9.5, 4.5), (4, 0, -4)), dict(DoF=False), (2, 4)),          # grazing views of the walls
    # half the view past the box's open side: waves whose mask is empty skip raygen and the closest
    # hit (PT_SKIP_MISS_WAVES), beside mixed waves; fused and material-sorted
    (((192, 64), 45.0, (0, 5, 10.5), (14, 5, 0)), dict(), (0, 1)),
    (((192, 64), 45.0, (0, 5, 10.5), (14, 5, 0)), dict(sortbyMaterial=True), (0, 1)),
])
def test_first_bounce_camera_masks(cornell_path, monkeypatch, cam, kw, shard):
    """First-bounce geom masks (pt_kernels.hip build_cmask): each wave of camera rays bounds only
    the geoms its 64 pixels' rays can reach.  Odd widths, shards, wide apertures, cameras inside the
    scene and grazing views: GPU == oracle bit for bit, and == the same context without masks
    (PT_AMD_NO_CMASK=1).  Then flags changed through pt_set_flags (masks rebuilt) still match."""
    from cuda_pathtracer_amd import PathTracer, Scene
    res, fovy, eye, look = cam
    rank, world = shard
    s = Scene(cornell_path)
    s.set_camera(res, fovy, eye, look, (0, 1, 0))
    s.finalize()
    o = O.OracleScene.from_json(cornell_path)
    o.set_camera(res, fovy, eye, look, (0, 1, 0))
    g, r, _, _ = _run(s, o, _gui(**kw), iters=4, rank=rank, world=world, spp=2)
    _assert_bitexact(g, r, f"masks {cam} {kw}")
    monkeypatch.setenv("PT_AMD_NO_CMASK", "1")
    g2, _, _, _ = _run(s, o, _gui(**kw), iters=4, rank=rank, world=world, spp=2)
    monkeypatch.delenv("PT_AMD_NO_CMASK")
    _assert_bitexact(g, g2, "masks on vs off")
    kw2 = dict(kw, aperture=0.8, focal_len=9.0, SSAA=not kw.get("SSAA", True), DoF=True)
    pt = PathTracer(s, _gui(**kw), rank=rank, world=world, spp=2)
    pt.set_flags(_gui(**kw2))
    img = None
    for it in (1, 3):
        pt.render_pass(it)
        img, _ = O.render_pass(o, _oflags(_gui(**kw2)), it, spp=2, rank=rank, world=world, image=img)
    gi = pt.image()
    pt.free()
    _assert_bitexact(gi, img, f"masks after set_flags {kw2}")


@pytest.mark.parametrize("look,want_skip", [((14, 5, 0), True), ((0, 5, 0), None)])
def test_fused_empty_wave_skip(cornell_path, monkeypatch, look, want_skip):
    """The fused first bounce's empty-wave instantiation (k_bounce mode kAnalyticSkip: waves whose
    camera mask is empty skip raygen and the closest hit) is chosen from the share of empty mask
    blocks (pt_ctx_cmask_info); forced on, forced off and chosen, the image equals the oracle's."""
    from cuda_pathtracer_amd import PathTracer, Scene
    res = (192, 64)
    s = Scene(cornell_path)
    s.set_camera(res, 45.0, (0, 5, 10.5), look, (0, 1, 0))
    s.finalize()
    o = O.OracleScene.from_json(cornell_path)
    o.set_camera(res, 45.0, (0, 5, 10.5), look, (0, 1, 0))
    pt = PathTracer(s, _gui(), spp=2)
    info = pt.cmask_info()
    pt.free()
    assert info["on"]
    assert info["skip_fused"] == (info["empty_frac"] >= 0.2)
    if want_skip is not None:
        assert info["skip_fused"] == want_skip and info["empty_frac"] > 0.3
    ref = None
    for force in ("1", "0", None):
        if force is None:
            monkeypatch.delenv("PT_AMD_SKIP_EMPTY", raising=False)
        else:
            monkeypatch.setenv("PT_AMD_SKIP_EMPTY", force)
        g, r, _, _ = _run(s, o, _gui(), iters=4, spp=2)
        _assert_bitexact(g, r, f"skip forced {force} look {look}")
        if ref is not None:
            _assert_bitexact(g, ref, "skip on vs off")
        ref = g


def test_set_flags_unchanged_is_cheap(cornell_path):
    """The reference re-reads its GUI flags on every pathtrace() call (pathtrace.cu:438-463), so a
    drop-in caller calls pt_set_flags once per iteration.  Unchanged flags — and flags that do not
    shape the camera rays (Russian roulette here) — must not synchronise the device or rebuild the
    first-bounce camera masks; a change of SSAA / DoF / aperture / focal distance must.  The image of
    the per-iteration pathtrace() sequence stays bit-exact against the oracle throughout."""
    from cuda_pathtracer_amd import PathTracer
    s, o = _pair(cornell_path, (64, 48))
    gui = _gui()
    pt = PathTracer(s, gui)
    assert pt.counters() == {"mask_builds": 1, "flag_syncs": 0}
    ref = None
    for it in range(1, 6):
        pt.set_flags(_gui())                       # what pathtrace() does every iteration
        pt.render_pass(it)
        ref, _ = O.render_pass(o, _oflags(_gui()), it, image=ref)
    assert pt.counters() == {"mask_builds": 1, "flag_syncs": 0}
    _assert_bitexact(pt.image(), ref, "unchanged flags")
    pt.set_flags(_gui(russianRoulette=False))      # not a camera-ray flag: no sync, no rebuild
    pt.render_pass(6)
    ref, _ = O.render_pass(o, _oflags(_gui(russianRoulette=False)), 6, image=ref)
    assert pt.counters() == {"mask_builds": 1, "flag_syncs": 0}
    for it, kw in ((7, dict(aperture=0.4)), (8, dict(aperture=0.4)), (9, dict(aperture=0.4, SSAA=False))):
        pt.set_flags(_gui(**kw))
        pt.render_pass(it)
        ref, _ = O.render_pass(o, _oflags(_gui(**kw)), it, image=ref)
    assert pt.counters() == {"mask_builds": 3, "flag_syncs": 2}
    _assert_bitexact(pt.image(), ref, "flags changed between iterations")
    pt.free()


@pytest.mark.parametrize("scene", ["cornell", "cornell_sorted", "room"])
def test_render_ahead_claimed_and_dropped_bitexact(cornell_path, room_path, scene):
    """pt_render_ahead (the drop-in loop's overlap of iteration i + 1's bounces with iteration i's
    image copy): every pathtrace()-shaped step — set_flags, render_pass(it), render_ahead(it + 1),
    image read — equals the oracle bit for bit, whether the iteration traced ahead is claimed (same
    iteration, same flags), dropped for changed flags, dropped for another iteration, or claimed
    after the image was reset or replaced; the counts include claimed iterations only."""
    from cuda_pathtracer_amd import PathTracer
    if scene == "room":
        s, o = _room_pair(room_path, (40, 32))
    else:
        s, o = _pair(cornell_path, (48, 40))
    base = dict(sortbyMaterial=True) if scene == "cornell_sorted" else dict()
    # (iteration, flag overrides, image action before the pass)
    plan = [(1, {}, None), (2, {}, None), (3, {}, None), (4, dict(russianRoulette=False), None),
            (5, dict(russianRoulette=False), None), (7, dict(russianRoulette=False), None),
            (8, dict(russianRoulette=False), "reset"), (9, dict(russianRoulette=False), "set"),
            (10, dict(russianRoulette=False, SSAA=False), None), (11, dict(russianRoulette=False, SSAA=False), None)]
    stats = []
    for ahead in (False, True):
        pt = PathTracer(s, _gui(**base))
        ref, live_ref = None, [0] * o.depth
        for it, kw, action in plan:
            g = _gui(**base, **kw)
            pt.set_flags(g)
            if action == "reset":
                pt.reset_image()
                ref = np.zeros_like(ref)
            elif action == "set":
                ref = (ref * np.float32(0.5)).astype(np.float32)
                pt.set_image(ref)
            pt.render_pass(it)
            ref, live = O.render_pass(o, _oflags(g), it, image=ref)
            live_ref = [a + b for a, b in zip(live_ref, live)]
            if ahead:
                pt.render_ahead(it + 1)
            _assert_bitexact(pt.image(), ref, f"{scene} ahead={ahead} iteration {it} {kw} {action}")
        st = pt.stats()
        assert st["device_error"] == 0
        assert st["bounce_live"] == live_ref
        stats.append(st)
        pt.free()
    assert stats[0] == stats[1]   # segments, passes, per-bounce live and emissive counts


def test_render_ahead_across_streams(cornell_path):
    """Render-ahead and passes of one context on two streams, arranged so that any missing
    cross-stream ordering overlaps or reorders shared work on the device (not by host timing):

    * race A — an ahead pass on stream B while passes still run on stream A (they share the path
      buffers, control and segment words): six 800x800 passes are queued on A, and B is released by
      an event recorded after the FIRST of them, so an unordered ahead pass would start exactly when
      pass 2 starts;
    * race B — the next ahead pass on B while the claim's settle on A still reads ahead_col: A sleeps
      (a 20+ ms device spin) before the claim, so an unordered ahead would rewrite ahead_col first;
    * alternating plain passes — pass i on A behind a device spin, pass i + 1 on B.

    The image must equal the oracle's sequential render bit for bit, and the per-bounce counts the
    oracle's; pt_render_ahead waits for the context's last work on another stream (ev_done) and a
    pass on a new stream waits for all of it."""
    import torch
    from cuda_pathtracer_amd import PathTracer
    s, o = _pair(cornell_path, (800, 800))
    pt = PathTracer(s, _gui())
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    spin = int(5e7)   # torch's bounded device spin (clock cycles): tens of milliseconds
    ref, live_ref = None, [0] * o.depth

    def oracle(it):
        nonlocal ref, live_ref
        ref, live = O.render_pass(o, _oflags(_gui()), it, image=ref)
        live_ref = [a + b for a, b in zip(live_ref, live)]

    # race A
    first_done = torch.cuda.Event()
    for it in range(1, 7):
        pt.render_pass(it, sa)
        if it == 1:
            first_done.record(sa)
    sb.wait_event(first_done)
    pt.render_ahead(7, sb)
    pt.render_pass(7, sa)   # claims 7
    # race B
    pt.render_ahead(8, sb)
    with torch.cuda.stream(sa):
        torch.cuda._sleep(spin)
    pt.render_pass(8, sa)   # claims 8: its settle reads ahead_col after the spin
    pt.render_ahead(9, sb)  # must not rewrite ahead_col before that settle
    pt.render_pass(9, sa)   # claims 9
    # alternating plain passes
    for it in range(10, 14):
        st = sa if it % 2 == 0 else sb
        with torch.cuda.stream(st):
            torch.cuda._sleep(spin // 4)
        pt.render_pass(it, st)
    torch.cuda.synchronize()
    for it in range(1, 14):
        oracle(it)
    _assert_bitexact(pt.image(), ref, "render-ahead and passes across streams")
    st = pt.stats()
    assert st["device_error"] == 0
    assert st["bounce_live"] == live_ref
    pt.free()


def test_render_ahead_needs_one_iteration_context(cornell_path):
    from cuda_pathtracer_amd import PathTracer
    s, _ = _pair(cornell_path, (16, 16))
    pt = PathTracer(s, _gui(), spp=2)
    with pytest.raises(Exception, match="one iteration"):
        pt.render_ahead(3)
    pt.free()


@pytest.mark.parametrize("sort", [False, True])
def test_async_lanes_stream_ordered_reads(cornell_path, sort):
    """Async lanes: a batched pass does not make the caller's stream wait for every lane, so the
    next pass starts during the tail.  Six passes issued back to back on one torch stream, then the
    image copied on that stream (pt_copy_image waits for the last finalize) and only that stream
    synchronised — no device-wide sync — equal the oracle bit for bit, for 2 and 3 lanes."""
    import os
    import torch
    from cuda_pathtracer_amd import PathTracer
    s, o = _pair(cornell_path, (48, 40))
    for lanes in ("2", "3"):
        os.environ["PT_AMD_LANES"] = lanes
        try:
            pt = PathTracer(s, _gui(sortbyMaterial=sort), spp=6)
        finally:
            os.environ.pop("PT_AMD_LANES", None)
        st = torch.cuda.Stream()
        dst = torch.empty((40, 48, 3), dtype=torch.float32, device="cuda")
        with torch.cuda.stream(st):
            for k in range(6):
                pt.render_pass(1 + 6 * k, st)
            pt.copy_image_to(dst.data_ptr(), st)
        st.synchronize()
        got = dst.cpu().numpy()
        ref = None
        for k in range(6):
            ref, _ = O.render_pass(o, _oflags(_gui(sortbyMaterial=sort)), 1 + 6 * k, spp=6, image=ref)
        pt.free()
        _assert_bitexact(got, ref, f"async lanes {lanes} sort {sort}")


@pytest.mark.parametrize("spp", [1, 2])
def test_config3_full_size_sorted_bitexact(cornell_path, tmp_path, spp):
    """BASELINE.json config 3 at its full size — cornell geometry at 1920x1080, DEPTH 16,
    material-sorted shading — GPU == oracle bit for bit over `spp` iterations in one pass.  spp=1
    takes the one-lane path with the single-pass library scan of the material histogram; spp=2 the
    two-lane path, whose histogram (5 materials x 32400 tiles per lane) spans ~40 tiles of the
    reduce/scan/apply kernels, exercising the cross-tile carry."""
    from cuda_pathtracer_amd import Scene, scenes
    path = scenes.cornell_hd(tmp_path, res=(1920, 1080), depth=16)
    g, r, st, live = _run(Scene(path), O.OracleScene.from_json(path), _gui(sortbyMaterial=True), iters=spp, spp=spp)
    _assert_bitexact(g, r, f"config 3 full size spp={spp}")
    assert st["bounce_live"] == live and live[0] == spp * 1920 * 1080


def test_config4_full_size_bitexact(tmp_path, monkeypatch):
    """BASELINE.json config 4 at its full width — 3840x2160, the 12-object room (diffuse, mirror,
    glass) — one iteration, GPU == oracle bit for bit with the first-bounce camera masks on (one
    per 64 pixels of the 4K tile); then the split pipeline under PT_AMD_VERIFY_BOUNDS=1 re-runs the
    plain closest-hit loop for every ray of the same iteration and counts 0 differences."""
    from cuda_pathtracer_amd import PathTracer, Scene, scenes
    path = scenes.multi_object(tmp_path, res=(3840, 2160), depth=8)
    g, r, st, live = _run(Scene(path), O.OracleScene.from_json(path), _gui(), iters=1)
    _assert_bitexact(g, r, "config 4 full size")
    assert st["bounce_live"] == live and live[0] == 3840 * 2160 and r.sum() > 0
    monkeypatch.setenv("PT_AMD_VERIFY_BOUNDS", "1")
    monkeypatch.setenv("PT_PIPELINE", "split")
    # (claimed tile schedule: the diagnostic split pipeline's look-back at this size outruns the
    # static schedule's co-resident grid)
    pt = PathTracer(Scene(path), _gui(sharedGPU=True))
    pt.render_pass(1)
    vs = pt.stats()
    gv = pt.image()
    pt.free()
    assert vs["bound_mismatch"] == 0 and vs["segments"] == sum(live)
    _assert_bitexact(gv, r, "config 4 full size, split pipeline")


def test_sorted_multitile_histogram_scan(cornell_path):
    """Two-lane sorted passes with a histogram of nmats x (P/2)/64 = 5 x 1875 > 4096 entries per lane
    (several tiles of k_hist_sums / k_hist_scan_sums / k_hist_apply, multi-element threads in the
    one-workgroup scan of the tile sums): bit-exact over two passes."""
    s, o = _pair(cornell_path, (200, 150))
    g, r, st, live = _run(s, o, _gui(sortbyMaterial=True), iters=16, spp=8)
    _assert_bitexact(g, r, "sorted 200x150 spp=8")
    assert st["bounce_live"] == live


@pytest.mark.parametrize("kw,tasks", [(dict(), None), (dict(), "1"), (dict(), "2"), (dict(sortbyMaterial=True), None)])
def test_config5_100k_triangles_bitexact(tmp_path, monkeypatch, kw, tasks):
    """BASELINE.json config 5's geometry at full size — 100k random triangles through OBJ + SAH BVH
    (depth-22 tree, child-pair layout, LDS stack), DEPTH 32 — at a reduced resolution: GPU == oracle
    bit for bit (the benchmarked tree itself, not the 3000-triangle parity scene); the 4-wide walk
    with one and with two triangle tasks per lane (PT_AMD_WALK_TASKS)."""
    from cuda_pathtracer_amd import Scene, scenes
    if tasks is not None:
        monkeypatch.setenv("PT_AMD_WALK_TASKS", tasks)
    path = scenes.random_triangles(tmp_path, n=100_000, res=(160, 90), depth=32)
    g, r, st, live = _run(Scene(path), O.OracleScene.from_json(path), _gui(**kw), iters=2, spp=2)
    _assert_bitexact(g, r, f"config 5 100k triangles {kw}")
    assert st["bounce_live"] == live and r.sum() > 0


def test_config5_full_size_bitexact(tmp_path):
    """BASELINE.json config 5 at its benched size: 100k random triangles (OBJ + SAH BVH), 3840x2160,
    DEPTH 32, one iteration — GPU == oracle bit for bit, with the same live-path count entering every
    bounce (pathtrace.cu:423-528).  8.3 M camera rays, ~25 M traced segments: the largest index
    ranges of the 4-wide walk's tickets and records at one iteration.  The oracle's per-path loops
    run on the host's cores (oracle_set_threads; its result does not depend on the thread count)."""
    import os
    from cuda_pathtracer_amd import Scene, scenes
    path = scenes.random_triangles(tmp_path, n=100_000, res=(3840, 2160), depth=32)
    O.set_threads(min(16, os.cpu_count() or 1))
    try:
        g, r, st, live = _run(Scene(path), O.OracleScene.from_json(path), _gui(), iters=1)
    finally:
        O.set_threads(1)
    _assert_bitexact(g, r, "config 5 full size")
    assert st["bounce_live"] == live and live[0] == 3840 * 2160 and r.sum() > 0


@pytest.mark.parametrize("config,spp,res,sort", [
    ("multi_object_4k", 128, (3840, 2160), False),
    ("random_triangles_100k", 128, (3840, 2160), False),
    ("cornell_hd_sorted", 256, (1920, 1080), True),
    ("cornell", 256, (800, 800), False),
])
def test_benched_pass_size_equals_two_half_passes(tmp_path, cornell_path, config, spp, res, sort):
    """Every BASELINE workload at the pass size bench.py runs it — configs 4 and 5: one pass of 128
    iterations at 3840x2160 (1.06 G paths; ~120 GB of path state, walk records and colours for config
    5); config 3: one pass of 256 iterations at 1920x1080, DEPTH 16, material-sorted, over the default
    three lanes (530.8 M paths: the sorted pipeline's largest record, histogram, work-list and byte
    offsets); the headline Cornell 800x800: one pass of 256 (163.8 M paths) — against two passes of
    half the size.  A size-independent property (batched passes equal sequential ones, DESIGN.md §3;
    pathtrace.cu:423-528): the same image bit for bit, the same live-path and emission counts per
    bounce, no device error."""
    from cuda_pathtracer_amd import PathTracer, Scene, scenes
    path = cornell_path if scenes.CONFIGS[config] is None else scenes.CONFIGS[config](tmp_path)
    scene = Scene(path)
    out = []
    for n, passes in ((spp, 1), (spp // 2, 2)):
        pt = PathTracer(scene, _gui(sortbyMaterial=sort), spp=n)
        it = 1
        for _ in range(passes):
            pt.render_pass(it)
            it += n
        st = pt.stats()
        assert st["device_error"] == 0 and st["bounce_live"][0] == spp * res[0] * res[1]
        out.append((pt.image(), st["bounce_live"], st["bounce_emit"]))
        pt.free()
    _assert_bitexact(out[0][0], out[1][0], f"{config}: one pass of {spp} vs two of {spp // 2}")
    assert out[0][1:] == out[1][1:]
    assert np.isfinite(out[0][0]).all() and out[0][0].sum() > 0


@pytest.mark.parametrize("spp", [1, 3])
@pytest.mark.parametrize("look", ["away", "light"])
def test_sorted_paths_that_all_end_early(cornell_path, spp, look):
    """Material-sorted shading when the producer retires (almost) every path itself: a camera
    facing away from the box (every camera ray misses: the next producer gets no work positions)
    and one looking straight up at the light (most camera rays meet the emitter).  Live-path and
    emission counts and the image equal the oracle's (shade_ends, pathtrace.cu:318-330)."""
    from cuda_pathtracer_amd import Scene
    eye, at, up = ((0, 5, 10.5), (0, 5, 30), (0, 1, 0)) if look == "away" else ((0, 6, 2.5), (0, 10, 0), (0, 1, 0))
    s = Scene(cornell_path)
    s.set_camera((48, 32), 45.0, eye, at, up)
    s.finalize()
    o = O.OracleScene.from_json(cornell_path)
    o.set_camera((48, 32), 45.0, eye, at, up)
    g, r, st, live = _run(s, o, _gui(sortbyMaterial=True), iters=3, spp=spp)
    _assert_bitexact(g, r, f"sorted, camera {look}, spp {spp}")
    assert list(st["bounce_live"][:len(live)]) == live
    if look == "away":
        assert live[0] == 3 * 48 * 32 and sum(live[1:]) == 0 and r.sum() == 0
    else:
        assert r.sum() > 0 and live[1] < live[0]


def test_context_synchronisation_is_scoped(cornell_path):
    """pt_get_image / pt_stats wait for their own context only (an event after its last pass) and
    copy on a high-priority stream of the context's own, so with long batched passes of another
    context queued, a small context's image and statistics are read while those passes still run
    (an event queued after them is still pending), and both stay bit-exact.  Runs inside the pytest
    process, whose earlier tests left torch streams behind: HIP gives each priority level of a
    process its own GPU_MAX_HW_QUEUES hardware queues, and the copy stream's level holds only copy
    streams, so no compute stream — the library's, torch's or the caller's — can sit in front of it
    (include/pt_amd.h, stream budget).  The stream accounting of both contexts is checked too."""
    import time
    import torch
    from cuda_pathtracer_amd import GuiDataContainer, PathTracer, Scene
    s = Scene(cornell_path)
    s.set_camera((32, 24), 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    s.finalize()
    o = O.OracleScene.from_json(cornell_path)
    o.set_camera((32, 24), 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    small = PathTracer(s, GuiDataContainer())
    small.render_pass(1)
    ref, _ = O.render_pass(o, O.flags(), 1)
    _assert_bitexact(small.image(), ref, "small context before")
    big = PathTracer(Scene(cornell_path), GuiDataContainer(), spp=64)
    si_small, si_big = small.stream_info(), big.stream_info()
    # the big context: caller + lanes + finalize; both contexts' busy streams within the budget
    assert si_small["busy_streams"] == 1 and si_small["lanes"] == 1, si_small
    assert si_big["busy_streams"] == 1 + (si_big["lanes"] - 1) + 1, si_big
    assert si_big["process_busy"] >= si_small["busy_streams"] + si_big["busy_streams"], (si_small, si_big)
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
    big.free()
    small.free()
    _assert_bitexact(img, ref, "small context read during the other context's passes")
    assert st["bounce_live"][0] == 32 * 24 and st["device_error"] == 0, st
    assert bst["bounce_live"][0] == 9 * 64 * 800 * 800 and bst["device_error"] == 0, bst
    assert running, (f"the small context's reads waited for the other context "
                     f"({t_small * 1e3:.2f} of {t_big * 1e3:.2f} ms; streams {si_small} {si_big})")


def test_lanes_capped_by_stream_budget(cornell_path, monkeypatch):
    """pt_create caps the lanes it picks by itself so that the busy streams of the live contexts stay
    within GPU_MAX_HW_QUEUES: with a budget of 4, a 2-lane batched context holds 3 (caller, lane,
    finalize), so a second one gets 1 lane (2 more streams, not 3); freeing both gives a third
    context its 2 lanes back.  The capped context still renders bit-exact."""
    import gc
    from cuda_pathtracer_amd import PathTracer
    gc.collect()   # (contexts of earlier tests not yet freed)
    monkeypatch.delenv("PT_AMD_LANES", raising=False)
    s, o = _pair(cornell_path, (40, 32))
    probe = PathTracer(s, _gui())
    base = probe.stream_info()["process_busy"] - 1   # busy streams of other live contexts, if any
    probe.free()
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", str(4 + base))
    a = PathTracer(s, _gui(), spp=4)
    ia = a.stream_info()
    assert ia["lanes"] == 2 and ia["busy_streams"] == 3 and not ia["lanes_capped"], ia
    b = PathTracer(s, _gui(), spp=4)
    ib = b.stream_info()
    assert ib["lanes"] == 1 and ib["lanes_capped"] and ib["process_busy"] == base + ia["busy_streams"] + 2, ib
    b.render_pass(1)
    ref, _ = O.render_pass(o, _oflags(_gui()), 1, spp=4)
    _assert_bitexact(b.image(), ref, "lane-capped context")
    a.free()
    b.free()
    c = PathTracer(s, _gui(), spp=4)
    ic = c.stream_info()
    assert ic["lanes"] == 2 and not ic["lanes_capped"] and ic["process_busy"] == base + 3, ic
    c.free()


@pytest.mark.parametrize("spp", [1, 4])
def test_signed_zero_accumulator_then_pass_bitexact(cornell_path, spp):
    """Passes skip the additions of zero colours (retire stores only nonzero colours, k_finalize_spp adds
    only flagged slots; the one-iteration path adds only nonzero colours into the image).  Those
    additions are identities on every value but -0, so an accumulator loaded with -0, NaN and ordinary
    values (pt_set_accum, the resume extension) then traced must equal the oracle, which adds every
    iteration's colour into every pixel — bit for bit, the signs of zeros included."""
    from cuda_pathtracer_amd import PathTracer
    s, o = _pair(cornell_path, (40, 32))
    rng = np.random.default_rng(7)
    img = rng.random((32, 40, 3), dtype=np.float32)
    img[::3] = np.float32(-0.0)
    img[1::7, :, 1] = np.float32(0.0)
    img[2, 5, :] = np.float32(np.nan)
    pt = PathTracer(s, _gui(), spp=spp)
    pt.set_image(img)
    pt.render_pass(1)
    got = pt.image()
    pt.free()
    ref, _ = O.render_pass(o, _oflags(_gui()), 1, spp=spp, image=img.copy())
    g, r = got.view(np.uint32), ref.view(np.uint32)
    same = (g == r) | (np.isnan(got) & np.isnan(ref))
    assert same.all(), f"spp={spp}: {int((~same).sum())} values differ in bits (signed zeros included)"
    assert np.signbit(got[np.asarray(got == 0)]).sum() == 0   # no -0 left after a pass
