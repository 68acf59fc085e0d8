"""The C++ host mirror on the GPU: the reference-shaped stream-compaction self-test
(tests/cpp/test_stream_compaction.cpp, after stream_compaction/src/main.cpp) and the headless CLI
(cuda_pathtracer_amd/host/main.cpp, after path_tracer/src/main.cpp runCuda + saveImage), whose PNG
must equal the oracle's tone-mapped render byte for byte."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

from oracle import binding as O

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.parametrize("size_log2", [12, 20, 24, 28])   # 28: SIZE = 1 << 28 (stream_compaction/src/main.cpp:8)
def test_reference_shaped_stream_compaction_selftest(size_log2):
    exe = ROOT / "tests" / "cpp" / "build" / "test_stream_compaction"
    res = subprocess.run([str(exe), str(size_log2)], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-2000:]
    assert "ALL PASSED" in res.stdout and "FAIL" not in res.stdout.replace("FAILED", "")


def test_cli_png_matches_oracle(tmp_path, cornell_path):
    exe = ROOT / "cuda_pathtracer_amd" / "pathtracer_amd"
    res = subprocess.run([str(exe), cornell_path, "--iterations", "2", "--out", str(tmp_path), "--hdr"],
                         capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stdout + res.stderr
    pngs = list(tmp_path.glob("cornell.*.2samp.png"))
    assert len(pngs) == 1, (res.stdout, list(tmp_path.iterdir()))
    from PIL import Image
    got = np.asarray(Image.open(pngs[0]).convert("RGB"))
    sc = O.OracleScene.from_json(cornell_path)
    img = None
    for it in (1, 2):
        img, _ = O.render_pass(sc, O.flags(), it, image=img)
    np.testing.assert_array_equal(got, O.tonemap(img, 2.0))
    # --hdr: Image::saveHDR of the same accumulator (RGBE: <= 2^-7 of each pixel's largest component)
    from oracle import hdr_oracle
    hdrs = list(tmp_path.glob("cornell.*.2samp.hdr"))
    assert len(hdrs) == 1
    dec = hdr_oracle.decode_hdr(hdrs[0].read_bytes())
    ref = (img / np.float32(2.0))[:, ::-1]
    assert (np.abs(dec - ref) <= ref.max(axis=2, keepdims=True) * 2 ** -7 + 1e-30).all()


def test_cli_room_textures_png_matches_oracle(tmp_path):
    """The C++ host renders the textured mesh scene (room.json: three OBJ chairs + a wall mesh, two
    JPEG textures decoded natively by pt_decode_jpeg) and its PNG equals the oracle's render, the
    oracle shading from its own JPEG restatement's texels (oracle/jpeg_oracle.py).  Resolution
    reduced to 160x160 so the CPU oracle stays fast; everything else as the bundled file."""
    import json
    scenes = ROOT / "tests" / "scenes"
    spec = json.loads((scenes / "room.json").read_text())
    spec["Camera"]["RES"] = [160, 160]
    (tmp_path / "Textures").symlink_to(scenes / "Textures")
    (tmp_path / "Models").symlink_to(scenes / "Models")
    path = tmp_path / "room.json"
    path.write_text(json.dumps(spec))
    exe = ROOT / "cuda_pathtracer_amd" / "pathtracer_amd"
    out = tmp_path / "out"
    out.mkdir()
    res = subprocess.run([str(exe), str(path), "--iterations", "2", "--out", str(out)], capture_output=True,
                         text=True, timeout=300)
    assert res.returncode == 0, res.stdout + res.stderr
    pngs = list(out.glob("*.2samp.png"))
    assert len(pngs) == 1, (res.stdout, list(out.iterdir()))
    from PIL import Image
    got = np.asarray(Image.open(pngs[0]).convert("RGB"))
    sc = O.OracleScene.from_json(str(path))
    img = None
    for it in (1, 2):
        img, _ = O.render_pass(sc, O.flags(), it, image=img)
    np.testing.assert_array_equal(got, O.tonemap(img, 2.0))


def test_cli_usage_and_bad_scene(tmp_path):
    exe = ROOT / "cuda_pathtracer_amd" / "pathtracer_amd"
    assert subprocess.run([str(exe)], capture_output=True, timeout=60).returncode == 1
    res = subprocess.run([str(exe), str(tmp_path / "nope.json")], capture_output=True, text=True, timeout=60)
    assert res.returncode != 0 and "error" in res.stderr
