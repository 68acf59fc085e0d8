"""In-tree build of the native library (libpt_amd.so, gfx950) and the CPU test oracle.

Everything is compiled with plain hipcc / g++ command lines (no cmake, no JIT cache) so the
shared objects sit next to the sources and travel to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "libpt_amd.so"
CLI = PKG / "pathtracer_amd"
DROPIN_LIB = PKG / "libpt_dropin.so"
HOST = PKG / "host"
HOST_LIB = PKG / "build" / "libpt_amd_host.a"
ORACLE_DIR = ROOT / "oracle"
ORACLE_LIB = ORACLE_DIR / "build" / "liboracle.so"

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# -ffp-contract=off: the evaluation contract — every multiply-add is two
# correctly-rounded operations unless the source writes fmaf(); keeps GPU == oracle bitwise.
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-function"]
DEVICE_SRCS = ["sc_kernels.hip", "sc_variants.hip", "pt_kernels.hip", "bvh_build.hip"]
# pt_kernels.hip: no SLP vectorisation.  Packing independent f32 ops into v_pk_* pairs needed
# register pairs and moves: k_bounce took 79 VGPRs (6 waves/SIMD) instead of 60 (8 waves), and
# measured 30.8k vs 32.7k Mray/s on the bench (same box, alternating runs; same bits).
EXTRA = {"pt_kernels.hip": ["-fno-slp-vectorize"]}
HOST_SRCS = ["pt_scene.cpp", "pt_mesh.cpp", "pt_image.cpp", "pt_jpeg.cpp"]


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout + res.stderr)
        raise RuntimeError(f"build step failed: {' '.join(cmd[:4])} ... ({res.returncode})")


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build_native(verbose: bool = False, force: bool = False) -> Path:
    objdir = PKG / "build"
    objdir.mkdir(exist_ok=True)
    headers = list(CSRC.glob("*.h")) + list((ROOT / "include").glob("*.h"))
    jobs = []
    objs = []
    for src in DEVICE_SRCS + HOST_SRCS:
        s = CSRC / src
        o = objdir / (src + ".o")
        objs.append(o)
        if force or _stale(o, [s] + headers):
            lang = ["-x", "hip", f"--offload-arch={ARCH}"] if src.endswith(".hip") else []
            jobs.append([HIPCC, *lang, *COMMON, *EXTRA.get(src, []), "-I", str(ROOT / "include"), "-c", str(s),
                         "-o", str(o)])
    with cf.ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    if force or jobs or _stale(LIB, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB), *map(str, objs), "-lz"], verbose)
    # C++ host mirror of the reference interface (host/) and the headless CLI over it
    host_srcs = [HOST / "pathtrace.cpp", HOST / "stream_compaction.cpp"]
    host_hdrs = list(HOST.glob("*.h")) + list(HOST.glob("stream_compaction/*.h"))
    host_objs = []
    for s in host_srcs:
        o = objdir / ("host_" + s.name + ".o")
        host_objs.append(o)
        if force or _stale(o, [s] + host_hdrs + headers):
            _run([HIPCC, f"--offload-arch={ARCH}", *COMMON, "-I", str(ROOT / "include"), "-I", str(HOST), "-c", str(s),
                  "-o", str(o)], verbose)
    if force or _stale(HOST_LIB, host_objs):
        if HOST_LIB.exists():
            HOST_LIB.unlink()
        _run(["ar", "rcs", str(HOST_LIB), *map(str, host_objs)], verbose)
    cli_src = HOST / "main.cpp"
    if force or _stale(CLI, [cli_src, LIB, HOST_LIB] + host_hdrs + headers):
        _run([HIPCC, f"--offload-arch={ARCH}", *COMMON, "-I", str(ROOT / "include"), "-I", str(HOST), str(cli_src),
              "-x", "none", str(HOST_LIB), "-o", str(CLI), "-L", str(PKG), "-lpt_amd", "-Wl,-rpath,$ORIGIN"], verbose)
    # bench harness: the drop-in call sequence over the C++ mirror (host/dropin_bench.cpp)
    dsrc = HOST / "dropin_bench.cpp"
    if force or _stale(DROPIN_LIB, [dsrc, LIB, HOST_LIB] + host_hdrs + headers):
        _run([HIPCC, f"--offload-arch={ARCH}", *COMMON, "-shared", "-I", str(ROOT / "include"), "-I", str(HOST),
              str(dsrc), "-x", "none", str(HOST_LIB), "-o", str(DROPIN_LIB), "-L", str(PKG), "-lpt_amd",
              "-Wl,-rpath,$ORIGIN"], verbose)
    return LIB


def build_oracle(verbose: bool = False, force: bool = False) -> Path:
    """The CPU checker (test infrastructure only): serial g++ build, no FMA contraction."""
    srcs = [ORACLE_DIR / "sc_oracle.cpp", ORACLE_DIR / "pt_oracle.cpp", ORACLE_DIR / "mesh_oracle.cpp"]
    ORACLE_LIB.parent.mkdir(exist_ok=True)
    if force or _stale(ORACLE_LIB, srcs):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math", "-pthread",
              "-o", str(ORACLE_LIB), *map(str, srcs)], verbose)
    return ORACLE_LIB


def build_cpp_tests(verbose: bool = False, force: bool = False) -> list[Path]:
    """C++ test programs (test infrastructure): the reference-shaped self-tests over the C++ host
    mirror, checked against the oracle.  Run by tests/test_cpp_gpu.py on the GPU box."""
    tdir = ROOT / "tests" / "cpp"
    outs = []
    for src in sorted(tdir.glob("test_*.cpp")):
        exe = tdir / "build" / src.stem
        exe.parent.mkdir(exist_ok=True)
        outs.append(exe)
        if force or _stale(exe, [src, LIB, HOST_LIB, ORACLE_LIB] + list(HOST.glob("*.h")) +
                           list(HOST.glob("stream_compaction/*.h"))):
            # only -I host: the test includes <stream_compaction/...> as the reference's main.cpp does
            _run([HIPCC, f"--offload-arch={ARCH}", *COMMON, "-I", str(HOST), str(src),
                  "-x", "none", str(HOST_LIB), "-o", str(exe), "-L", str(PKG), "-lpt_amd", "-L", str(ORACLE_LIB.parent),
                  "-loracle", "-Wl,-rpath,$ORIGIN/../../../cuda_pathtracer_amd:$ORIGIN/../../../oracle/build"], verbose)
    return outs


PIN_DIR = ROOT / "tests" / "pin"
PIN_LIB = PIN_DIR / "build" / "libthrust_pin.so"


def build_pin(verbose: bool = False, force: bool = False) -> Path:
    """Test infrastructure: rocThrust (system ROCm, not reference code) behind a small C ABI, to pin
    the oracle's restatement of the reference's Thrust calls (tests/pin/thrust_pin.hip)."""
    src = PIN_DIR / "thrust_pin.hip"
    PIN_LIB.parent.mkdir(exist_ok=True)
    if force or _stale(PIN_LIB, [src]):
        _run([HIPCC, "-x", "hip", f"--offload-arch={ARCH}", "-O2", "-std=c++17", "-fPIC", "-shared",
              "-ffp-contract=off", "-o", str(PIN_LIB), str(src)], verbose)
    return PIN_LIB


TESTHOOKS_LIB = PKG / "build" / "libpt_amd_testhooks.so"


def build_test_hooks(verbose: bool = False, force: bool = False) -> Path:
    """Test infrastructure: the library with sc_kernels.hip's test hooks compiled in
    (-DPT_SC_TEST_HOOKS: PT_AMD_TEST_SCAN_OVERSUB), loaded only by tests/test_scan_gpu.py's
    stall test through PT_AMD_LIB.  The shipping libpt_amd.so has no hook."""
    objdir = PKG / "build"
    src = CSRC / "sc_kernels.hip"
    obj = objdir / "sc_kernels_testhooks.o"
    headers = list(CSRC.glob("*.h")) + list((ROOT / "include").glob("*.h"))
    if force or _stale(obj, [src] + headers):
        _run([HIPCC, "-x", "hip", f"--offload-arch={ARCH}", *COMMON, "-DPT_SC_TEST_HOOKS", "-I", str(ROOT / "include"),
              "-c", str(src), "-o", str(obj)], verbose)
    others = [objdir / (s + ".o") for s in DEVICE_SRCS + HOST_SRCS if s != "sc_kernels.hip"]
    if force or _stale(TESTHOOKS_LIB, [obj] + others):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(TESTHOOKS_LIB), str(obj),
              *map(str, others), "-lz"], verbose)
    return TESTHOOKS_LIB


TRAV_LIB = PKG / "build" / "libpt_amd_trav.so"


def build_trav_stats(verbose: bool = False, force: bool = False) -> Path:
    """Diagnostic library (not the product): pt_kernels.hip with the BVH walk's lane counters
    (-DPT_TRAV_STATS), read by scripts/trav_stats.py for the bench's roofline.walk_counters.  Built
    here so it always matches the product library's ABI."""
    objdir = PKG / "build"
    src = CSRC / "pt_kernels.hip"
    obj = objdir / "pt_kernels_trav.o"
    headers = list(CSRC.glob("*.h")) + list((ROOT / "include").glob("*.h"))
    if force or _stale(obj, [src] + headers):
        _run([HIPCC, "-x", "hip", f"--offload-arch={ARCH}", *COMMON, *EXTRA["pt_kernels.hip"], "-DPT_TRAV_STATS",
              "-I", str(ROOT / "include"), "-c", str(src), "-o", str(obj)], verbose)
    others = [objdir / (s + ".o") for s in DEVICE_SRCS + HOST_SRCS if s != "pt_kernels.hip"]
    if force or _stale(TRAV_LIB, [obj] + others):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(TRAV_LIB), str(obj),
              *map(str, others), "-lz"], verbose)
    return TRAV_LIB


def build_all(verbose: bool = False, force: bool = False) -> None:
    build_native(verbose, force)
    build_test_hooks(verbose, force)
    build_trav_stats(verbose, force)
    build_oracle(verbose, force)
    build_cpp_tests(verbose, force)
    build_pin(verbose, force)


if __name__ == "__main__":
    build_all(verbose="-v" in sys.argv, force="-f" in sys.argv)
    print(LIB)
