"""Register and code-size report of every shipped kernel instantiation (no GPU needed).

Compiles the device sources to gfx950 assembly with the product's own flags (build.py COMMON +
EXTRA), then reads, per kernel, the code object metadata the loader uses (.vgpr_count,
.sgpr_count, .vgpr_spill_count, .sgpr_spill_count, .private_segment_fixed_size = scratch bytes
per lane, .group_segment_fixed_size = static LDS) and the ISA line count of its body, and the
occupancy those registers allow (waves per SIMD: 512 VGPRs / granule-rounded count, at most 8).

    python scripts/kernel_resources.py [--out profiles/r06_kernel_resources.txt] [--filter k_bounce]
"""
from __future__ import annotations

import argparse
import re
import subprocess
import sys
import tempfile
from pathlib import Path

import yaml

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from cuda_pathtracer_amd import build as B  # noqa: E402

CXXFILT = "c++filt"


def assemble(src: str, tmp: Path) -> str:
    out = tmp / (src + ".s")
    cmd = [B.HIPCC, "-x", "hip", f"--offload-arch={B.ARCH}", "--cuda-device-only", "-S", *B.COMMON,
           *B.EXTRA.get(src, []), "-I", str(ROOT / "include"), str(B.CSRC / src), "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return out.read_text()


def demangle(names: list[str]) -> dict[str, str]:
    res = subprocess.run([CXXFILT], input="\n".join(names), capture_output=True, text=True, check=True)
    return dict(zip(names, res.stdout.splitlines()))


def parse(asm: str) -> list[dict]:
    m = re.search(r"^\s*\.amdgpu_metadata\s*$(.*?)^\s*\.end_amdgpu_metadata", asm, re.S | re.M)
    meta = yaml.safe_load(m.group(1)) if m else {}
    lines = asm.splitlines()
    body: dict[str, int] = {}
    cur = None
    for ln in lines:
        s = ln.strip()
        if cur is None:
            lab = re.match(r"^([A-Za-z_.$][\w.$]*):\s*(;.*)?$", ln)
            if lab and not lab.group(1).startswith("."):
                cur, body[cur] = lab.group(1), 0
            continue
        if s.startswith(".Lfunc_end"):
            cur = None
        elif s and not s.startswith((";", ".")) and not s.endswith(":"):
            body[cur] += 1
    rows = []
    for k in meta.get("amdhsa.kernels", []):
        sym = k[".symbol"][:-3] if k[".symbol"].endswith(".kd") else k[".symbol"]
        v = int(k[".vgpr_count"]) + int(k.get(".agpr_count", 0))
        waves = min(8, 512 // max(8, (v + 7) // 8 * 8))
        rows.append({"symbol": sym, "vgpr": int(k[".vgpr_count"]), "agpr": int(k.get(".agpr_count", 0)),
                     "sgpr": int(k[".sgpr_count"]), "vgpr_spill": int(k.get(".vgpr_spill_count", 0)),
                     "sgpr_spill": int(k.get(".sgpr_spill_count", 0)),
                     "scratch": int(k.get(".private_segment_fixed_size", 0)),
                     "lds": int(k.get(".group_segment_fixed_size", 0)),
                     "isa_lines": body.get(sym, 0), "waves_by_vgpr": waves})
    return rows


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--out", default=None)
    ap.add_argument("--filter", default=None, help="substring of the demangled name")
    ap.add_argument("--src", nargs="*", default=["pt_kernels.hip", "sc_kernels.hip", "bvh_build.hip"])
    a = ap.parse_args()
    rows = []
    with tempfile.TemporaryDirectory() as td:
        for src in a.src:
            for r in parse(assemble(src, Path(td))):
                r["src"] = src
                rows.append(r)
    names = demangle([r["symbol"] for r in rows])
    hdr = f"{'kernel':<64} {'vgpr':>4} {'sgpr':>4} {'v_spill':>7} {'s_spill':>7} {'scratch':>7} {'lds':>6} " \
          f"{'isa':>6} {'w/simd':>6}"
    out = [f"# {B.ARCH}, flags: {' '.join(B.COMMON)} (+ {B.EXTRA}); scripts/kernel_resources.py",
           "# vgpr/sgpr: .vgpr_count/.sgpr_count; v_spill/s_spill: .vgpr_spill_count/.sgpr_spill_count "
           "(SGPRs spill to VGPR lanes, not memory); scratch: bytes per lane; lds: static bytes; "
           "isa: instruction lines; w/simd: waves per SIMD the VGPRs allow", hdr]
    for r in sorted(rows, key=lambda r: (r["src"], names[r["symbol"]])):
        n = names[r["symbol"]].replace("(anonymous namespace)::", "")
        n = re.sub(r"\((?:\(anonymous namespace\)::)?KArgs\)$", "", n)
        if a.filter and a.filter not in n:
            continue
        n = n if len(n) <= 64 else n[:61] + "..."
        out.append(f"{n:<64} {r['vgpr']:>4} {r['sgpr']:>4} {r['vgpr_spill']:>7} {r['sgpr_spill']:>7} "
                   f"{r['scratch']:>7} {r['lds']:>6} {r['isa_lines']:>6} {r['waves_by_vgpr']:>6}")
    text = "\n".join(out) + "\n"
    if a.out:
        Path(a.out).write_text(text)
    sys.stdout.write(text)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
