"""The kernel-parameter layout `fresh_param` (pt_kernels.hip) relies on, read from the built library's
own code object metadata (no GPU).

The tile loops of k_bounce, k_trace and k_sort_produce re-read their by-value parameters from the
kernarg segment at fixed byte offsets: KArgs at 0 and, for k_sort_produce, SortArgs right after it at
sizeof(KArgs) rounded up to SortArgs' 8-byte alignment.  A reordered or added parameter would make
those loads read the wrong bytes, so the offsets the compiler actually assigned (the .args of every
instantiation in libpt_amd.so's gfx950 code object) are checked here.
"""
from __future__ import annotations

import shutil
import struct
import subprocess

import pytest
import yaml

from cuda_pathtracer_amd import build as B

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def _code_objects(tmp_path):
    """The gfx950 ELF code objects inside the library's .hip_fatbin section."""
    fat = tmp_path / "fat.bin"
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", str(B.LIB), str(tmp_path / "lib.copy")],
                   check=True, capture_output=True)
    blob = fat.read_bytes()
    out, i = [], 0
    while (j := blob.find(b"\x7fELF", i)) >= 0:
        i = j + 4
        if blob[j + 4] != 2:   # ELF64 only
            continue
        shoff = struct.unpack_from("<Q", blob, j + 0x28)[0]
        shentsize, shnum = struct.unpack_from("<HH", blob, j + 0x3A)
        p = tmp_path / f"co_{j}.o"
        p.write_bytes(blob[j:j + shoff + shentsize * shnum])
        out.append(p)
    return out


def _kernels(path):
    text = subprocess.run([READELF, "--notes", str(path)], check=True, capture_output=True, text=True).stdout
    if "amdhsa.kernels:" not in text:
        return []
    body = text[text.index("---") + 3:]
    body = body[:body.index("\n...")] if "\n..." in body else body
    return yaml.safe_load(body).get("amdhsa.kernels", [])


@pytest.mark.skipif(shutil.which("objcopy") is None or not B.LIB.exists(), reason="needs objcopy and the built library")
def test_fresh_param_offsets_match_the_compiled_layout(tmp_path):
    kernels = [k for co in _code_objects(tmp_path) for k in _kernels(co)]
    names = {"k_bounce": 0, "k_trace": 0, "k_sort_produce": 0}
    for k in kernels:
        short = next((n for n in names if f"{len(n)}{n}I" in k[".name"]), None)
        if short is None:
            continue
        names[short] += 1
        args = [a for a in k[".args"] if a[".value_kind"] == "by_value"]
        assert args[0][".offset"] == 0, k[".name"]   # KArgs: fresh_args() reads offset 0
        if short == "k_sort_produce":
            assert len(args) == 2
            kargs = args[0][".size"]
            assert args[1][".offset"] == (kargs + 7) // 8 * 8, k[".name"]   # SortArgs after KArgs
        else:
            assert len(args) == 1, k[".name"]
    assert all(v > 0 for v in names.values()), names
