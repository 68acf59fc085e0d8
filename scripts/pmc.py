"""In-run PMC measurement for bench.py (and the profiling scripts): HBM traffic and VALU issue
counts per launch of the render kernels, from rocprofv3 --pmc passes over the bench's own workload
(scripts/prof_render.py with the same scene, batch and flags).

Rules (MI355X_MICROARCH.md "HBM" and "rocprofv3 PMC slots"): one counter group per rocprofv3 run,
--kernel-trace only (no other trace domains with --pmc), each run under its own KILL time limit;
FETCH_SIZE (3 TCC slots) and WRITE_SIZE (2) in separate passes.  Units and corrections: both in KiB;
FETCH_SIZE reports half the bytes of a wide coalesced read on gfx950, so it is doubled; WRITE_SIZE is
exact for 16-B/lane streaming stores.  Infinity-Cache hits are counted as fabric requests, so for
MALL-resident data these are upper bounds on HBM bytes.  SQ_* wave counters are summed over waves;
SQ_WAVE_CYCLES / SQ_ACTIVE_* / SQ_WAIT_* count quad-cycles (x4 = shader cycles); GRBM_GUI_ACTIVE is
summed over the 8 XCDs (effective clock = GRBM_GUI_ACTIVE / 8 / kernel time).
"""
from __future__ import annotations

import csv
import os
import shutil
import subprocess
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
GROUPS = {
    "fetch": ["FETCH_SIZE"],
    "write": ["WRITE_SIZE"],
    "sq": ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY",
           "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"],
    "l2": ["TCC_HIT_sum", "TCC_MISS_sum"],                       # L2 hit rate (per-XCD L2s summed)
    "vmem": ["SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH"],
    # where waves wait: issue-blocked cycles by unit, instruction-fetch stalls, in-flight levels
    "stall1": ["SQ_WAVE_CYCLES", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM",
               "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_IFETCH", "SQ_IFETCH_LEVEL"],
    "stall2": ["SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM", "SQ_INST_LEVEL_LDS", "SQ_INSTS_LDS",
               "SQ_INST_LEVEL_SMEM", "SQ_INSTS_SMEM", "SQ_WAIT_ANY", "SQ_LDS_BANK_CONFLICT"],
    # vector L1: accesses, requests to L2 and their summed latency (average L2 round trip per request)
    "tcp": ["TCP_TOTAL_ACCESSES_sum", "TCP_TCC_READ_REQ_sum", "TCP_TCC_READ_REQ_LATENCY_sum", "TCP_TCP_LATENCY_sum"],
    "ta": ["TA_TA_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum"],
}


def short_name(k: str) -> str:
    return k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].strip()


def _load(d: Path):
    """{kernel: {counter: [value per dispatch]}} and {kernel: [duration ns per dispatch]}."""
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in d.rglob("*counter_collection*.csv"):
        for row in csv.DictReader(open(f)):
            vals[short_name(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for f in d.rglob("*kernel_trace*.csv"):
        for row in csv.DictReader(open(f)):
            dur[short_name(row["Kernel_Name"])].append(float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
    return vals, dur


def collect(workload: list[str], out_dir: Path, timeout: int = 120, groups=("fetch", "write", "sq")) -> dict:
    """Run one rocprofv3 --pmc pass per counter group over `workload` (argv of prof_render.py);
    return per-kernel means per launch: read/write bytes (corrected) and the SQ counters."""
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    out_dir = Path(out_dir)
    shutil.rmtree(out_dir, ignore_errors=True)
    out_dir.mkdir(parents=True, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    res: dict = {"_passes": {}}
    per: dict = defaultdict(dict)
    for g in groups:
        d = out_dir / g
        cmd = ["timeout", "-s", "KILL", str(timeout), prof, "--kernel-trace", "--pmc", *GROUPS[g],
               "--output-format", "csv", "-d", str(d), "-o", "run", "--",
               sys.executable, str(ROOT / "scripts" / "prof_render.py"), *workload]
        with open(out_dir / f"{g}.log", "w") as log:
            rc = subprocess.run(cmd, stdout=log, stderr=subprocess.STDOUT, cwd="/tmp", env=env).returncode
        res["_passes"][g] = rc
        if rc != 0:
            break   # a failed or killed pass: stop (never retry a GPU step)
        for line in (out_dir / f"{g}.log").read_text().splitlines():   # prof_render.py: segments [live...]
            if line[:1].isdigit():
                res["segments"] = int(line.split()[0])
                if "[" in line:
                    import ast
                    res["bounce_live"] = ast.literal_eval(line[line.index("["):])
        vals, dur = _load(d)
        for k, cs in vals.items():
            for c, v in cs.items():
                per[k][c] = sum(v) / len(v)
            per[k]["launches"] = max(len(v) for v in cs.values())
            if dur.get(k):
                per[k].setdefault("dur_ns_" + g, sum(dur[k]) / len(dur[k]))
    for k, m in per.items():
        if "FETCH_SIZE" in m:
            m["read_bytes"] = 2.0 * 1024.0 * m["FETCH_SIZE"]
        if "WRITE_SIZE" in m:
            m["write_bytes"] = 1024.0 * m["WRITE_SIZE"]
        if "read_bytes" in m and "write_bytes" in m:
            m["bytes_per_launch"] = m["read_bytes"] + m["write_bytes"]
    res["kernels"] = dict(per)
    res["workload"] = workload
    return res


def pick(res: dict, prefix: str) -> dict | None:
    """The per-launch record of the first kernel whose short name starts with `prefix`."""
    for k, m in res.get("kernels", {}).items():
        if k.startswith(prefix):
            return m
    return None


if __name__ == "__main__":
    import json
    print(json.dumps(collect(sys.argv[2:], Path(sys.argv[1])), indent=1))
