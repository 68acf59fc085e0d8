"""Per-kernel HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE csv output.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports exactly half of the bytes
of a wide (16 B/lane) coalesced read on gfx950, so it is doubled; WRITE_SIZE is exact for 16-B
streaming stores.  Both counters are in KiB.  Infinity-Cache hits are counted as fabric
requests, so these are upper bounds on HBM bytes for MALL-resident data (cornell's path state
is MALL-resident at 800x800).
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

KEYS = {"k_bounce<false": "k_bounce", "k_bounce<true": "k_bounce_first", "k_scan_lag<0": "scan",
        "k_scan_tiles<0": "scan_tiles", "k_scan_mall<0": "scan_mall", "k_trace": "k_trace", "k_compact_paths": "k_compact_paths"}


def load(dirpath: Path, counter: str):
    per = defaultdict(list)
    for f in dirpath.rglob("*counter_collection*.csv"):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return per


def main(root: str) -> None:
    root = Path(root)
    out = {"_note": "bytes per launch; FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE; KiB->B",
           "_kernels": {}}
    for wl in ("render", "scan"):
        fetch = load(root / f"{wl}_FETCH_SIZE", "FETCH_SIZE")
        write = load(root / f"{wl}_WRITE_SIZE", "WRITE_SIZE")
        for name in sorted(set(fetch) | set(write)):
            f = fetch.get(name, [])
            w = write.get(name, [])
            if not f and not w:
                continue
            rd = 2.0 * 1024.0 * (sum(f) / len(f)) if f else 0.0
            wr = 1024.0 * (sum(w) / len(w)) if w else 0.0
            short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            out["_kernels"][short] = {"launches": max(len(f), len(w)), "read_bytes": rd, "write_bytes": wr,
                                      "bytes_per_launch": rd + wr}
            for k, key in KEYS.items():
                if short.startswith(k):
                    out[key] = rd + wr
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
