"""Busy time of the bounce kernels from a rocprofv3 kernel-trace CSV: the union of the launch
intervals of k_bounce<false,...> (bounces >= 1), which overlap pairwise since batched passes run
two lanes of iterations concurrently.  Per pass = union / passes, passes = k_bounce<true,...>
launches / lanes.  bench.py's roofline uses the same definition over its profiled passes
(roofline.busy_ms / profiled passes), measured with HIP events."""
import csv
import sys


def union_ms(iv):
    iv.sort()
    tot, end = 0, -1
    for a, b in iv:
        if a > end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot / 1e6


path = sys.argv[1]
lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows = list(csv.DictReader(open(path)))
later = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
         if "k_bounce<false" in r["Kernel_Name"]]
first = [r for r in rows if "k_bounce<true" in r["Kernel_Name"]]
passes = len(first) / lanes
dur = sum(b - a for a, b in later) / 1e6
u = union_ms(later)
print(f"k_bounce<false,...>: {len(later)} launches, summed {dur:.3f} ms, union {u:.3f} ms; "
      f"{passes:.0f} passes ({lanes} lanes): union per pass {u / max(passes, 1):.4f} ms, "
      f"average launch {dur / max(len(later), 1) * 1e3:.1f} us")
