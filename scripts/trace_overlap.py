"""GPU occupancy over time from a rocprofv3 kernel-trace CSV: the share of the traced span with no
kernel running, with one, and with two or more (lanes overlapping), and the gaps between
consecutive kernel intervals.  usage: trace_overlap.py run_kernel_trace.csv [skip_first_ms]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
skip = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 0.0
t0 = iv[0][0] + skip
iv = [x for x in iv if x[0] >= t0]
ev = []
for a, b, _ in iv:
    ev += [(a, 1), (b, -1)]
ev.sort()
lvl, last, acc = 0, ev[0][0], {}
for t, d in ev:
    acc[min(lvl, 2)] = acc.get(min(lvl, 2), 0) + (t - last)
    lvl += d
    last = t
span = ev[-1][0] - ev[0][0]
print(f"span {span / 1e6:.2f} ms, kernels {len(iv)}")
for k in (0, 1, 2):
    print(f"  {'idle' if k == 0 else ('1 kernel' if k == 1 else '2+ kernels')}: {acc.get(k, 0) / 1e6:8.2f} ms  {100 * acc.get(k, 0) / span:5.1f}%")
