"""Reproduce the bench line's headline roofline fraction from rocprofv3 output.

  python scripts/union_check.py KTRACE_KERNEL_TRACE.csv BENCH.json PMC_SUMMARY.json [lanes]

* effective launch time of the dominant kernel = the union of its launch intervals in the
  --kernel-trace CSV / its launches (the two lanes' launches overlap; launches x this fits the step);
* VALU wave-instructions per launch from the in-run --pmc summary (scripts/pmc.py, SQ_INSTS_VALU);
* frac = VALU per launch / effective time / (256 CUs x 4 SIMDs x 2.4 GHz / 2) — compared with the
  bench line's roofline.frac, plus the byte figures (hbm.*) recomputed over the trace's time.
"""
import csv
import json
import sys

VALU_PEAK = 256 * 4 * 2.4e9 / 2
HBM = 8000.0


def union_ns(iv):
    iv.sort()
    tot, end = 0, -1
    for a, b in iv:
        if a > end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot


def main():
    trace, bench, pmc = sys.argv[1:4]
    line = json.loads([l for l in open(bench) if l.startswith("{")][-1])
    r = line["roofline"]
    prefix = r["kernel"] if r["kernel"].startswith("k_") else "k_bounce<false"
    if prefix.startswith("k_traverse4<false"):
        prefix = "k_traverse4<false"
    rows = [x for x in csv.DictReader(open(trace)) if prefix in x["Kernel_Name"].replace("(anonymous namespace)::", "")]
    iv = [(int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in rows]
    n = len(iv)
    avg_ms = sum(b - a for a, b in iv) / max(n, 1) / 1e6
    eff_ms = union_ns(iv) / max(n, 1) / 1e6
    summ = json.load(open(pmc))
    km = next((m for k, m in summ.get("kernels", {}).items() if k.startswith(prefix.split("<")[0]) and
               k.startswith(prefix)), None)
    print(f"rocprofv3 --kernel-trace: {n} launches of {prefix}; average duration {avg_ms:.4f} ms; "
          f"union of their intervals / launches = {eff_ms:.4f} ms")
    print(f"bench line (HIP events): avg_launch_ms {r['avg_launch_ms']:.4f}, effective_launch_ms "
          f"{r['effective_launch_ms']:.4f}, launches_per_step {r['launches_per_step']:.1f}, kernel_ms_per_step "
          f"{r['kernel_ms_per_step']:.3f}, ms_per_step {line['ms_per_step']:.3f}")
    print(f"line: bound {r['bound']}, frac {r['frac']:.4f} ({r['unit']})")
    if km and "SQ_INSTS_VALU" in km:
        valu = km["SQ_INSTS_VALU"]
        f = valu / (eff_ms * 1e-3) / VALU_PEAK
        print(f"VALU issue from the trace: SQ_INSTS_VALU {valu:.4g} per launch / {eff_ms:.4f} ms / {VALU_PEAK:.4g} "
              f"= {f:.4f}  (line {r.get('valu_issue', {}).get('frac', float('nan')):.4f})")
    for k in ("model_184B", "kernel_min", "counter_traffic"):
        h = r.get("hbm", {}).get(k)
        if h:
            f = h["bytes_per_launch"] / (eff_ms * 1e-3) / 1e9 / HBM
            print(f"hbm.{k}: {h['bytes_per_launch']:.4g} B per launch / {eff_ms:.4f} ms / 8 TB/s = {f:.4f}  "
                  f"(line {h['frac']:.4f})")
    print(f"fractions above 1 in the line: {r.get('fractions_above_1')}; model ratios above 1: "
          f"{list(r.get('model_ratios_above_1', {}))}")


if __name__ == "__main__":
    main()
