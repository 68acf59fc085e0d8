# Config 3 bench line (with its in-run PMC passes) and the per-launch durations of the sorted
# pipeline's kernels by bounce (first lane, first pass of the PMC run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --config cornell_hd_sorted --steps 5 --warmup 1 --no-cpu-baseline --no-scan \
    > gpurun_out/cfg3.json 2> gpurun_out/cfg3.err || { echo "bench failed"; tail -20 gpurun_out/cfg3.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/cfg3.json') if l.startswith('{')][-1]); r=d['roofline']
print('cfg3', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'B/seg', round(r.get('traffic_per_segment') or 0,1))"
python3 scripts/kernel_totals.py gpurun_out/bench_pmc/fetch/run_kernel_trace.csv | head -8
python3 - <<'PY'
import csv
rows = sorted(csv.DictReader(open('gpurun_out/bench_pmc/fetch/run_kernel_trace.csv')), key=lambda r: int(r['Start_Timestamp']))
seq = [(r['Kernel_Name'], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3) for r in rows]
for name in ('k_hist_apply', 'k_sort_produce<false', 'k_hist_sums'):
    print(name, [round(d) for k, d in seq if name in k][:17])
PY
