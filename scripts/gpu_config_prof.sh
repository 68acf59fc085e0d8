# rocprofv3 kernel-trace stats of one BASELINE config bench run (CFG, SPP env).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/cfgprof_${CFG}"
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$R/bench.py" --config "$CFG" --spp ${SPP:-1} --steps ${STEPS:-10} --warmup 2 --no-scan --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "prof failed"; tail -5 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('$CFG', round(d['value'],1), round(d['ms_per_step'],3))"
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:8.1f} pct={r['Percentage']}")
PY
