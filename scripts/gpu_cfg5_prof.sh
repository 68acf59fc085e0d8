# rocprofv3 kernel-trace stats of the config-5 bench (k_traverse + k_bounce split).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/cfg5prof"
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$R/bench.py" --config random_triangles_100k --spp ${SPP:-8} --samples ${SPP:-8} --steps 3 --warmup 1 --no-scan --no-cpu-baseline --no-pmc > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "prof failed"; tail -5 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(round(d['value'],1), round(d['ms_per_step'],3))"
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]:
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:9.1f} pct={r['Percentage']}")
PY
