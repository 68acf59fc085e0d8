# HBM traffic per launch from PMC counters (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and
# WRITE_SIZE in SEPARATE rocprofv3 passes (TCC slots), --kernel-trace only, each under its own
# time limit; the chain stops at the first failure.  Workloads: 10 render passes of cornell
# 800x800 (scripts/prof_render.py) and the 2^28 scan (scripts/scan_ablate.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/traffic"
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$R/gpurun_out/traffic/render_$ctr" -o run -- \
      python3 "$R/scripts/prof_render.py" 10 > "$R/gpurun_out/traffic/render_$ctr.log" 2>&1 \
      || { echo "render $ctr failed"; tail -5 "$R/gpurun_out/traffic/render_$ctr.log"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$R/gpurun_out/traffic/scan_$ctr" -o run -- \
      python3 "$R/scripts/scan_ablate.py" > "$R/gpurun_out/traffic/scan_$ctr.log" 2>&1 \
      || { echo "scan $ctr failed"; tail -5 "$R/gpurun_out/traffic/scan_$ctr.log"; exit 1; }
  echo "$ctr ok"
done
python3 "$R/scripts/traffic_summary.py" "$R/gpurun_out/traffic" > "$R/gpurun_out/traffic/summary.json"
cat "$R/gpurun_out/traffic/summary.json"
