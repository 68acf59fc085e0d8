# Per-launch kernel durations of 10 render passes (rocprofv3 --kernel-trace), summarised per bounce.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/ktrace${KT_TAG:+_$KT_TAG}"
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- \
    python3 "$R/scripts/prof_render.py" 10 ${KT_ARGS:-} > "$OUT/render.log" 2>&1 \
    || { echo "ktrace failed"; tail -5 "$OUT/render.log"; exit 1; }
python3 "$R/scripts/trace_summary.py" $(find "$OUT" -name "*kernel_trace.csv") | tee "$OUT/summary.txt"
