# Bench + rocprofv3 kernel-trace summary on the GPU box.  Each GPU step has its own time limit
# and the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
timeout -k 10 600 python "$R/bench.py" ${BENCH_ARGS:-} > "$R/gpurun_out/bench.json" 2> "$R/gpurun_out/bench.err" || { echo "bench failed rc=$?"; tail -20 "$R/gpurun_out/bench.err"; exit 1; }
cat "$R/gpurun_out/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- \
    python3 "$R/bench.py" --steps 50 --no-cpu-baseline --scan-reps 5 > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err" \
    || { echo "rocprof failed rc=$?"; tail -20 "$R/gpurun_out/prof_bench.err"; exit 1; }
find "$R/gpurun_out/prof" -name "*stats*" | head
python3 "$R/scripts/trace_busy.py" "$(find "$R/gpurun_out/prof" -name "*kernel_trace.csv" | head -1)" | tee "$R/gpurun_out/prof/busy.txt"
