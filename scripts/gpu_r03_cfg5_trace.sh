# Config 5 under rocprofv3 kernel trace (one lane by default now): where the GPU time goes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out/c5trace; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5trace -o run -- \
    python3 bench.py --config random_triangles_100k --steps 1 --warmup 1 --spp 32 --samples 32 --no-cpu-baseline --no-scan --no-pmc --no-walk-counters \
    > gpurun_out/c5trace/bench.json 2> gpurun_out/c5trace/bench.err || { echo "trace failed"; tail -5 gpurun_out/c5trace/bench.err; exit 1; }
python3 scripts/kernel_totals.py gpurun_out/c5trace/run_kernel_trace.csv | head -12
grep '^{' gpurun_out/c5trace/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', round(d['value'],1), 'ms/step', round(d['ms_per_step'],2))"
