# Cornell bench under rocprofv3 kernel trace: per-kernel stats and the GPU's idle / overlap shares.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out/ctrace; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ctrace -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-scan --no-pmc ${BENCH_ARGS:-} > gpurun_out/ctrace/bench.json 2> gpurun_out/ctrace/bench.err \
    || { echo "trace failed"; tail -5 gpurun_out/ctrace/bench.err; exit 1; }
f=$(find gpurun_out/ctrace -name "*kernel_trace.csv" | head -1)
python3 scripts/kernel_totals.py $f | head -12
python3 scripts/trace_overlap.py $f 3000
grep '^{' gpurun_out/ctrace/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', round(d['value']), 'ms/step', round(d['ms_per_step'],2))"
