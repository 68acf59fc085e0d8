# Development loop on the GPU box: parity tests, the bounded-hit verification, a short bench.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
if [ -z "$NO_VERIFY" ]; then
  timeout -k 10 300 python -u scripts/verify_bounds.py ${VERIFY_PASSES:-8} > gpurun_out/verify.log 2>&1; rc=$?
  cat gpurun_out/verify.log; [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));r=d['roofline'];print('value',round(d['value'],1),'ms/step',round(d['ms_per_step'],4),'bounce_ms',round(r['avg_launch_ms'],4),'first_ms',round(d['first_bounce_avg_ms'],4),'scan',round(d.get('scan',{}).get('GB/s',0),1))"
