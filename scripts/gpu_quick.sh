# Quick round: GPU suite (optional -k), then Cornell bench lines (no PMC, no CPU legs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/quick
O=gpurun_out/quick
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      ${PYTEST_K:+-k "$PYTEST_K"} > $O/tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit 1
fi
for k in $(seq 1 ${RUNS:-2}); do
  timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-scan --no-pmc ${BENCH_ARGS:-} \
      > $O/bench_$k.json 2> $O/bench_$k.err || { echo "bench failed"; tail -5 $O/bench_$k.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$k.json'));r=d['roofline'];print('cornell', round(d['value'],1), d['unit'], round(d['ms_per_step'],3), 'ms/step; k_bounce avg', round(r['avg_launch_ms']*1e3,1), 'us frac', round(r['frac'],3))"
done
