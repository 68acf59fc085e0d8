# Sorted-pipeline round: the full GPU suite, then config 3's bench line and kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/sorted
O=gpurun_out/sorted
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      ${PYTEST_K:+-k "$PYTEST_K"} > $O/tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 300 python -u bench.py --config cornell_hd_sorted --steps 5 --warmup 2 --no-cpu-baseline --no-scan --no-pmc \
    > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('config3', round(d['value'],1), d['unit'], round(d['ms_per_step'],2), 'ms/step')"
CFG=cornell_hd_sorted SPP=32 STEPS=3 bash scripts/gpu_config_prof.sh
