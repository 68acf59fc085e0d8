# Round-4 evidence run: GPU parity tests, counter list, the bench line (with its in-run PMC passes),
# and the rocprofv3 kernel-trace stats of the same bench command (without the nested PMC leg, and without
# the drop-in leg, whose render-ahead passes launch the same k_bounce instantiation one iteration at a time).
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r04}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      > "$O/pytest_gpu.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -5 "$O/pytest_gpu.log"
  [ $rc -eq 0 ] || exit 1
fi
if [ "${LIST_COUNTERS:-0}" = 1 ]; then
  (cd /tmp && TMPDIR=/tmp timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1); echo "list rc=$?"
fi
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.log"; rc=$?
echo "bench rc=$rc"; tail -3 "$O/bench.log"; cat "$O/bench.json"
[ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktrace" -o run -- \
    python3 "$R/bench.py" --no-pmc --no-cpu-baseline --no-dropin --steps 20 ${BENCH_ARGS:-} > "$O/ktrace_bench.json" 2> "$O/ktrace_bench.log"; rc=$?
echo "ktrace rc=$rc"
[ $rc -eq 0 ] || exit 1
find "$O/ktrace" -name "*kernel_stats.csv" -exec head -12 {} \;
