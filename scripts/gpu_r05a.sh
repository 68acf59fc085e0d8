# Round-5 first check: the new parity tests (benched pass sizes, full 2^28 scan, C++ self-test at
# 2^28, context-scoped synchronisation), then a quick Cornell bench line with the drop-in leg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
    -k "${PYTEST_K:-benched_pass_size or scoped or 2e28 or selftest or set_flags or async_lanes or deferred or resume}" \
    > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests.log | tail -30; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-scan --no-pmc > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value'],1), d['ms_per_step'], json.dumps(d.get('dropin')))"
