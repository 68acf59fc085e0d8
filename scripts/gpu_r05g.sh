# Context stream reuse check: the synchronisation tests, then config 3 and Cornell bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "scoped or deferred or async_lanes or set_flags or resume or two_lanes" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head; exit 1; }
for c in cornell_hd_sorted cornell; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-scan --no-pmc --no-dropin > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$c.json'));print('$c', round(d['value'],1), round(d['ms_per_step'],3))"
done
