# Context-scoped sync test under 16 and default hardware queues, then the bench's drop-in leg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05b; mkdir -p $O
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python -u -m pytest tests/test_render_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 200 \
    --timeout-method thread -k scoped > $O/t16.log 2>&1; echo "hwq16 rc=$?"; grep -E "Error|passed|failed" $O/t16.log | tail -3
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-scan --no-pmc > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value'],1), d['ms_per_step'], json.dumps(d.get('dropin')))"
