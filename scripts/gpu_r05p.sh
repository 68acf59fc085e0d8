# Round 5: later bounces prefetch the next tile's path (new) vs load it in place (np): render parity tests,
# then the Cornell bench line A/B and config 4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit 1; }
CASES="new:-: np:np:" RUNS=3 STEPS=20 bash scripts/gpu_ab_env.sh || exit 1
CASES="new:-: np:np:" BENCH_ARGS="--config multi_object_4k" RUNS=1 STEPS=5 bash scripts/gpu_ab_env.sh
