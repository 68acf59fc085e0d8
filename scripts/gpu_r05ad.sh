# Round 5: analytic bounce kernels for scenes whose materials are all plain (no texture, not refractive:
# k_bounce modes 5 / 6) (new) vs the committed tree (ab): render parity tests, then Cornell and config 4 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05ad; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit 1; }
CASES="new:-: ab:ab:" RUNS=3 STEPS=20 bash scripts/gpu_ab_env.sh || exit 1
CASES="new:-: ab:ab:" BENCH_ARGS="--config multi_object_4k" RUNS=2 STEPS=5 bash scripts/gpu_ab_env.sh
