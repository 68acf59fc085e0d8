# First-bounce waves with an empty camera mask skip raygen + closest hit: render parity (camera-mask,
# sorted, config-3 full size, first-bounce cases), then A/B against PT_SKIP_MISS_WAVES=0 ("noskip")
# on config 3 and on the Cornell bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/skip; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 600 --timeout-method thread -k "mask or sort or Sort or config3 or ends or verified or first or cornell" \
    > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
VARIANTS="noskip" RUNS=3 STEPS=10 BENCH_ARGS="--config cornell_hd_sorted" bash scripts/gpu_ab_variants.sh || exit 1
VARIANTS="noskip" RUNS=3 STEPS=20 bash scripts/gpu_ab_variants.sh || exit 1
