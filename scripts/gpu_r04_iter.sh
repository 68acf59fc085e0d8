# Sorted producer with the tile's iteration found incrementally and kept uniform: sorted-pipeline
# parity + the preview GPU tests, then config 3 A/B against the HEAD build (library "head").
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/iter; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py tests/test_preview_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 600 --timeout-method thread -k "sort or Sort or config3 or ends or verified or many_materials or histogram or preview or session or window" \
    > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
VARIANTS="head" RUNS=3 STEPS=10 BENCH_ARGS="--config cornell_hd_sorted" bash scripts/gpu_ab_variants.sh || exit 1
