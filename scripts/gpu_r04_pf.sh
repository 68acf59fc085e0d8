# Packed work list (slot, sorted position) per work position: sorted-pipeline parity, config 3 A/B
# against the separate arrays (library "sep").
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/pf; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 600 --timeout-method thread -k "sort or Sort or config3 or ends or verified or many_materials or histogram" \
    > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
VARIANTS="sep" RUNS=3 STEPS=10 BENCH_ARGS="--config cornell_hd_sorted" bash scripts/gpu_ab_variants.sh || exit 1
