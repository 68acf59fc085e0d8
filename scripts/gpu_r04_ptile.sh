# Sorted camera-ray producer skipping whole tiles whose camera-mask blocks are all empty (their
# ballots, barriers and material bookkeeping too): sorted/mask parity, then config 3 A/B against
# PT_SKIP_EMPTY_TILES=0 ("notile").
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/ptile; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 600 --timeout-method thread -k "sort or Sort or config3 or ends or mask or skip or first" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
VARIANTS="notile" RUNS=3 STEPS=10 BENCH_ARGS="--config cornell_hd_sorted" bash scripts/gpu_ab_variants.sh || exit 1
