# Plain fused first bounce skipping tiles whose four camera-mask blocks are empty: first-bounce and
# mask parity, then Cornell A/B against PT_SKIP_EMPTY_TILES=0 ("notile").
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/tile; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 600 --timeout-method thread -k "mask or skip or first or cornell" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
VARIANTS="notile" RUNS=3 STEPS=20 bash scripts/gpu_ab_variants.sh || exit 1
