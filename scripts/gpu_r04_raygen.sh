# Raygen's uniform camera products made on the host (fused first bounce 70 -> 62 VGPRs, camera-ray
# producer without its 20-byte spill): render parity, then Cornell and config 3 A/B against HEAD.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/raygen; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 600 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
VARIANTS="head" RUNS=3 STEPS=20 bash scripts/gpu_ab_variants.sh || exit 1
VARIANTS="head" RUNS=2 STEPS=10 BENCH_ARGS="--config cornell_hd_sorted" bash scripts/gpu_ab_variants.sh || exit 1
