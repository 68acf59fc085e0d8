# Round 4: the exact t-cull — mesh parity + the device re-walk verification, then A/B of the cull
# on the tessellated-mesh workload and on config 5 (PT_AMD_TCULL forces it on/off).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/tcull; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py tests/test_bvh_device_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 600 --timeout-method thread -k "room or mesh or bvh or config5 or walk or concurrent or tcull or tessellated" \
    > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
[ "${SKIP_AB:-0}" = 1 ] && exit 0
VARIANTS="on:PT_AMD_TCULL=1 off:PT_AMD_TCULL=0" RUNS=2 STEPS=3 \
    BENCH_ARGS="--config tessellated_meshes_100k --samples 128 --spp 128" bash scripts/gpu_ab_env.sh || exit 1
VARIANTS="off:PT_AMD_TCULL=0 on:PT_AMD_TCULL=1" RUNS=2 STEPS=2 \
    BENCH_ARGS="--config random_triangles_100k --samples 128 --spp 128" bash scripts/gpu_ab_env.sh || exit 1
