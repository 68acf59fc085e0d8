# Round 4: the 4-wide walk's cooperative quad fetch — mesh parity tests, then alternating config-5
# bench runs of the working tree against variant libraries (scripts/build_variants.sh, built here).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/walk; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_render_gpu.py tests/test_bvh_device_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread -k "room or mesh or bvh or config5 or walk or concurrent" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
[ -z "$VARIANTS" ] && exit 0
VARIANTS="$VARIANTS" RUNS=${RUNS:-2} STEPS=${STEPS:-2} BENCH_ARGS="${BENCH_ARGS:---config random_triangles_100k --samples 128 --spp 128}" \
    bash scripts/gpu_ab_variants.sh
