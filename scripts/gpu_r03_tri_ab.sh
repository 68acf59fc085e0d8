# Walk task loads (triangle layout A/B): mesh parity tests, then config 5 alternating with the
# 48-byte array-of-structures variant (libpt_amd_aos.so, -DPT_T4_TRI_PACK=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_render_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "mesh or room or bvh or walk or triangles or config5 or config_scenes" > gpurun_out/mesh_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/mesh_tests.log; exit 1; }
tail -1 gpurun_out/mesh_tests.log
VARIANTS="aos" BENCH_ARGS="--config random_triangles_100k --spp 32 --samples 32" STEPS=2 RUNS=2 bash scripts/gpu_ab_variants.sh
