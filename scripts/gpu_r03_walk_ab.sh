# k_traverse4 change: mesh parity tests (the device re-walk of every record, config 5 bit-exact),
# then config 5 A/B of the working-tree library against variant builds (scripts/build_variants.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/wab
timeout -k 10 600 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q \
    -k "${PYTEST_K:-walk_records or config5 or mesh_traversal}" --timeout 300 --timeout-method thread > gpurun_out/wab/tests.log 2>&1
rc=$?; tail -3 gpurun_out/wab/tests.log; [ $rc -eq 0 ] || exit 1
BENCH_ARGS="--config random_triangles_100k" STEPS=${STEPS:-4} RUNS=${RUNS:-2} bash scripts/gpu_ab_variants.sh
