# Cornell A/B of the working-tree library against variant builds (scripts/build_variants.sh),
# after the render parity tests (-k PYTEST_K) of the working tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/cab
timeout -k 10 600 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q \
    -k "${PYTEST_K:-batched or bitexact}" --timeout 300 --timeout-method thread > gpurun_out/cab/tests.log 2>&1
rc=$?; tail -3 gpurun_out/cab/tests.log; [ $rc -eq 0 ] || exit 1
STEPS=${STEPS:-20} RUNS=${RUNS:-3} bash scripts/gpu_ab_variants.sh
