# GPU test suite only (verbose on failures; prints of the statistical test kept with -s).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x -s -p no:cacheprovider ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "channel means|passed|failed|Error|error" gpurun_out/pytest_gpu.log | tail -15
exit $rc
