set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
timeout -k 10 600 python -m pytest tests -q -m gpu -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
PT_PIPELINE=split timeout -k 10 600 python -m pytest tests/test_render_gpu.py -q -m gpu -x -p no:cacheprovider > gpurun_out/pytest_split.log 2>&1; rc=$?
echo "pytest split rc=$rc"; tail -2 gpurun_out/pytest_split.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/ab_pipeline.py
