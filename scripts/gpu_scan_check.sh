# Scan parity tests on the GPU, then the scan timing sweep (stops at the first failure).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_scan_gpu.py tests/test_cpp_gpu.py -q -x -m gpu -p no:cacheprovider > gpurun_out/pytest_scan.log 2>&1 \
  || { echo "scan tests failed"; tail -30 gpurun_out/pytest_scan.log; exit 1; }
tail -1 gpurun_out/pytest_scan.log
bash scripts/gpu_scan_ablate.sh
