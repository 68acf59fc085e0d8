# Everything the round's evidence needs, in one box session: GPU parity tests, bench + kernel-trace
# stats, PMC traffic passes, scan A/B.  Stops at the first failing step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash scripts/gpu_test_bench.sh || exit 1
bash scripts/gpu_traffic.sh || exit 1
bash scripts/gpu_scan_ablate.sh || exit 1
