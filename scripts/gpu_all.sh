# tests -> bench (+rocprof kernel trace) -> per-bounce trace; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash scripts/gpu_test_bench.sh || exit 1
bash scripts/gpu_ablate.sh || exit 1
