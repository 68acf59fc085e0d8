# Round 5: later bounces at 8 waves per SIMD (lw8) after the code-size cuts vs the tree (new).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
CASES="new:-: lw8:lw8:" RUNS=3 STEPS=20 bash scripts/gpu_ab_env.sh || exit 1
CASES="new:-: lw8:lw8:" BENCH_ARGS="--config multi_object_4k" RUNS=2 STEPS=5 bash scripts/gpu_ab_env.sh
