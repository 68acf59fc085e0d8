# Round 5: analytic first bounces at 8 waves per SIMD (fw8: 64 VGPRs, 5 spilled) vs the tree (new, 7 waves).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
CASES="new:-: fw8:fw8:" RUNS=3 STEPS=20 bash scripts/gpu_ab_env.sh || exit 1
CASES="new:-: fw8:fw8:" BENCH_ARGS="--config multi_object_4k" RUNS=2 STEPS=5 bash scripts/gpu_ab_env.sh
