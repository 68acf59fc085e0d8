# Round 5: config 5 at its bench default (128 iterations per pass) with one lane (default) vs two lanes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
CASES="l1:-: l2:-:PT_AMD_LANES=2" BENCH_ARGS="--config random_triangles_100k" RUNS=2 STEPS=2 bash scripts/gpu_ab_env.sh
