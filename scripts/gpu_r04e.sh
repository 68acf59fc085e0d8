# Late round-4 evidence (TAG r04e): the r04c chain (GPU suite, bench + kernel trace, config lines,
# config 3 breakdown), then the fused empty-wave skip's env A/B on config 4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${TAG:-r04e} bash scripts/gpu_r04c.sh || exit 1
cd "$R" && VARIANTS="auto: off:PT_AMD_SKIP_EMPTY=0" RUNS=2 STEPS=5 BENCH_ARGS="--config multi_object_4k" bash scripts/gpu_ab_env.sh || exit 1
