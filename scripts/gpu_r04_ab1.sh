# Round 4 A/B batch: k_traverse4 occupancy variants on config 5, then Cornell lane counts.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
VARIANTS="w5b1 w5b2 b1" RUNS=2 STEPS=2 BENCH_ARGS="--config random_triangles_100k --samples 128 --spp 128" \
    bash scripts/gpu_ab_variants.sh || exit 1
VARIANTS="l2: l3:PT_AMD_LANES=3 l4:PT_AMD_LANES=4" RUNS=2 STEPS=20 bash scripts/gpu_ab_env.sh || exit 1
