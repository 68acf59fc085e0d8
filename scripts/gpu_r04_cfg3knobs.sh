# Config 3 knobs after the compacted records: histogram-scan grid 8 per CU (hg8), producers at 6
# waves per SIMD (pw6), and 2 / 4 lanes instead of 3 — alternating on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
VARIANTS="hg8 pw6" RUNS=2 STEPS=10 BENCH_ARGS="--config cornell_hd_sorted" bash scripts/gpu_ab_variants.sh || exit 1
VARIANTS="l3:PT_AMD_LANES=3 l2:PT_AMD_LANES=2 l4:PT_AMD_LANES=4" RUNS=2 STEPS=10 BENCH_ARGS="--config cornell_hd_sorted" bash scripts/gpu_ab_env.sh || exit 1
