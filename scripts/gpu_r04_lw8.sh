# Cornell: later bounces at 8 waves per SIMD (PT_LATER_WAVES=8, SGPRs capped) vs the default, re-measured
# with the round-4 kernels; alternating on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
VARIANTS="lw8" RUNS=3 STEPS=20 bash scripts/gpu_ab_variants.sh || exit 1
