# The empty-camera-mask skip in the FUSED first bounce ("fskip") vs the default (off there): config 4
# (4K, 16:9: many empty waves) and Cornell, alternating on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
VARIANTS="fskip" RUNS=3 STEPS=5 BENCH_ARGS="--config multi_object_4k" bash scripts/gpu_ab_variants.sh || exit 1
