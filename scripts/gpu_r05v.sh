# Round 5: config 5's walk refill threshold and ray chunk around their defaults (16 idle lanes, 256 rays).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
CASES="d:-: r12:-:PT_AMD_REFILL=12 r20:-:PT_AMD_REFILL=20 c192:-:PT_AMD_TCHUNK=192 c320:-:PT_AMD_TCHUNK=320" BENCH_ARGS="--config random_triangles_100k --samples 64 --spp 64" RUNS=2 STEPS=2 bash scripts/gpu_ab_env.sh
