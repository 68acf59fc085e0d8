# Round 5: more HIP hardware queues per process (GPU_MAX_HW_QUEUES, default 4) and the lane counts they
# allow without two streams sharing a queue: Cornell 2 / 3 lanes, config 3 3 / 4 lanes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
CASES="q4:-: q8:-:GPU_MAX_HW_QUEUES=8 q8l3:-:GPU_MAX_HW_QUEUES=8,PT_AMD_LANES=3 q4l3:-:PT_AMD_LANES=3" RUNS=2 STEPS=20 bash scripts/gpu_ab_env.sh || exit 1
CASES="q4:-: q8:-:GPU_MAX_HW_QUEUES=8 q8l4:-:GPU_MAX_HW_QUEUES=8,PT_AMD_LANES=4" BENCH_ARGS="--config cornell_hd_sorted" RUNS=2 STEPS=10 bash scripts/gpu_ab_env.sh
