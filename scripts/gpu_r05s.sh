# Round 5: rank 0's share of an 8-GPU strong-scaling step traced alone (PT_BENCH_SHARD_OF=8: 100 rows x 256
# iterations per pass), with 2 (default), 3 and 4 lanes (8 hardware queues so lanes do not share one); and
# the same for N = 4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
CASES="s8l2:-:PT_BENCH_SHARD_OF=8 s8l3:-:PT_BENCH_SHARD_OF=8,PT_AMD_LANES=3,GPU_MAX_HW_QUEUES=8 s8l4:-:PT_BENCH_SHARD_OF=8,PT_AMD_LANES=4,GPU_MAX_HW_QUEUES=8 s4l2:-:PT_BENCH_SHARD_OF=4 s4l3:-:PT_BENCH_SHARD_OF=4,PT_AMD_LANES=3,GPU_MAX_HW_QUEUES=8" RUNS=2 STEPS=50 bash scripts/gpu_ab_env.sh
