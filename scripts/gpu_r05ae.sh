# Round 5: the sorted producers at 6 / 8 waves per SIMD after the code-size cuts vs 7 (new): config 3 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
CASES="new:-: pw6:pw6: pw8:pw8:" BENCH_ARGS="--config cornell_hd_sorted" RUNS=3 STEPS=10 bash scripts/gpu_ab_env.sh
