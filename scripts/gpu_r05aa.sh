# Round 5: the bounded hit's exact tests as one candidate loop (one inlined exact test; the plain per-geom
# loop for uncovered directions folded into it) (new) vs the committed tree (ab): render parity tests, the
# bounded-vs-plain device verification at scale, then Cornell, config 4 and config 3 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05aa; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit 1; }
timeout -k 10 900 python -u scripts/verify_bounds.py 8 6 64 > $O/verify_bounds.txt 2>&1; rc=$?
tail -2 $O/verify_bounds.txt; [ $rc -eq 0 ] || exit 1
CASES="new:-: ab:ab:" RUNS=3 STEPS=20 bash scripts/gpu_ab_env.sh || exit 1
CASES="new:-: ab:ab:" BENCH_ARGS="--config multi_object_4k" RUNS=2 STEPS=5 bash scripts/gpu_ab_env.sh || exit 1
CASES="new:-: ab:ab:" BENCH_ARGS="--config cornell_hd_sorted" RUNS=2 STEPS=10 bash scripts/gpu_ab_env.sh
