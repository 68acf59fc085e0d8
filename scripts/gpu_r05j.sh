# Round 5: the walk's refill segment cursor (new) vs a binary search per refill (bs), and refill at 8 idle lanes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "mesh or bvh or config5 or tcull or triangles or room or walk or traverse" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit 1; }
CASES="new:-: bs:bs: r8:-:PT_AMD_REFILL=8" BENCH_ARGS="--config random_triangles_100k --samples 64 --spp 64" RUNS=2 STEPS=2 bash scripts/gpu_ab_env.sh
