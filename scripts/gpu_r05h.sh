# Round 5: the walk's 72-byte group loads (new) vs six 12-byte loads (x3) and the camera-ray walk at
# 4 waves per SIMD (f4): mesh parity tests with the tree's library, then config 5 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "mesh or bvh or config5 or tcull or triangles or room or walk or traverse" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit 1; }
VARIANTS="x3 f4" BENCH_ARGS="--config random_triangles_100k --samples 64 --spp 64" RUNS=2 STEPS=2 bash scripts/gpu_ab_variants.sh
