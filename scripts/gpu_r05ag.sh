# Round 5: 12-byte colour-buffer elements (branch exp/col12, built as libpt_amd_ab.so) vs the tree's 16-byte
# (new): render parity tests with the 12-byte library, then Cornell, config 4 and config 3 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05ag; mkdir -p $O
PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_ab.so timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit 1; }
CASES="new:-: c12:ab:" RUNS=3 STEPS=20 bash scripts/gpu_ab_env.sh || exit 1
CASES="new:-: c12:ab:" BENCH_ARGS="--config multi_object_4k" RUNS=2 STEPS=5 bash scripts/gpu_ab_env.sh || exit 1
CASES="new:-: c12:ab:" BENCH_ARGS="--config cornell_hd_sorted" RUNS=2 STEPS=10 bash scripts/gpu_ab_env.sh
