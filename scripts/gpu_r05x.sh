# Round 5: the material-sorted producer specialised to LDS materials (new) vs the committed tree (ab):
# sorted parity tests, then config 3 A/B (and the producers at 6 waves per SIMD, pw6).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "sort or sorted or material or config3 or benched" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit 1; }
CASES="new:-: ab:ab: pw6:pw6:" BENCH_ARGS="--config cornell_hd_sorted" RUNS=3 STEPS=10 bash scripts/gpu_ab_env.sh
