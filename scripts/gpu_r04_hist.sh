# Round 4: k_hist_apply2 (lane-parallel work list of the sorted pipeline) — sorted-pipeline parity
# tests, then config 3 A/B against the per-run form (variant h1 = -DPT_HIST_APPLY=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/hist; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py tests/test_pin_thrust.py -m gpu -x -q -p no:cacheprovider \
    --timeout 600 --timeout-method thread -k "sort or Sort or config3 or ends or lanes or async or many_materials or histogram or pin" \
    > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
VARIANTS="h1" RUNS=2 STEPS=10 BENCH_ARGS="--config cornell_hd_sorted" bash scripts/gpu_ab_variants.sh || exit 1
