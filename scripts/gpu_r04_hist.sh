# Round 4: k_hist_apply2 (lane-parallel work list of the sorted pipeline), built as variant h2
# (-DPT_HIST_APPLY=2): sorted-pipeline parity tests on that library, then config 3 A/B vs the default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/hist; mkdir -p $O
PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_h2.so timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py \
    -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread \
    -k "sort or Sort or config3 or ends or lanes or async or many_materials or histogram" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
VARIANTS="h2" RUNS=2 STEPS=10 BENCH_ARGS="--config cornell_hd_sorted" bash scripts/gpu_ab_variants.sh || exit 1
