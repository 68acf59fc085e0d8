# A walk variant (build/libpt_amd_$V.so): the mesh parity tests with it, then config 5 A/B vs the tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/walkv; mkdir -p $O
PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_$V.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread -k "${PYTEST_K:-mesh or bvh or config5 or tcull or triangles or room or walk or traverse}" \
    > $O/tests_$V.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests_$V.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests_$V.log | head -20; exit 1; }
VARIANTS="$V" BENCH_ARGS="--config random_triangles_100k --samples 64 --spp 64" RUNS=${RUNS:-2} STEPS=2 bash scripts/gpu_ab_variants.sh
