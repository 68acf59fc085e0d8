# Triangle tasks per lane per trip (PT_T4_TASKS = 2, 3, 4; 3 at 4 waves per SIMD): mesh parity of 3 and 4,
# then config 5 A/B at 64 iterations per pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05e; mkdir -p $O
for V in k3 k4; do
  PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_$V.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
      --timeout 300 --timeout-method thread -k "mesh or bvh or config5 or tcull or triangles or room or walk or traverse" \
      > $O/tests_$V.log 2>&1; rc=$?
  echo "$V tests rc=$rc"; tail -1 $O/tests_$V.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests_$V.log | head -20; exit 1; }
done
BASE=k2 VARIANTS="k3 k4 k3w4" BENCH_ARGS="--config random_triangles_100k --samples 64 --spp 64" RUNS=2 STEPS=2 bash scripts/gpu_ab_variants.sh
