# Sorted pipeline with compacted records (only the survivors that go on, consecutive per run; each
# record carries its rank in the run): sorted-pipeline parity, config 3 A/B against the HEAD build
# ("head"), then the fused first bounce's empty-mask skip ("fskip") A/B on config 4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/compact; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 600 --timeout-method thread -k "sort or Sort or config3 or ends or verified or many_materials or histogram or mask" \
    > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
VARIANTS="head" RUNS=3 STEPS=10 BENCH_ARGS="--config cornell_hd_sorted" bash scripts/gpu_ab_variants.sh || exit 1
VARIANTS="fskip" RUNS=2 STEPS=5 BENCH_ARGS="--config multi_object_4k" bash scripts/gpu_ab_variants.sh || exit 1
