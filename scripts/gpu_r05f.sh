# Walk knobs re-measured with two triangle tasks per lane: fold batch, leaf+node overlap (variants),
# refill threshold and ray chunk (environment), config 5 at 64 iterations per pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05f; mkdir -p $O
VARIANTS="fb2 fb8 ov0" BENCH_ARGS="--config random_triangles_100k --samples 64 --spp 64" RUNS=1 STEPS=2 bash scripts/gpu_ab_variants.sh || exit 1
for e in "PT_AMD_REFILL=8" "PT_AMD_REFILL=32" "PT_AMD_TCHUNK=128" "PT_AMD_TCHUNK=512" "X=1"; do
  env $e timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-scan --no-pmc --no-walk-counters --no-dropin \
      --config random_triangles_100k --samples 64 --spp 64 > $O/e.json 2> $O/e.err || { echo "bench $e failed"; tail -5 $O/e.err; exit 1; }
  python -c "import json;d=json.load(open('$O/e.json'));print('$e', round(d['value'],1), round(d['roofline']['avg_launch_ms'],3))"
done
