# Alternating bench runs of the working-tree library and variant libraries (scripts/build_variants.sh)
# on one box: VARIANTS="a b" BENCH_ARGS="--config random_triangles_100k --samples 32 --spp 32" RUNS=2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/abv; mkdir -p $O
for k in $(seq 1 ${RUNS:-2}); do
  for v in ${BASE:-new} $VARIANTS; do
    if [ $v = new ]; then unset PT_AMD_LIB; else export PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_$v.so; fi
    timeout -k 10 300 python -u bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-scan --no-pmc --no-walk-counters --no-dropin \
        ${BENCH_ARGS:-} > $O/b_${v}_$k.json 2> $O/b_${v}_$k.err || { echo "bench $v failed"; tail -5 $O/b_${v}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${v}_$k.json'));r=d['roofline'];print('$v', round(d['value'],1), round(d['ms_per_step'],2), 'ms/step', r.get('kernel'), round(r.get('avg_launch_ms',0),3))"
  done
done
