# Alternating bench runs of (library, environment) variants on one box:
#   CASES="new:-: bs:bs: r8:-:PT_AMD_REFILL=8" BENCH_ARGS="--config random_triangles_100k" RUNS=2
# each case is name:lib:env (lib "-" = the tree's library, else build/libpt_amd_<lib>.so; env: A=1,B=2).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/abe; mkdir -p $O
for k in $(seq 1 ${RUNS:-2}); do
  for c in $CASES; do
    name=${c%%:*}; rest=${c#*:}; lib=${rest%%:*}; envs=${rest#*:}
    if [ "$lib" = - ]; then unset PT_AMD_LIB; else export PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_$lib.so; fi
    envline=$(echo "$envs" | tr ',' ' ')
    env $envline timeout -k 10 300 python -u bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-scan --no-pmc \
        --no-walk-counters --no-dropin ${BENCH_ARGS:-} > $O/b_${name}_$k.json 2> $O/b_${name}_$k.err \
        || { echo "bench $name failed"; tail -5 $O/b_${name}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${name}_$k.json'));r=d['roofline'];print('$name', round(d['value'],1), round(d['ms_per_step'],2), 'ms/step', r.get('kernel'), round(r.get('avg_launch_ms',0),3), round(r.get('first_traverse_avg_ms',0) or 0,2))"
  done
done
