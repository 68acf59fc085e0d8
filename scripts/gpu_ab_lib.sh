# A/B timing of the working-tree library vs build/libpt_amd_<v>.so for v in $VARIANTS (default: ab;
# scripts/build_ab.sh, scripts/build_flags_ab.sh), alternating on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/ab
O=gpurun_out/ab
for k in $(seq 1 ${RUNS:-3}); do
  for v in new ${VARIANTS:-ab}; do
    if [ $v = new ]; then unset PT_AMD_LIB; else export PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_$v.so; fi
    timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-scan --no-pmc ${BENCH_ARGS:-} \
        > $O/b_${v}_$k.json 2> $O/b_${v}_$k.err || { echo "bench $v failed"; tail -5 $O/b_${v}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${v}_$k.json'));r=d['roofline'];print('$v', round(d['value'],1), round(d['ms_per_step'],3), 'k_bounce', round(r['avg_launch_ms']*1e3,1), 'us; first', round(d.get('first_bounce_avg_ms',0)*1e3,1))"
  done
done
