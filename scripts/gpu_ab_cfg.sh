# A/B of library builds (product vs build/libpt_amd_<v>.so for v in $VARIANTS, default ab) on one BASELINE config, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/abcfg
O=gpurun_out/abcfg
for k in $(seq 1 ${RUNS:-2}); do
  for v in new ${VARIANTS:-ab}; do
    if [ $v = new ]; then unset PT_AMD_LIB; else export PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_$v.so; fi
    timeout -k 10 300 python -u bench.py --config ${CFG:-cornell_hd_sorted} --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-scan --no-pmc ${BENCH_ARGS:-} \
        > $O/b_${v}_$k.json 2> $O/b_${v}_$k.err || { echo "bench $v failed"; tail -5 $O/b_${v}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${v}_$k.json'));print('$v', round(d['value'],1), round(d['ms_per_step'],3))"
  done
done
