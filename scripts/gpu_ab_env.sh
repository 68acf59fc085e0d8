# A/B of environment settings of one library build, alternating on one box:
# VARIANTS="name1:VAR=x,VAR2=y name2:" (empty assignment list = defaults); BENCH_ARGS for bench.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/abenv
O=gpurun_out/abenv
for k in $(seq 1 ${RUNS:-3}); do
  for v in ${VARIANTS:-base:}; do
    name=${v%%:*}; assigns=${v#*:}
    ( IFS=','; for a in $assigns; do export "$a"; done; unset IFS
      timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-scan --no-pmc --no-dropin ${BENCH_ARGS:-} \
          > $O/b_${name}_$k.json 2> $O/b_${name}_$k.err ) || { echo "bench $name failed"; tail -5 $O/b_${name}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${name}_$k.json'));r=d['roofline'];print('$name', round(d['value'],1), round(d['ms_per_step'],3), 'k_bounce', round(r['avg_launch_ms']*1e3,1), 'us')"
  done
done
