# A/B of bench.py argument sets on one box, alternating: ARGSETS="name1|--spp 16;name2|--spp 64"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/abargs
O=gpurun_out/abargs
IFS=';' read -ra SETS <<< "${ARGSETS:-base|}"
for k in $(seq 1 ${RUNS:-2}); do
  for v in "${SETS[@]}"; do
    name=${v%%|*}; args=${v#*|}
    timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-scan --no-pmc $args \
        > $O/b_${name}_$k.json 2> $O/b_${name}_$k.err || { echo "bench $name failed"; tail -5 $O/b_${name}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${name}_$k.json'));r=d['roofline'];print('$name', round(d['value'],1), round(d['ms_per_step'],3), 'k_bounce', round(r['avg_launch_ms']*1e3,1), 'us')"
  done
done
