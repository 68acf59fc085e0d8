# k_traverse ticket chunk / refill sweep on the config-5 bench (spp 8).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/mesh
O=gpurun_out/mesh
for cfg in ${CFGS:-64:16 128:16 256:16 64:32}; do
  export PT_AMD_TCHUNK=${cfg%%:*} PT_AMD_REFILL=${cfg##*:}
  timeout -k 10 300 python -u bench.py --config random_triangles_100k --spp 8 --samples 8 --steps 3 --warmup 1 \
      --no-cpu-baseline --no-scan --no-pmc > $O/bench_c$cfg.json 2> $O/bench_c$cfg.err || { echo "bench failed"; tail -3 $O/bench_c$cfg.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_c$cfg.json'));print('chunk:refill $cfg', round(d['value'],1), d['unit'], round(d['ms_per_step'],1), 'ms/step')"
done
