# Cornell bench at several iterations-per-pass batch sizes (bit-identical results).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for s in ${SPPS:-1 2 4 8}; do
  timeout -k 10 300 python bench.py --spp $s --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline --no-scan \
      > gpurun_out/spp$s.json 2> gpurun_out/spp$s.err || { echo "spp $s failed"; tail -5 gpurun_out/spp$s.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/spp$s.json')); print('spp=$s', round(d['value'],1), 'Mray/s', round(d['ms_per_step'],3), 'ms/step', 'bounce avg', round(d['roofline']['avg_launch_ms']*1e3,1), 'us')"
done
