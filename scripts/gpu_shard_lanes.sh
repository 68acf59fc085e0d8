set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/shard
export PT_BENCH_SHARD_OF=8
for L in 2 3 4 2 3; do
  PT_AMD_LANES=$L timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-scan --no-pmc > gpurun_out/shard/l$L.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/shard/l$L.json'));print('lanes', $L, round(d['value'],1), round(d['ms_per_step'],3))"
done
