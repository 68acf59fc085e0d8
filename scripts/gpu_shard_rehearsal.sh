# Strong-scaling rehearsal on one GPU: the 1-GPU bench line, then rank 0's share of an N-GPU step
# traced alone (PT_BENCH_SHARD_OF=N) for N = 2, 4, 8.  Predicted N-GPU value ~ N x rank 0's rate
# (row-interleaved shards are balanced); the gather and the collectives are not in it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/shard
O=gpurun_out/shard
for n in 1 2 4 8; do
  if [ $n = 1 ]; then unset PT_BENCH_SHARD_OF; else export PT_BENCH_SHARD_OF=$n; fi
  timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-scan --no-pmc \
      > $O/shard_$n.json 2> $O/shard_$n.err || { echo "shard $n failed"; tail -5 $O/shard_$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/shard_$n.json'));print('shard_of', $n, 'rank-0 Mray/s', round(d['value'],1), 'ms/step', round(d['ms_per_step'],3), 'predicted x$n', round(d['value']*$n,1))"
done
