# Multi-rank bench rehearsal on one GPU (PT_BENCH_REHEARSAL=1: ranks share the device, gloo
# collectives): exercises the N > 1 path of bench.py (row shards, gather, max-over-ranks timing)
# with its current defaults.  Functional only; never a measurement.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/rehearsal
O=gpurun_out/rehearsal
: > $O/lines.jsonl
for n in ${NS:-2 4}; do
  PT_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 3 --warmup 1 \
      --no-cpu-baseline --no-scan --no-pmc >> $O/lines.jsonl 2> $O/n$n.err || { echo "n=$n failed"; tail -5 $O/n$n.err; exit 1; }
  echo "n=$n ok"
done
python3 -c "
import json
for l in open('$O/lines.jsonl'):
    if not l.startswith('{'): continue   # (gloo prints its connection lines on stdout)
    d=json.loads(l); print(d['n_gpus'], round(d['value'],1), d['scaling'], d['config']['passes_per_step'], d['config']['iterations_per_pass'], d['config']['parallelism'])"
