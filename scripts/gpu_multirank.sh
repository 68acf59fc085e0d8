# Functional rehearsal of bench.py's N>1 path on a 1-GPU box: 2 ranks share the GPU, gloo
# collectives (PT_BENCH_REHEARSAL=1) and the claimed tile schedule (PT_AMD_SCHEDULE=claim: the two
# ranks share the GPU).  Checks the sharding, gather and max/sum reductions run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
PT_AMD_SCHEDULE=claim PT_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus ${NPROC:-2} --steps 20 --warmup 3 --no-scan \
    > gpurun_out/multirank.json 2> gpurun_out/multirank.err || { echo "rehearsal failed"; tail -20 gpurun_out/multirank.err; exit 1; }
cat gpurun_out/multirank.json
