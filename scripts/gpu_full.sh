# Full GPU evidence pass: all GPU tests, then the bench lines of configs 3-5 (config 5 also with
# the bvh_cull extension).  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
bash scripts/gpu_tests.sh || exit 1
bash scripts/gpu_configs.sh || exit 1
timeout -k 10 300 python bench.py --config random_triangles_100k --bvh-cull --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-scan \
    >> gpurun_out/configs.jsonl 2> gpurun_out/config_cull.err || { echo "cull bench failed"; tail -5 gpurun_out/config_cull.err; exit 1; }
tail -1 gpurun_out/configs.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('config 5 + bvh_cull', round(d['value'],1), 'Mray/s', round(d['ms_per_step'],2), 'ms/step')"
