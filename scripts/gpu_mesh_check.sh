# Mesh parity tests then config-5 timing with and without the bvh_cull extension.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
PYTEST_K="room or config_scenes" bash scripts/gpu_tests.sh || exit 1
for cull in "" "--bvh-cull"; do
  timeout -k 10 300 python bench.py --config random_triangles_100k $cull --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-scan \
      > gpurun_out/tri.json 2> gpurun_out/tri.err || { echo "bench failed"; tail -5 gpurun_out/tri.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/tri.json')); print('cull=$cull', round(d['value'],1), 'Mray/s', round(d['ms_per_step'],2), 'ms/step')"
done
