# Mesh traversal round: parity tests of the mesh paths, k_traverse counters on config 5's scene,
# and config-5 bench lines (k_traverse vs the walk inside the bounce kernel).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/mesh
O=gpurun_out/mesh
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_render_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      -k "mesh or room or config5 or config_scenes or concurrent" > $O/tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
fi
python -c "from cuda_pathtracer_amd import scenes; print(scenes.random_triangles('$O/sc', n=100000, res=(960, 540), depth=32))" > $O/scene.txt || exit 1
timeout -k 10 300 python -u scripts/trav_stats.py $(cat $O/scene.txt) 1 > $O/trav.txt 2>&1; rc=$?
echo "trav rc=$rc"; cat $O/trav.txt | tail -2; [ $rc -eq 0 ] || exit 1
for mode in pre inline; do
  [ $mode = inline ] && export PT_AMD_MESH_INLINE=1
  timeout -k 10 300 python -u bench.py --config random_triangles_100k --spp 4 --samples 4 --steps 3 --warmup 1 \
      --no-cpu-baseline --no-scan --no-pmc > $O/bench_$mode.json 2> $O/bench_$mode.err; rc=$?
  echo "bench $mode rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench_$mode.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$mode.json'));print('$mode', round(d['value'],1), d['unit'], round(d['ms_per_step'],1), 'ms/step')"
done
