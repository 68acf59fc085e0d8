# Round 3: k_traverse4 (4-wide layout, leaf tasks) vs round 2's pair walk on config 5.
# Mesh parity tests first, then counters (diagnostic build) and config-5 bench lines for both walks.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/trav3; mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_render_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
      -k "mesh or room or config5 or random_triangles or bvh_walk or refraction or config_scenes or glass" > $O/tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
fi
python -c "from cuda_pathtracer_amd import scenes; print(scenes.random_triangles('$O/sc4k', n=100000, res=(3840, 2160), depth=32))" > $O/scene4k.txt || exit 1
for walk in ${WALKS:-quad pairs}; do
  if [ $walk = pairs ]; then export PT_AMD_TRAV=pairs; else unset PT_AMD_TRAV; fi
  timeout -k 10 300 python -u scripts/trav_stats.py $(cat $O/scene4k.txt) 1 > $O/trav_$walk.txt 2>&1 || { echo "trav failed"; tail -3 $O/trav_$walk.txt; exit 1; }
  echo "$walk: $(tail -1 $O/trav_$walk.txt)"
  timeout -k 10 300 python -u bench.py --config random_triangles_100k --steps ${STEPS:-3} --warmup 1 \
      --no-cpu-baseline --no-scan --no-pmc --no-walk-counters > $O/bench_$walk.json 2> $O/bench_$walk.err || { echo "bench failed"; tail -3 $O/bench_$walk.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$walk.json'));r=d['roofline'];print('  $walk bench', round(d['value'],1), d['unit'], round(d['ms_per_step'],1), 'ms/step', r.get('kernel'), round(r.get('avg_launch_ms',0),3))"
done
