# k_traverse sweep: LDS stack rows and iterations per pass, config-5 bench lines; counters at 4K.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/mesh
O=gpurun_out/mesh
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_render_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      -k "mesh or room or config5 or config_scenes or concurrent" > $O/tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
fi
python -c "from cuda_pathtracer_amd import scenes; print(scenes.random_triangles('$O/sc4k', n=100000, res=(3840, 2160), depth=32))" > $O/scene4k.txt || exit 1
for rows in ${ROWS:-12 24}; do
  export PT_AMD_STACK_ROWS=$rows
  timeout -k 10 300 python -u scripts/trav_stats.py $(cat $O/scene4k.txt) 1 > $O/trav_r$rows.txt 2>&1 || { echo "trav failed"; tail -3 $O/trav_r$rows.txt; exit 1; }
  echo "rows $rows: $(tail -1 $O/trav_r$rows.txt)"
  for spp in ${SPPS:-4 8}; do
    timeout -k 10 300 python -u bench.py --config random_triangles_100k --spp $spp --samples $spp --steps 3 --warmup 1 \
        --no-cpu-baseline --no-scan --no-pmc > $O/bench_r${rows}_s$spp.json 2> $O/bench_r${rows}_s$spp.err || { echo "bench failed"; tail -3 $O/bench_r${rows}_s$spp.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_r${rows}_s$spp.json'));print('  rows $rows spp $spp bench', round(d['value'],1), d['unit'], round(d['ms_per_step'],1), 'ms/step')"
  done
done
