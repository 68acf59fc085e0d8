# Round 5 config-5 evidence: the bench line with its in-run PMC passes and walk counters, then the walk
# counters with one triangle task per lane (round 4's walk) for comparison.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 900 python -u bench.py --config random_triangles_100k --steps 2 > $O/cfg5.json 2> $O/cfg5.err; rc=$?
tail -3 $O/cfg5.err; cat $O/cfg5.json; [ $rc -eq 0 ] || exit 1
S=$(ls -d gpurun_out/bench_scenes 2>/dev/null)
SC=$(python -c "import sys; sys.path.insert(0,'.'); from cuda_pathtracer_amd import scenes; print(scenes.random_triangles('$O/scene'))")
for k in 1 2; do
  PT_AMD_WALK_TASKS=$k timeout -k 10 300 python -u scripts/trav_stats.py $SC 128 > $O/trav_k$k.txt 2>&1 || exit 1
  echo "K=$k $(tail -1 $O/trav_k$k.txt)"
done
