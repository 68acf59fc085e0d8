# Round 5 config-5 evidence: the default walk (two triangle tasks per lane, no cull) re-walked against the
# reference's node-at-a-time walk over >= 1 G segments, then the config-5 bench line with its in-run PMC
# passes and walk counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05l; mkdir -p $O
TCULL=auto timeout -k 10 900 python -u scripts/verify_tcull_big.py > $O/verify_walk_1g.txt 2>&1; rc=$?
tail -4 $O/verify_walk_1g.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u bench.py --config random_triangles_100k --steps 2 > $O/cfg5.json 2> $O/cfg5.err; rc=$?
tail -3 $O/cfg5.err; cat $O/cfg5.json; exit $rc
