# Round 5 (last): the full GPU suite of the final tree, then the drop-in leg alone.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest_gpu.log | head -20; exit 1; }
RUNS=2 ITERS=200 timeout -k 10 300 python -u scripts/dropin_ahead_ab.py > $O/dropin_ab.jsonl 2> $O/dropin_ab.err; rc=$?
cat $O/dropin_ab.jsonl; exit $rc
