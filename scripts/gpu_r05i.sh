# Round 5: render-ahead (pt_render_ahead) — its parity tests, the mirror's CLI and sync tests, then the
# drop-in call sequence with and without it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "render_ahead or set_flags or cli or context_synchronisation or batched_pass_equals or tiles_and_batched or resume" \
    > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit 1; }
timeout -k 10 300 python -u scripts/dropin_ahead_ab.py > $O/dropin_ab.jsonl 2> $O/dropin_ab.err; rc=$?
cat $O/dropin_ab.jsonl; exit $rc
