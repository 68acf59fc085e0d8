# Round 5: the bounded closest hit (with the one-geom camera masks) against the plain per-geom loop on the
# device over ~5 G segments (scripts/verify_bounds.py 8 6 64), then the render-ahead tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 900 python -u scripts/verify_bounds.py 8 6 64 > $O/verify_bounds.txt 2>&1; rc=$?
tail -12 $O/verify_bounds.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "render_ahead" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; exit $rc
