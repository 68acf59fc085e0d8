# PC sampling (rocprofv3 beta, host-trap) of the Cornell bench: which instructions of the hot
# kernels the waves sit on.  Lists the available configurations first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/pcs"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$O/list.txt" 2>&1; echo "list rc=$?"
grep -i -A12 "pc.sampl" "$O/list.txt" | head -40 || true
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${PCS_METHOD:-host_trap} \
    --pc-sampling-unit ${PCS_UNIT:-time} --pc-sampling-interval ${PCS_INTERVAL:-1} --output-format csv -d "$O/run" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-pmc --no-cpu-baseline --no-scan --no-dropin \
    > "$O/bench.json" 2> "$O/bench.err"; rc=$?
echo "pcs rc=$rc"; tail -5 "$O/bench.err"
find "$O/run" -type f | head; for f in $(find "$O/run" -name "*.csv"); do echo "== $f"; head -3 "$f"; wc -l "$f"; done
exit $rc
