set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/dropin_trace"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O" -o run -- python3 "$R/scripts/dropin_trace.py" > "$O/out.txt" 2>&1; echo "rc=$?"
find "$O" -name "*.csv" | head
