# Scan tuning sweep: one process per setting, each under its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
run() { TAG="$1" timeout -k 10 120 env ${2//,/ } python scripts/scan_ablate.py >> gpurun_out/scan_ablate.log 2>&1 || { echo "FAILED $1"; exit 1; }; }
: > gpurun_out/scan_ablate.log
for v in ${SWEEP:-base:SC_EXPERIMENT=0 single:SC_MALL=0}; do run "${v%%:*}" "${v#*:}"; done
grep -v amdgpu.ids gpurun_out/scan_ablate.log
