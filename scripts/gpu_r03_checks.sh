# Round 3 checks: the bounded closest hit against the plain per-geom loop over > 2 G rays
# (scripts/verify_bounds.py), then the 2- and 4-rank bench rehearsal on one GPU (gloo; functional
# only, scripts/gpu_rehearsal.sh).  Each step under its own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/verify_bounds.py ${VB_PASSES:-20} 30 > gpurun_out/verify_bounds.txt 2>&1 \
    || { echo "verify failed"; tail -5 gpurun_out/verify_bounds.txt; exit 1; }
tail -1 gpurun_out/verify_bounds.txt
python3 -c "
import re; t=sum(int(m.group(1)) for m in re.finditer(r'segments=\s*(\d+)', open('gpurun_out/verify_bounds.txt').read())); print('rays checked', t)"
bash scripts/gpu_rehearsal.sh
