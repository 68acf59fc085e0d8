# Stall / issue counters for Cornell and config 4's scene at 800x800 (scripts/stall_pmc.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/stall4/s800
python -c "from cuda_pathtracer_amd import scenes; scenes.multi_object('gpurun_out/stall4/s800', res=(800, 800))" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python "$R/scripts/stall_pmc.py" "$R/gpurun_out/stall4/cornell" > "$R/gpurun_out/stall4/cornell.txt" 2>&1 || exit 1
timeout -k 10 400 python "$R/scripts/stall_pmc.py" "$R/gpurun_out/stall4/mo" scene=$R/gpurun_out/stall4/s800/multi_object.json > "$R/gpurun_out/stall4/mo.txt" 2>&1 || exit 1
cat "$R/gpurun_out/stall4/cornell.txt" "$R/gpurun_out/stall4/mo.txt"
