# Timing ablations of the bounce kernel (results intentionally wrong in ablated modes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/ablate"
cd /tmp && export TMPDIR=/tmp
for ex in ${EXPERIMENTS:-0}; do
  PT_EXPERIMENT=$ex timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/ablate/e$ex" -o run -- \
      python3 "$R/scripts/prof_render.py" 10 > "$R/gpurun_out/ablate/e$ex.log" 2>&1 || { echo "ablation $ex failed"; tail -5 "$R/gpurun_out/ablate/e$ex.log"; exit 1; }
done
echo done
