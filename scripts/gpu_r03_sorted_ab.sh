# Sorted-pipeline parity, then alternating config-3 runs of the working tree and variant libraries.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
bash scripts/gpu_r03_sorted.sh || exit 1
python3 scripts/kernel_totals.py gpurun_out/bench_pmc/fetch/run_kernel_trace.csv
VARIANTS="${VARIANTS:-w6 w6b}" BENCH_ARGS="--config cornell_hd_sorted" RUNS=2 bash scripts/gpu_ab_variants.sh
