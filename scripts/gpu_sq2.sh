# Second SQ counter group for the render kernels: instruction mix by type and LDS stalls.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/sq2"
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAVES --output-format csv -d "$OUT" -o run -- \
    python3 "$R/scripts/prof_render.py" 10 > "$OUT/render.log" 2>&1 \
    || { echo "render SQ2 pass failed"; tail -5 "$OUT/render.log"; exit 1; }
python3 "$R/scripts/sq_summary.py" "$OUT" | tee "$OUT/summary.txt"
