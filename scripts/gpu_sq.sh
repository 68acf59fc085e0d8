# Wave-state breakdown of the render kernels from SQ PMC counters (one rocprofv3 pass, --kernel-trace
# only): WAVE_CYCLES = ACTIVE_INST_ANY + WAIT_INST_ANY + WAIT_ANY (MI355X_MICROARCH.md "rocprofv3
# PMC slots"), plus VALU activity and instruction counts.  Workload: scripts/prof_render.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/sq${SQ_TAG:+_$SQ_TAG}"
rm -rf "$OUT"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU --output-format csv -d "$OUT" -o run -- \
    python3 "$R/scripts/prof_render.py" 10 ${SQ_ARGS:-} > "$OUT/render.log" 2>&1 \
    || { echo "render SQ pass failed"; tail -5 "$OUT/render.log"; exit 1; }
python3 "$R/scripts/sq_summary.py" "$OUT" | tee "$OUT/summary.txt"
