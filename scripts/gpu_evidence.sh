# Evidence run of the current tree on one GPU box, every GPU step under its own time limit, the chain
# stopping at the first failure (replaces the per-round gpu_r0*.sh launchers):
#   TAG=r06a STEPS="tests bench ktrace configs" bash scripts/gpu_evidence.sh
#   tests   — pytest -m gpu (PYTEST_K selects)
#   bench   — the default bench line (in-run PMC, CPU baselines, scan, drop-in) + its PMC summary
#   ktrace  — rocprofv3 --kernel-trace --stats of the same bench command (no PMC / CPU / drop-in legs)
#             and scripts/union_check.py (the line's frac from the trace and the PMC summary)
#   configs — bench lines of BASELINE configs 3-5 (+ the tessellated workload), with their PMC passes
#   ab      — alternating bench lines of the working tree and build/libpt_amd_$VARIANTS.so (RUNS)
# Outputs under gpurun_out/$TAG; copy what is judged into profiles/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-ev}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
for step in ${STEPS:-tests bench ktrace}; do
  case $step in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
        ${PYTEST_K:+-k "$PYTEST_K"} > "$O/pytest_gpu.log" 2>&1; rc=$?
    echo "pytest rc=$rc"; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit 1 ;;
  bench)
    timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.log"; rc=$?
    echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$O/bench.log"; exit 1; }
    cp gpurun_out/bench_pmc/summary.json "$O/bench_pmc_summary.json" 2>/dev/null
    python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print('bench', round(d['value'],1), d['unit'], round(d['ms_per_step'],3), 'ms/step; bound', r['bound'], 'frac', round(r['frac'],4), r['unit'])
print('  hbm', {k: round(v['frac'],3) for k, v in r.get('hbm', {}).items() if isinstance(v, dict)}, 'valu/seg', r.get('valu_issue', {}).get('instructions_per_segment'))
print('  dropin', d.get('dropin', {}).get('value'), 'scan GB/s', d.get('scan', {}).get('GB/s'), 'cpu', d.get('cpu_baseline', {}).get('value'))" ;;
  ktrace)
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktrace" -o run -- \
        python3 "$R/bench.py" --no-pmc --no-cpu-baseline --no-dropin --steps 20 ${BENCH_ARGS:-} > "$O/ktrace_bench.json" 2> "$O/ktrace_bench.log" ); rc=$?
    echo "ktrace rc=$rc"; [ $rc -eq 0 ] || exit 1
    find "$O/ktrace" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
    head -8 "$O/kernel_stats.csv"
    if [ -f "$O/bench.json" ] && [ -f "$O/bench_pmc_summary.json" ]; then
      python3 scripts/union_check.py "$(find "$O/ktrace" -name '*kernel_trace.csv' | head -1)" "$O/bench.json" \
          "$O/bench_pmc_summary.json" | tee "$O/union_check.txt"
    fi ;;
  configs)
    : > "$O/configs.jsonl"
    for c in "cornell_hd_sorted --steps 10" "multi_object_4k --steps 5" "random_triangles_100k --steps 2" \
             "tessellated_meshes_100k --steps 3"; do
      set -- $c
      timeout -k 10 400 python bench.py --config $c --warmup 2 --no-cpu-baseline --no-scan \
          >> "$O/configs.jsonl" 2> "$O/config_$1.err" || { echo "config $1 failed"; tail -5 "$O/config_$1.err"; exit 1; }
      cp gpurun_out/bench_pmc/summary.json "$O/pmc_$1.json" 2>/dev/null
    done
    python3 -c "
import json
for l in open('$O/configs.jsonl'):
    d = json.loads(l); r = d['roofline']
    print(d['config']['workload'][:50], '|', round(d['value'], 1), '| ms/step', round(d['ms_per_step'], 2), '| bound', r['bound'], 'frac', round(r['frac'], 3), '| B/seg', r.get('traffic_per_segment'))" ;;
  ab)
    for k in $(seq 1 ${RUNS:-3}); do
      for v in new ${VARIANTS:-base}; do
        if [ $v = new ]; then unset PT_AMD_LIB; else export PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_$v.so; fi
        timeout -k 10 300 python -u bench.py --steps ${AB_STEPS:-20} --warmup 3 --no-cpu-baseline --no-scan --no-pmc --no-dropin ${BENCH_ARGS:-} \
            > "$O/ab_${v}_$k.json" 2> "$O/ab_${v}_$k.err" || { echo "bench $v failed"; tail -5 "$O/ab_${v}_$k.err"; exit 1; }
        python3 -c "import json;d=json.load(open('$O/ab_${v}_$k.json'));r=d['roofline'];print('$v', round(d['value'],1), round(d['ms_per_step'],3), 'eff', round(r['effective_launch_ms']*1e3,1), 'us; first', round(d.get('first_bounce_avg_ms',0)*1e3,1))"
      done
    done
    unset PT_AMD_LIB ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
