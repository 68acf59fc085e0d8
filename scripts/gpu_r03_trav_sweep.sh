# Round 3: k_traverse4 knobs on config 5 (refill threshold, LDS stack rows), then one bench line
# with the in-run PMC (VALU, SALU, VMEM, L2, wave states) for each walk.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/trav3s; mkdir -p $O
bench() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --config random_triangles_100k --steps ${STEPS:-3} --warmup 1 \
      --no-cpu-baseline --no-scan --no-pmc --no-walk-counters > $O/b_$name.json 2> $O/b_$name.err || { echo "bench $name failed"; tail -3 $O/b_$name.err; return 1; }
  python -c "import json;d=json.load(open('$O/b_$name.json'));r=d['roofline'];print('$name', round(d['value'],1), round(d['ms_per_step'],1), 'ms/step', r.get('kernel'), round(r.get('avg_launch_ms',0),3))"
}
for cfg in ${CFGS:-"refill4 PT_AMD_REFILL=4" "refill8 PT_AMD_REFILL=8" "refill32 PT_AMD_REFILL=32" "rows8 PT_AMD_STACK_ROWS=8" "rows24 PT_AMD_STACK_ROWS=24" "base PT_X=0"}; do
  set -- $cfg
  bench "$@" || exit 1
done
if [ "${PMC:-1}" = 1 ]; then
  for walk in quad pairs; do
    if [ $walk = pairs ]; then export PT_AMD_TRAV=pairs; else unset PT_AMD_TRAV; fi
    timeout -k 10 900 python -u bench.py --config random_triangles_100k --steps 3 --warmup 1 --no-cpu-baseline --no-scan \
        --pmc-passes 1 --pmc-timeout 200 > $O/pmc_$walk.json 2> $O/pmc_$walk.err || { echo "pmc bench failed"; tail -3 $O/pmc_$walk.err; exit 1; }
    python - <<EOF
import json
d = json.load(open("$O/pmc_$walk.json")); r = d["roofline"]
v = r.get("valu_issue", {})
print("$walk", round(d["value"], 1), "valu/seg", round(v.get("instructions_per_segment", 0), 1), "frac", round(v.get("frac", 0), 3),
      "salu/seg", round(r.get("salu_per_segment", 0), 1), "vmem/seg", round(r.get("vmem_rd_per_segment", 0), 1),
      "l2", round(r.get("l2_hit_rate", 0), 3), "waves", r.get("wave_states"), "walk", r.get("walk_counters"))
EOF
  done
fi
