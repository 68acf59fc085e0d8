# Config 3's camera-ray producer: where its time goes, by ablation (timing only, not bit-exact):
# abl1 = no closest hit (every camera ray misses), abl2 = one material key (one ballot round),
# abl3 = both.  Isolated per-launch durations from the bench's in-run PMC passes (dispatches
# serialised), per library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O="$R/gpurun_out/prodabl"; mkdir -p "$O"
for v in ${VARS:-new abl1 abl2 abl3}; do
  if [ $v = new ]; then unset PT_AMD_LIB; else export PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_$v.so; fi
  timeout -k 10 400 python3 bench.py --config cornell_hd_sorted --steps 3 --warmup 1 --no-cpu-baseline --no-scan \
      --no-walk-counters --no-dropin > "$O/$v.json" 2> "$O/$v.err" || { echo "$v failed"; tail -5 "$O/$v.err"; exit 1; }
  cp gpurun_out/bench_pmc/summary.json "$O/$v.pmc.json"
  echo "== $v"; python3 - "$O/$v.pmc.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    if "produce" in k or "hist" in k:
        w = v["SQ_WAVES"]
        print(f"{k[:44]:44s} {v['launches']:4d} x {v['dur_ns_sq']/1e3:8.1f} us  VALU/wave {v['SQ_INSTS_VALU']/w:9.0f}  MB {v['bytes_per_launch']/1e6:8.1f}")
PY
done
