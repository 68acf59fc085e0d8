# Two variants in one call: paired walk tasks (config 5 parity + A/B) and FMA-form world-box bounds
# (the bounded-hit verification and Cornell A/B with in-run VALU counts).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05d; mkdir -p $O
V=pairs bash scripts/gpu_walk_variant.sh || exit 1
PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_bfma.so timeout -k 10 600 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_bfma.log 2>&1; rc=$?
echo "bfma tests rc=$rc"; tail -2 $O/tests_bfma.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests_bfma.log | head; exit 1; }
for k in 1 2; do
  for v in new bfma; do
    if [ $v = new ]; then unset PT_AMD_LIB; else export PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_$v.so; fi
    timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-scan --no-dropin --pmc-passes 3 \
        > $O/b_${v}_$k.json 2> $O/b_${v}_$k.err || { echo "bench $v failed"; tail -5 $O/b_${v}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${v}_$k.json'));r=d['roofline'];u=r.get('valu_issue',{});print('$v', round(d['value'],1), round(d['ms_per_step'],3), 'valu/seg', round(u.get('instructions_per_segment',0),3), 'iso', round(r.get('isolated',{}).get('avg_launch_ms',0)*1e3,1))"
  done
done
