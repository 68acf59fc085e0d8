# k_bounce's early exit of idle workgroups + GPU-ordered image copy: render parity subset, then the
# Cornell bench (with the drop-in leg) alternating the working tree and HEAD (build_ab.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_render_gpu.py tests/test_cpp_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit 1; }
for k in 1 2; do
  for v in new ab; do
    if [ $v = new ]; then unset PT_AMD_LIB; DI=""; else export PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_ab.so; DI="--no-dropin"; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-scan --no-pmc $DI \
        > $O/b_${v}_$k.json 2> $O/b_${v}_$k.err || { echo "bench $v failed"; tail -5 $O/b_${v}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${v}_$k.json'));r=d['roofline'];print('$v', round(d['value'],1), round(d['ms_per_step'],3), 'later eff', round(r['effective_launch_ms']*1e3,1), 'avg', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],3), 'dropin', d.get('dropin',{}).get('value'), d.get('dropin',{}).get('ms_per_call'))"
  done
done
