# Config 3 (material-sorted) sweep: lanes x iterations per pass, each run under its own limit.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/cfg3sweep
O=gpurun_out/cfg3sweep
for spp in 64 128; do
  for L in 2 3 4; do
    PT_AMD_LANES=$L timeout -k 10 200 python -u bench.py --config cornell_hd_sorted --spp $spp --steps 4 --warmup 1 \
        --no-cpu-baseline --no-scan --no-pmc > $O/s${spp}_l$L.json 2> $O/s${spp}_l$L.err || { echo "spp $spp lanes $L failed"; tail -3 $O/s${spp}_l$L.err; exit 1; }
    python -c "import json;d=json.load(open('$O/s${spp}_l$L.json'));print('spp', $spp, 'lanes', $L, round(d['value'],1), round(d['ms_per_step'],2))"
  done
done
