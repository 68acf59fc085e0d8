# Config 3: iterations per pass 128 vs 256 (alternating, default lanes), each run under its own limit.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/cfg3spp
O=gpurun_out/cfg3spp
for k in 1 2; do
  for spp in ${SPPS:-128 256}; do
    timeout -k 10 240 python -u bench.py --config cornell_hd_sorted --spp $spp --steps 4 --warmup 1 \
        --no-cpu-baseline --no-scan --no-pmc > $O/s${spp}_$k.json 2> $O/s${spp}_$k.err || { echo "spp $spp failed"; tail -3 $O/s${spp}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('$O/s${spp}_$k.json'));print('spp', $spp, round(d['value'],1), round(d['ms_per_step'],2))"
  done
done
