# Config 4: two vs three lanes (alternating), each run under its own limit.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/cfg4lanes
O=gpurun_out/cfg4lanes
for k in 1 2; do
  for L in 2 3; do
    PT_AMD_LANES=$L timeout -k 10 240 python -u bench.py --config multi_object_4k --steps 3 --warmup 1 \
        --no-cpu-baseline --no-scan --no-pmc > $O/l${L}_$k.json 2> $O/l${L}_$k.err || { echo "lanes $L failed"; tail -3 $O/l${L}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('$O/l${L}_$k.json'));print('lanes', $L, round(d['value'],1), round(d['ms_per_step'],2))"
  done
done
