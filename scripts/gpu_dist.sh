# Distributed GPU tests + a bench line with its in-run PMC leg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/dist
O=gpurun_out/dist
timeout -k 10 400 python -u -m pytest tests/test_distributed_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -6 $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u bench.py --steps 20 --no-cpu-baseline --no-scan > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python -c "
import json;d=json.load(open('$O/bench.json'));r=d['roofline']
print(round(d['value'],1), 'bound', r['bound'], 'frac', round(r['frac'],3), 'traffic/seg', r.get('traffic_per_segment'), 'valu/seg', r.get('valu_issue',{}).get('instructions_per_segment'), 'valu frac', r.get('valu_issue',{}).get('frac'), r.get('wave_states'))"
