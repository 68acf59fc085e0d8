# Round 3: sorted-pipeline parity (every render test that sorts) + device BVH build parity, then a
# short config-3 bench line.  Each GPU step under its own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bvh_device_gpu.py tests/test_render_gpu.py -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread -k "device_bvh or sort or Sort or material or lanes or config3 or emit" \
    > gpurun_out/sorted_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/sorted_tests.log; exit 1; }
tail -2 gpurun_out/sorted_tests.log
grep -E "nodes;" gpurun_out/sorted_tests.log || true
timeout -k 10 400 python -u bench.py --config cornell_hd_sorted --steps 5 --warmup 1 --no-cpu-baseline --no-scan \
    > gpurun_out/cfg3.json 2> gpurun_out/cfg3.err || { echo "bench failed"; tail -20 gpurun_out/cfg3.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/cfg3.json') if l.startswith('{')][-1]); r=d['roofline']
print('cfg3', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'B/seg', r.get('traffic_per_segment'), 'first', r.get('first_producer_bytes_per_path'))"
