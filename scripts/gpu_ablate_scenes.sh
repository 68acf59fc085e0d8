set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/abl
python scripts/ablate_scenes.py gpurun_out/abl
for v in base nosphere diffsphere noceiling; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-scan --steps 100 --scene gpurun_out/abl/$v.json > gpurun_out/abl/$v.out 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abl/$v.out'));r=d['roofline'];print('$v',round(d['value'],1),'bounce_ms',round(r['avg_launch_ms'],4),'first_ms',round(d['first_bounce_avg_ms'],4),'live',[round(x) for x in d['bounce_live_per_pass']])"
done
