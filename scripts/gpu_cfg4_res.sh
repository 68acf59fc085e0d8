# Config 4's scene at Cornell's resolution vs 4K and at fewer iterations per pass: is the
# per-segment rate set by the scene or by the pass's memory footprint?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/c4/s800 gpurun_out/c4/s4k
python -c "from cuda_pathtracer_amd import scenes; scenes.multi_object('gpurun_out/c4/s800', res=(800, 800)); scenes.multi_object('gpurun_out/c4/s4k')" || exit 1
: > gpurun_out/c4/lines.jsonl
run() {   # label, scene, extra
  timeout -k 10 240 python bench.py --scene $2 --warmup 1 --no-cpu-baseline --no-scan --no-pmc ${@:3} \
      >> gpurun_out/c4/lines.jsonl 2> gpurun_out/c4/$1.err || { echo "$1 failed"; tail -5 gpurun_out/c4/$1.err; exit 1; }
  python3 -c "import json;d=[json.loads(l) for l in open('gpurun_out/c4/lines.jsonl')][-1];r=d['roofline'];print('$1', round(d['value'],1), 'k_bounce', round(r['avg_launch_ms']*1e3,1), 'us', round(r['segments_per_launch']/1e6,2), 'M seg/launch')"
}
run s800_spp32 gpurun_out/c4/s800/multi_object.json --steps 10 --samples 256 || exit 1
run s4k_spp32 gpurun_out/c4/s4k/multi_object.json --steps 2 --samples 64 || exit 1
run s4k_spp8 gpurun_out/c4/s4k/multi_object.json --steps 2 --samples 64 --spp 8 || exit 1
run s4k_spp4 gpurun_out/c4/s4k/multi_object.json --steps 2 --samples 64 --spp 4 || exit 1
