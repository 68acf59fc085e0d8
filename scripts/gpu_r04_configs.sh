# Bench lines for BASELINE.json configs 3-5 (1 GPU), each under its own time limit.
# Iterations per pass: the bench defaults (256 for config 3, 128 for configs 4 and 5); plus the tessellated-mesh workload (not a BASELINE config).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
run() {   # name, extra args
  timeout -k 10 300 python bench.py --config $1 --warmup 2 --no-cpu-baseline --no-scan ${@:2} \
      >> gpurun_out/configs.jsonl 2> gpurun_out/config_$1.err || { echo "config $1 failed"; tail -5 gpurun_out/config_$1.err; exit 1; }
  echo "config $1 ${@:2} ok"
}
run cornell_hd_sorted --steps 10 || exit 1
run multi_object_4k --steps 5 || exit 1
run random_triangles_100k --steps 2 --spp 128 --samples 128 || exit 1
run tessellated_meshes_100k --steps 3 --spp 128 --samples 128 || exit 1
python3 - <<'PY'
import json
for line in open("gpurun_out/configs.jsonl"):
    d = json.loads(line)
    print(d["config"]["workload"][:60], "|", round(d["value"], 1), d["unit"],
          "| ms/step", round(d["ms_per_step"], 2), "| frac", round(d["roofline"]["frac"], 3))
PY
