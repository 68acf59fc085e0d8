# Bench lines for BASELINE.json configs 3-5 (1 GPU), each under its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
for c in ${CONFIGS:-cornell_hd_sorted multi_object_4k random_triangles_100k}; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-scan \
      >> gpurun_out/configs.jsonl 2> gpurun_out/config_$c.err || { echo "config $c failed"; tail -5 gpurun_out/config_$c.err; exit 1; }
  echo "config $c ok"
done
python3 - <<'PY'
import json
for line in open("gpurun_out/configs.jsonl"):
    d = json.loads(line)
    print(d["config"]["workload"][:60], "|", round(d["value"], 1), d["unit"], "| ms/step", round(d["ms_per_step"], 2),
          "| frac", round(d["roofline"]["frac"], 3))
PY
