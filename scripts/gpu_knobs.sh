# Runtime-knob sweep of the Cornell bench on one box: lanes (PT_AMD_LANES) and iterations per pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/knobs
O=gpurun_out/knobs
run() {   # tag, env, args
  env $2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-scan --no-pmc $3 ${BENCH_ARGS:-} > $O/$1.json 2> $O/$1.err \
      || { echo "$1 failed"; tail -3 $O/$1.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1', round(d['value'],1), round(d['ms_per_step'],3))"
}
for k in 1 2; do
  for L in ${LANES:-2 3 4}; do run lanes${L}_$k "PT_AMD_LANES=$L" "" || exit 1; done
done
