# PMC counter passes (one counter group per rocprofv3 run; --kernel-trace only, no sys/runtime trace).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$R/gpurun_out/pmc/counters.txt" 2>&1 || true
i=0
for grp in "${PMC_GROUPS[@]:-}"; do :; done
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$R/gpurun_out/pmc/g$i" -o run -- \
      python3 "$R/scripts/prof_render.py" ${PROF_ARGS:-10} > "$R/gpurun_out/pmc/g$i.log" 2>&1 || { echo "pmc group $i failed"; tail -5 "$R/gpurun_out/pmc/g$i.log"; exit 1; }
  echo "group $i ok: $grp"
done < "$R/scripts/pmc_groups.txt"
