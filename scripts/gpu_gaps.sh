# Kernel-to-kernel gaps within one lane: rocprofv3 kernel trace of the render-only workload
# (no HIP profiling events) vs the bench's command (events around every bounce).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/gaps; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/render -o run -- python3 $R/scripts/prof_render.py 6 > $O/render.log 2>&1 || { tail -5 $O/render.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/bench -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-scan --no-cpu-baseline --no-pmc > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python3 $R/scripts/gaps.py $O/render $O/bench
