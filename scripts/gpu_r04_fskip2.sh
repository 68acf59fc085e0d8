# The fused first bounce's empty-wave instantiation chosen per context (share of empty camera-mask
# blocks >= 0.2): mask parity tests, the choice on the bench workloads, then Cornell and config 4
# A/B against the same build with the fused skip forced off (PT_AMD_SKIP_EMPTY=0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/fskip2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 600 --timeout-method thread -k "mask or skip or first" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 - <<'PY' || exit 1
import sys, tempfile
sys.path.insert(0, ".")
import cuda_pathtracer_amd as P
from cuda_pathtracer_amd import scenes
d = tempfile.mkdtemp()
for name, path in [("cornell 800x800", "tests/scenes/cornell.json"), ("config 3 1920x1080", scenes.cornell_hd(d)),
                   ("config 4 3840x2160", scenes.multi_object(d))]:
    s = P.Scene(path)
    pt = P.PathTracer(s, P.GuiDataContainer(), spp=2)
    print(name, pt.cmask_info(), flush=True)
    pt.free()
PY
VARIANTS="auto: off:PT_AMD_SKIP_EMPTY=0" RUNS=2 STEPS=5 BENCH_ARGS="--config multi_object_4k" bash scripts/gpu_ab_env.sh || exit 1
