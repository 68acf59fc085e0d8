# Phase stamps (-DPT_STAMPS library, scripts/stamps_build.sh) for Cornell and config 4's scene.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/stamps
python -c "from cuda_pathtracer_amd import scenes; print(scenes.multi_object('gpurun_out/stamps', res=(1920, 1080)))" > gpurun_out/stamps/mo.txt || exit 1
timeout -k 10 120 python -u scripts/stamps_run.py > gpurun_out/stamps/cornell.txt 2>&1 || exit 1
timeout -k 10 120 python -u scripts/stamps_run.py $(cat gpurun_out/stamps/mo.txt) > gpurun_out/stamps/mo_stamps.txt 2>&1 || exit 1
cat gpurun_out/stamps/cornell.txt gpurun_out/stamps/mo_stamps.txt
