# Late round-4 evidence of the current tree: GPU suite + bench + kernel trace (gpu_r04.sh), the
# config lines (gpu_r04_configs.sh), then config 3's per-kernel breakdown (gpu_r03_cfg3_prof.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${TAG:-r04c} bash scripts/gpu_r04.sh || exit 1
cd "$R" && bash scripts/gpu_r04_configs.sh || exit 1
cd "$R" && bash scripts/gpu_r03_cfg3_prof.sh || exit 1
