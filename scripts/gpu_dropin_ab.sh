# Drop-in call components under the A/B knobs (scripts/dropin_probe.py), alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/dropin_ab; mkdir -p $O
for k in 1 2; do
  for v in "new" "PT_AMD_COPY_HOSTWAIT=1" "PT_AMD_NO_EARLY_EXIT=1" "PT_AMD_COPY_HOSTWAIT=1 PT_AMD_NO_EARLY_EXIT=1" "PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_ab.so"; do
    echo "== $v"; env ${v/new/X=1} timeout -k 10 120 python -u scripts/dropin_probe.py 2>&1 | tail -1 || exit 1
  done
done
