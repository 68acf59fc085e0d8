# Variant libraries of the working tree's pt_kernels.hip for A/B runs on one GPU box:
#   VARIANTS="name:-DX=1,-DY=2 name2:-DZ=0" scripts/build_variants.sh
# -> cuda_pathtracer_amd/build/libpt_amd_<name>.so (PT_AMD_LIB selects one; scripts/gpu_ab_variants.sh).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/cuda_pathtracer_amd/build
python -c "import sys; sys.path.insert(0, '$R'); from cuda_pathtracer_amd import build; build.build_native()"
for v in $VARIANTS; do
  name=${v%%:*}; flags=$(echo ${v#*:} | tr ',' ' ')
  /opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize $flags -I $R/include \
      -c $R/cuda_pathtracer_amd/csrc/pt_kernels.hip -o $B/pt_kernels_$name.o &
  pids="$pids $!"
done
for p in $pids; do wait $p || { echo "variant compile failed" >&2; exit 1; }; done
for v in $VARIANTS; do
  name=${v%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $B/libpt_amd_$name.so $B/pt_kernels_$name.o \
      $B/sc_kernels.hip.o $B/sc_variants.hip.o $B/bvh_build.hip.o $B/pt_scene.cpp.o $B/pt_mesh.cpp.o $B/pt_image.cpp.o $B/pt_jpeg.cpp.o -lz
  echo $B/libpt_amd_$name.so
done
