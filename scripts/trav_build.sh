# Diagnostic library with k_traverse counters (-DPT_TRAV_STATS), built on the CPU next to the
# product library: cuda_pathtracer_amd/build/libpt_amd_trav.so (dev tool only).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/cuda_pathtracer_amd/build
python -c "import sys; sys.path.insert(0, '$R'); from cuda_pathtracer_amd import build; build.build_native()"
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -DPT_TRAV_STATS -I $R/include \
    -c $R/cuda_pathtracer_amd/csrc/pt_kernels.hip -o $B/pt_kernels_trav.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $B/libpt_amd_trav.so $B/pt_kernels_trav.o \
    $B/sc_kernels.hip.o $B/sc_variants.hip.o $B/bvh_build.hip.o $B/pt_scene.cpp.o $B/pt_mesh.cpp.o $B/pt_image.cpp.o $B/pt_jpeg.cpp.o -lz
echo $B/libpt_amd_trav.so
