# A/B helper: build the working-tree pt_kernels.hip with extra compiler flags ($FLAGS) as
# build/libpt_amd_${NAME:-ab}.so (timed beside the product library by scripts/gpu_ab_lib.sh).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/cuda_pathtracer_amd/build
N=${NAME:-ab}
mkdir -p $B/$N
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $FLAGS -I $R/include \
    -c $R/cuda_pathtracer_amd/csrc/pt_kernels.hip -o $B/$N/pt_kernels.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $B/libpt_amd_$N.so $B/$N/pt_kernels.o \
    $B/sc_kernels.hip.o $B/bvh_build.hip.o $B/pt_scene.cpp.o $B/pt_mesh.cpp.o $B/pt_image.cpp.o $B/pt_jpeg.cpp.o -lz
echo $B/libpt_amd_$N.so
