# A/B helper: build the committed (HEAD, or $REV) pt_kernels.hip as build/libpt_amd_ab.so next to the
# working-tree library, so one GPU call can time both (PT_AMD_LIB selects the library).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/cuda_pathtracer_amd/build
mkdir -p $B/ab
git -C $R show ${REV:-HEAD}:cuda_pathtracer_amd/csrc/pt_kernels.hip > $B/ab/pt_kernels.hip
cp $R/cuda_pathtracer_amd/csrc/*.h $B/ab/
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -I $R/include -I $R/cuda_pathtracer_amd/csrc \
    -c $B/ab/pt_kernels.hip -o $B/ab/pt_kernels.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $B/libpt_amd_ab.so $B/ab/pt_kernels.o \
    $B/sc_kernels.hip.o $B/sc_variants.hip.o $B/bvh_build.hip.o $B/pt_scene.cpp.o $B/pt_mesh.cpp.o $B/pt_image.cpp.o $B/pt_jpeg.cpp.o -lz
echo $B/libpt_amd_ab.so
