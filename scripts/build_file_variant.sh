# A variant library built from another version of pt_kernels.hip (e.g. git HEAD) for A/B runs:
#   scripts/build_file_variant.sh NAME FILE [extra hipcc flags]  -> cuda_pathtracer_amd/build/libpt_amd_NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/cuda_pathtracer_amd/build
name=$1; src=$2; shift 2
python -c "import sys; sys.path.insert(0, '$R'); from cuda_pathtracer_amd import build; build.build_native()"
tmp=$R/cuda_pathtracer_amd/csrc/_variant_$name.hip
cp "$src" "$tmp"
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize "$@" -I $R/include \
    -c "$tmp" -o $B/pt_kernels_$name.o || { rm -f "$tmp"; exit 1; }
rm -f "$tmp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $B/libpt_amd_$name.so $B/pt_kernels_$name.o \
    $B/sc_kernels.hip.o $B/sc_variants.hip.o $B/bvh_build.hip.o $B/pt_scene.cpp.o $B/pt_mesh.cpp.o $B/pt_image.cpp.o $B/pt_jpeg.cpp.o -lz
echo $B/libpt_amd_$name.so
