# Host-only AddressSanitizer + UBSan fuzz of pt_decode_jpeg (cuda_pathtracer_amd/csrc/pt_jpeg.cpp):
# byte-mutated copies (overwrites, deletions, insertions, truncations) of a JPEG, N per seed.
#   scripts/fuzz/jpeg_asan.sh file.jpg [seeds] [n]
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
O=${TMPDIR:-/tmp}/pt_jpeg_asan
g++ -O1 -g -std=c++17 -fsanitize=address,undefined -fno-sanitize-recover=all -I "$R/include" -I "$R/cuda_pathtracer_amd/csrc" \
    "$R/scripts/fuzz/jpeg_asan_main.cpp" "$R/cuda_pathtracer_amd/csrc/pt_jpeg.cpp" -o "$O"
for s in $(seq 1 ${2:-3}); do "$O" "$1" "$s" "${3:-300}"; done
