// Host-only harness for scripts/fuzz/jpeg_asan.sh (not part of the product or the tests).
// ASan harness: byte-mutated copies of a JPEG through pt_decode_jpeg (host code only).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>
#include "pt_amd.h"
namespace pt { thread_local std::string g_err; int fail(int code, const std::string& m) { g_err = m; return code; } }
int main(int argc, char** argv) {
    FILE* f = std::fopen(argv[1], "rb");
    std::vector<uint8_t> src;
    int ch;
    while ((ch = std::fgetc(f)) != EOF) src.push_back((uint8_t)ch);
    std::fclose(f);
    std::mt19937 rng(std::atoi(argv[2]));
    const int n = std::atoi(argv[3]);
    std::vector<uint8_t> out(64u << 20);
    for (int i = 0; i < n; ++i) {
        std::vector<uint8_t> b = src;
        const int muts = 1 + (int)(rng() % 12);
        for (int m = 0; m < muts && !b.empty(); ++m) {
            const size_t k = rng() % b.size();
            const unsigned r = rng() % 10;
            if (r < 6) b[k] = (uint8_t)rng();
            else if (r < 8) b.erase(b.begin() + (long)k, b.begin() + (long)std::min(b.size(), k + 1 + rng() % 64));
            else b.insert(b.begin() + (long)k, (size_t)(1 + rng() % 16), (uint8_t)rng());
        }
        if (rng() % 5 == 0 && !b.empty()) b.resize(rng() % b.size());
        int32_t w, h, c;
        pt_decode_jpeg(b.data(), (int64_t)b.size(), &w, &h, &c, out.data(), (int64_t)out.size());
    }
    std::printf("ok %d\n", n);
    return 0;
}
