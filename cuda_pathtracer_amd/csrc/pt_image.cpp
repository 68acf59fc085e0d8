// Image output: saveImage (main.cpp:88-112) + Image::savePNG (image.cpp:22-42).
// The reference writes through stb_image_write 0.98; this writes the same 8-bit RGB pixels as a
// standard PNG (zlib deflate, filter 0 per row).  Pixel bytes are what parity is checked on.
#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "pt_internal.h"

namespace {

void put_u32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24));
    v.push_back((uint8_t)(x >> 16));
    v.push_back((uint8_t)(x >> 8));
    v.push_back((uint8_t)x);
}

void chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
    put_u32(out, (uint32_t)data.size());
    const size_t start = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    const uint32_t crc = (uint32_t)crc32(0L, out.data() + start, (uInt)(out.size() - start));
    put_u32(out, crc);
}

}  // namespace

extern "C" {

int pt_tonemap(const float* rgb, int32_t W, int32_t H, float samples, uint8_t* out) {
    if (!rgb || !out || W <= 0 || H <= 0) return pt::fail(PT_ERR_ARG, "bad tonemap arguments");
    for (int x = 0; x < W; ++x)
        for (int y = 0; y < H; ++y) {
            const float* p = rgb + 3 * ((size_t)x + (size_t)y * W);
            uint8_t* o = out + 3 * ((size_t)y * W + (size_t)(W - 1 - x));   // img.setPixel(width-1-x, y, ...)
            for (int k = 0; k < 3; ++k) {
                float v = p[k] / samples;
                v = v > 0.0f ? v : 0.0f;           // glm::clamp = min(max(x, 0), 1)
                v = v < 1.0f ? v : 1.0f;
                o[k] = (uint8_t)(v * 255.f);
            }
        }
    return PT_OK;
}

int pt_save_png(const char* path, const float* rgb, int32_t W, int32_t H, float samples) {
    if (!path) return pt::fail(PT_ERR_ARG, "null path");
    std::vector<uint8_t> px((size_t)W * H * 3);
    int rc = pt_tonemap(rgb, W, H, samples, px.data());
    if (rc) return rc;
    std::vector<uint8_t> raw;
    raw.reserve((size_t)H * (W * 3 + 1));
    for (int y = 0; y < H; ++y) {
        raw.push_back(0);
        raw.insert(raw.end(), px.begin() + (size_t)y * W * 3, px.begin() + (size_t)(y + 1) * W * 3);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK)
        return pt::fail(PT_ERR_IO, "zlib compress failed");
    z.resize(zlen);
    std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> ihdr;
    put_u32(ihdr, (uint32_t)W);
    put_u32(ihdr, (uint32_t)H);
    ihdr.push_back(8);   // bit depth
    ihdr.push_back(2);   // colour type RGB
    ihdr.push_back(0);
    ihdr.push_back(0);
    ihdr.push_back(0);
    chunk(png, "IHDR", ihdr);
    chunk(png, "IDAT", z);
    chunk(png, "IEND", {});
    FILE* f = std::fopen(path, "wb");
    if (!f) return pt::fail(PT_ERR_IO, std::string("cannot open ") + path);
    const size_t w = std::fwrite(png.data(), 1, png.size(), f);
    std::fclose(f);
    if (w != png.size()) return pt::fail(PT_ERR_IO, "short write");
    return PT_OK;
}

}  // extern "C"
