// Image output: saveImage (main.cpp:88-112) + Image::savePNG (image.cpp:22-42).
// The reference writes through stb_image_write 0.98; this writes the same 8-bit RGB pixels as a
// standard PNG (zlib deflate, filter 0 per row).  Pixel bytes are what parity is checked on.
#include <zlib.h>

#include <algorithm>
#include <cmath>
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

// Image::saveHDR (image.cpp:44-49) through stb_image_write's Radiance writer as vendored by the
// reference (external/include/stb_image_write.h:246-387): RGBE pixels (stbiw__linear_to_rgbe)
// with per-channel run-length coding of every scanline 8..32767 pixels wide, restated here.
// Pixels are saveImage's (main.cpp:88-112): x-mirrored, value = accumulated / samples.
namespace {

void to_rgbe(uint8_t* rgbe, const float* lin) {
    const float m = lin[1] > lin[2] ? lin[1] : lin[2];
    const float maxcomp = lin[0] > m ? lin[0] : m;
    if ((double)maxcomp < 1e-32) {
        rgbe[0] = rgbe[1] = rgbe[2] = rgbe[3] = 0;
        return;
    }
    int e = 0;
    const float scale = (float)std::frexp((double)maxcomp, &e) * 256.0f / maxcomp;
    for (int k = 0; k < 3; ++k) rgbe[k] = (uint8_t)(lin[k] * scale);
    rgbe[3] = (uint8_t)(e + 128);
}

// One channel of one scanline: literal dumps (<= 128 bytes, length byte n) up to the next run of
// >= 3 equal bytes, then that run in pieces of <= 127 (length byte 128 + n).
void rle_channel(std::vector<uint8_t>& out, const uint8_t* c, int w) {
    int x = 0;
    while (x < w) {
        int r = x;
        while (r + 2 < w && !(c[r] == c[r + 1] && c[r] == c[r + 2])) ++r;
        const bool run = r + 2 < w;
        if (!run) r = w;
        for (; x < r;) {
            const int n = std::min(r - x, 128);
            out.push_back((uint8_t)n);
            out.insert(out.end(), c + x, c + x + n);
            x += n;
        }
        if (run) {
            const uint8_t v = c[x];
            while (r < w && c[r] == v) ++r;
            for (; x < r;) {
                const int n = std::min(r - x, 127);
                out.push_back((uint8_t)(n + 128));
                out.push_back(v);
                x += n;
            }
        }
    }
}

}  // namespace

int pt_encode_hdr(const float* rgb, int32_t W, int32_t H, float samples, uint8_t* out, int64_t cap, int64_t* size) {
    if (!rgb || W <= 0 || H <= 0 || !size) return pt::fail(PT_ERR_ARG, "bad hdr arguments");
    std::vector<uint8_t> f;
    char head[160];
    const int n = std::snprintf(head, sizeof head,
                                "#?RADIANCE\n# Written by stb_image_write.h\nFORMAT=32-bit_rle_rgbe\n"
                                "EXPOSURE=          1.0000000000000\n\n-Y %d +X %d\n", H, W);
    f.insert(f.end(), head, head + n);
    std::vector<uint8_t> line((size_t)W * 4);
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {   // img.setPixel(width - 1 - x, y, image[x + y*width] / samples)
            const float* p = rgb + 3 * ((size_t)x + (size_t)y * W);
            const float lin[3] = {p[0] / samples, p[1] / samples, p[2] / samples};
            uint8_t e[4];
            to_rgbe(e, lin);
            const int X = W - 1 - x;
            if (W < 8 || W >= 32768) std::memcpy(&line[4 * (size_t)X], e, 4);
            else for (int k = 0; k < 4; ++k) line[(size_t)W * k + X] = e[k];
        }
        if (W < 8 || W >= 32768) {
            f.insert(f.end(), line.begin(), line.end());
        } else {
            const uint8_t hdr[4] = {2, 2, (uint8_t)((W & 0xff00) >> 8), (uint8_t)(W & 0xff)};
            f.insert(f.end(), hdr, hdr + 4);
            for (int k = 0; k < 4; ++k) rle_channel(f, &line[(size_t)W * k], W);
        }
    }
    *size = (int64_t)f.size();
    if (out) {
        if (cap < (int64_t)f.size()) return pt::fail(PT_ERR_ARG, "hdr buffer too small");
        std::memcpy(out, f.data(), f.size());
    }
    return PT_OK;
}

int pt_save_hdr(const char* path, const float* rgb, int32_t W, int32_t H, float samples) {
    if (!path) return pt::fail(PT_ERR_ARG, "null path");
    int64_t n = 0;
    if (int rc = pt_encode_hdr(rgb, W, H, samples, nullptr, 0, &n)) return rc;
    std::vector<uint8_t> buf((size_t)n);
    if (int rc = pt_encode_hdr(rgb, W, H, samples, buf.data(), n, &n)) return rc;
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return pt::fail(PT_ERR_IO, std::string("cannot open ") + path);
    const size_t w = std::fwrite(buf.data(), 1, buf.size(), fp);
    std::fclose(fp);
    if (w != buf.size()) return pt::fail(PT_ERR_IO, "short write");
    return PT_OK;
}

}  // extern "C"
