// JPEG decoding of scene textures, natively in the host library.
//
// The reference loads every TEXTURE_FILE with stbi_load(file, &w, &h, &comp, 0)
// (Texture::load, path_tracer/src/sceneStructs.h:171-175; called from scene.cpp:61-71, which
// exits on failure).  The decoder is stb_image 2.06, vendored at
// path_tracer/external/include/stb_image.h.  This file restates that decoder's arithmetic, so
// texels are the reference's byte for byte:
//   * markers, DQT (8-bit tables only), DHT, DRI, SOF0/1/2, SOS:      stb_image.h:2579-2831
//   * canonical Huffman codes and their decoding:                    :1499-1538, :1588-1635
//   * the bit buffer, incl. zero fill after a marker in the stream:  :1567-1582
//   * receive + extend, baseline block decode with in-block dequant: :1642-1747
//   * progressive DC / AC scans (first and refinement passes):       :1749-1893, :2553-2577
//   * integer IDCT (jidctint-derived, 12-bit constants, 2 extra bits after the column pass):
//     :1906-2004 — the SSE2 IDCT stb selects on x86 is bit-identical by construction (:2006-2012)
//   * upsampling: h2v2 triangle filter (:2889-2911; its SSE2 version computes the same sums),
//     h2 (:2859-2885), v2 (:2849-2857), nearest for other ratios (:3030-3039), and the
//     near/far row pairing of load_jpeg_image (:3328-3362)
//   * YCbCr -> RGB: the reduced-precision fixed point (:3070-3096).  With req_comp = 0 the
//     output has 3 channels (step 3), which stb converts with this scalar routine (its SIMD
//     converter handles step 4 only, :3104-3108).
// Only JPEG is handled (the reference's scenes ship JPEG textures); other formats fail loudly.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "pt_internal.h"

namespace pt {
namespace {

// Natural (row-major) position of zigzag index k; corrupt streams may run 15 past the end.
const uint8_t kNatural[64 + 15] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

constexpr int kNoMarker = 0xff;

struct Huff {
    uint8_t values[256];
    uint8_t size[257];
    uint32_t maxcode[18];   // one past the last code of each length, left-aligned to 16 bits
    int delta[17];          // symbol index - code, per length
    int nsym;               // symbols defined (values[0 .. nsym))
    bool defined;           // set by a DHT segment; a scan that names an undefined table fails
};

// Canonical code assignment (JPEG Annex C): lengths in symbol order, codes counting up.
bool build_huff(Huff& h, const int count[16]) {
    int k = 0;
    for (int len = 1; len <= 16; ++len)
        for (int j = 0; j < count[len - 1]; ++j) {
            if (k >= 256) return false;
            h.size[k++] = (uint8_t)len;
        }
    h.size[k] = 0;
    int code = 0, s = 0;
    for (int len = 1; len <= 16; ++len) {
        h.delta[len] = s - code;
        const int first = s;
        while (h.size[s] == len) { ++s; ++code; }
        if (s > first && code - 1 >= (1 << len)) return false;
        h.maxcode[len] = (uint32_t)code << (16 - len);
        code <<= 1;
    }
    h.maxcode[17] = 0xffffffffu;
    h.nsym = k;
    return true;
}

struct Comp {
    int id = 0, h = 1, v = 1, tq = 0, hd = 0, ha = 0, dc_pred = 0;
    int x = 0, y = 0, w2 = 0, h2 = 0;
    std::vector<uint8_t> data;     // w2 x h2 samples
    std::vector<int16_t> coeff;    // progressive: coeff_w x coeff_h blocks of 64
    int coeff_w = 0, coeff_h = 0;
};

uint8_t clamp255(int x) { return (uint8_t)(x < 0 ? 0 : (x > 255 ? 255 : x)); }

struct Decoder {
    const uint8_t* p = nullptr;
    const uint8_t* end = nullptr;
    std::string err;

    Huff huff_dc[4]{}, huff_ac[4]{};   // value-initialised: `defined` false until a DHT sets it
    uint8_t dequant[4][64] = {};
    int img_x = 0, img_y = 0, img_n = 0;
    int h_max = 1, v_max = 1, mcu_x = 0, mcu_y = 0;
    Comp comp[4];
    bool progressive = false;
    int spec_start = 0, spec_end = 0, succ_high = 0, succ_low = 0, eob_run = 0;
    int scan_n = 0, order[4] = {0, 0, 0, 0};
    int restart_interval = 0, todo = 0;
    // entropy-coded bit buffer: valid bits at the top of `buf`
    uint32_t buf = 0;
    int bits = 0;
    int marker = kNoMarker;
    bool nomore = false;

    int get8() { return p < end ? *p++ : 0; }
    int get16() { const int a = get8(); return (a << 8) | get8(); }
    bool at_eof() const { return p >= end; }
    void skip(int n) { p = (n < 0 || end - p < n) ? end : p + n; }
    bool fail(const char* m) { err = m; return false; }

    // Refill to more than 24 bits; a marker inside the entropy data stops the refill for good and
    // later refills append zero bytes (stb_image.h:1567-1582).
    void fill() {
        do {
            const int b = nomore ? 0 : get8();
            if (b == 0xff) {
                const int c = get8();
                if (c != 0) {
                    marker = c;
                    nomore = true;
                    return;
                }
            }
            buf |= (uint32_t)b << (24 - bits);
            bits += 8;
        } while (bits <= 24);
    }
    uint32_t take(int n) {   // the next n (1..16) bits, in stream order
        if (bits < n) fill();
        const uint32_t v = buf >> (32 - n);
        buf <<= n;
        // past a marker the buffer's low bits are zeros (as stb's): keep `bits` non-negative so a
        // later fill never shifts by 32 or more (valid files never get here)
        bits = bits >= n ? bits - n : 0;
        return v;
    }
    int bit() { return (int)take(1); }
    // receive(n) + extend: an n-bit magnitude whose leading 0 marks a negative value
    int receive_extend(int n) {
        const int v = (int)take(n);
        return (v >> (n - 1)) ? v : v - ((1 << n) - 1);
    }
    int huff_decode(const Huff& h) {
        if (!h.defined) return -1;   // the scan names a table no DHT defined
        if (bits < 16) fill();
        const uint32_t top = buf >> 16;
        int k = 1;
        while (k <= 16 && top >= h.maxcode[k]) ++k;
        if (k == 17) { bits = bits >= 16 ? bits - 16 : 0; return -1; }
        if (k > bits) return -1;
        const int idx = (int)(buf >> (32 - k)) + h.delta[k];
        if (idx < 0 || idx >= h.nsym) return -1;
        buf <<= k;
        bits -= k;
        return h.values[idx];
    }

    void reset() {
        buf = 0;
        bits = 0;
        nomore = false;
        for (auto& c : comp) c.dc_pred = 0;
        marker = kNoMarker;
        todo = restart_interval ? restart_interval : 0x7fffffff;
        eob_run = 0;
    }

    int next_marker() {
        if (marker != kNoMarker) { const int m = marker; marker = kNoMarker; return m; }
        int x = get8();
        if (x != 0xff) return kNoMarker;
        while (x == 0xff) x = get8();
        return x;
    }

    // ---- blocks --------------------------------------------------------------------------
    bool block_baseline(int16_t out[64], int c) {
        Comp& C = comp[c];
        const uint8_t* dq = dequant[C.tq];
        const int t = huff_decode(huff_dc[C.hd]);
        if (t < 0 || t > 15) return fail("bad huffman code");
        std::memset(out, 0, 64 * sizeof(int16_t));
        const int diff = t ? receive_extend(t) : 0;
        C.dc_pred += diff;
        out[0] = (int16_t)(C.dc_pred * dq[0]);
        for (int k = 1; k < 64;) {
            const int rs = huff_decode(huff_ac[C.ha]);
            if (rs < 0) return fail("bad huffman code");
            const int run = rs >> 4, size = rs & 15;
            if (size == 0) {
                if (rs != 0xf0) break;   // end of block
                k += 16;
                continue;
            }
            k += run;
            const int z = kNatural[k++];
            out[z] = (int16_t)(receive_extend(size) * dq[z]);
        }
        return true;
    }
    bool block_prog_dc(int16_t* out, int c) {
        if (spec_end != 0) return fail("can't merge dc and ac");
        if (succ_high == 0) {
            std::memset(out, 0, 64 * sizeof(int16_t));
            const int t = huff_decode(huff_dc[comp[c].hd]);
            if (t < 0 || t > 15) return fail("bad huffman code");
            const int diff = t ? receive_extend(t) : 0;
            comp[c].dc_pred += diff;
            out[0] = (int16_t)(comp[c].dc_pred * (1 << succ_low));
        } else if (bit()) {
            out[0] = (int16_t)(out[0] + (1 << succ_low));
        }
        return true;
    }
    // refinement bit of an already-nonzero coefficient (stb_image.h:1833-1840)
    void refine(int16_t* q, int16_t b) {
        if (bit() && (*q & b) == 0) *q = (int16_t)(*q > 0 ? *q + b : *q - b);
    }
    bool block_prog_ac(int16_t* out, int c) {
        if (spec_start == 0) return fail("can't merge dc and ac");
        const Huff& ha = huff_ac[comp[c].ha];
        if (succ_high == 0) {
            if (eob_run) { --eob_run; return true; }
            for (int k = spec_start; k <= spec_end;) {
                const int rs = huff_decode(ha);
                if (rs < 0) return fail("bad huffman code");
                const int run = rs >> 4, size = rs & 15;
                if (size == 0) {
                    if (run < 15) {
                        eob_run = (1 << run) + (run ? (int)take(run) : 0) - 1;
                        break;
                    }
                    k += 16;
                    continue;
                }
                k += run;
                const int z = kNatural[k++];
                out[z] = (int16_t)(receive_extend(size) * (1 << succ_low));
            }
            return true;
        }
        const int16_t b = (int16_t)(1 << succ_low);
        if (eob_run) {
            --eob_run;
            for (int k = spec_start; k <= spec_end; ++k) {
                int16_t* q = &out[kNatural[k]];
                if (*q != 0) refine(q, b);
            }
            return true;
        }
        int k = spec_start;
        do {
            const int rs = huff_decode(ha);
            if (rs < 0) return fail("bad huffman code");
            int run = rs >> 4, size = rs & 15, val = 0;
            if (size == 0) {
                if (run < 15) {
                    eob_run = (1 << run) - 1 + (run ? (int)take(run) : 0);
                    run = 64;   // rest of the band: refine only
                }
            } else {
                if (size != 1) return fail("bad huffman code");
                val = bit() ? b : -b;
            }
            while (k <= spec_end) {
                int16_t* q = &out[kNatural[k++]];
                if (*q != 0) {
                    refine(q, b);
                } else {
                    if (run == 0) { *q = (int16_t)val; break; }
                    --run;
                }
            }
        } while (k <= spec_end);
        return true;
    }

    // ---- integer IDCT (stb_image.h:1906-2004) --------------------------------------------
    static int f2f(float x) { return (int)(x * 4096 + 0.5); }
    struct Idct1d { int t0, t1, t2, t3, x0, x1, x2, x3; };
    static Idct1d idct_1d(int s0, int s1, int s2, int s3, int s4, int s5, int s6, int s7) {
        Idct1d r;
        const int p1 = (s2 + s6) * f2f(0.5411961f);   // even part
        r.t2 = p1 + s6 * f2f(-1.847759065f);
        r.t3 = p1 + s2 * f2f(0.765366865f);
        const int e0 = (s0 + s4) * 4096, e1 = (s0 - s4) * 4096;
        r.x0 = e0 + r.t3;
        r.x3 = e0 - r.t3;
        r.x1 = e1 + r.t2;
        r.x2 = e1 - r.t2;
        int a0 = s7, a1 = s5, a2 = s3, a3 = s1;        // odd part
        int q3 = a0 + a2, q4 = a1 + a3, q1 = a0 + a3, q2 = a1 + a2;
        const int q5 = (q3 + q4) * f2f(1.175875602f);
        a0 = a0 * f2f(0.298631336f);
        a1 = a1 * f2f(2.053119869f);
        a2 = a2 * f2f(3.072711026f);
        a3 = a3 * f2f(1.501321110f);
        q1 = q5 + q1 * f2f(-0.899976223f);
        q2 = q5 + q2 * f2f(-2.562915447f);
        q3 = q3 * f2f(-1.961570560f);
        q4 = q4 * f2f(-0.390180644f);
        r.t3 = a3 + (q1 + q4);
        r.t2 = a2 + (q2 + q3);
        r.t1 = a1 + (q2 + q4);
        r.t0 = a0 + (q1 + q3);
        return r;
    }
    static void idct_block(uint8_t* out, int stride, const int16_t* d) {
        int v[64];
        for (int i = 0; i < 8; ++i) {   // columns, 2 extra bits of precision kept
            const int16_t* c = d + i;
            Idct1d r = idct_1d(c[0], c[8], c[16], c[24], c[32], c[40], c[48], c[56]);
            r.x0 += 512; r.x1 += 512; r.x2 += 512; r.x3 += 512;
            v[i + 0] = (r.x0 + r.t3) >> 10;
            v[i + 56] = (r.x0 - r.t3) >> 10;
            v[i + 8] = (r.x1 + r.t2) >> 10;
            v[i + 48] = (r.x1 - r.t2) >> 10;
            v[i + 16] = (r.x2 + r.t1) >> 10;
            v[i + 40] = (r.x2 - r.t1) >> 10;
            v[i + 24] = (r.x3 + r.t0) >> 10;
            v[i + 32] = (r.x3 - r.t0) >> 10;
        }
        for (int i = 0; i < 8; ++i) {   // rows: remove 2^17 with rounding, +128 level shift
            const int* w = v + 8 * i;
            Idct1d r = idct_1d(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7]);
            const int bias = 65536 + (128 << 17);
            r.x0 += bias; r.x1 += bias; r.x2 += bias; r.x3 += bias;
            uint8_t* o = out + (size_t)i * stride;
            o[0] = clamp255((r.x0 + r.t3) >> 17);
            o[7] = clamp255((r.x0 - r.t3) >> 17);
            o[1] = clamp255((r.x1 + r.t2) >> 17);
            o[6] = clamp255((r.x1 - r.t2) >> 17);
            o[2] = clamp255((r.x2 + r.t1) >> 17);
            o[5] = clamp255((r.x2 - r.t1) >> 17);
            o[3] = clamp255((r.x3 + r.t0) >> 17);
            o[4] = clamp255((r.x3 - r.t0) >> 17);
        }
    }

    // ---- scans ---------------------------------------------------------------------------
    // restart-interval countdown after an MCU: false = stop this scan (the marker is no restart)
    bool restart_or_stop() {
        if (--todo > 0) return true;
        if (bits < 24) fill();
        if (!(marker >= 0xd0 && marker <= 0xd7)) return false;
        reset();
        return true;
    }
    bool scan_data() {
        reset();
        int16_t blk[64];
        if (scan_n == 1) {   // non-interleaved: the component's own block grid, scanline order
            const int c = order[0];
            Comp& C = comp[c];
            const int w = (C.x + 7) >> 3, h = (C.y + 7) >> 3;
            for (int j = 0; j < h; ++j)
                for (int i = 0; i < w; ++i) {
                    if (!progressive) {
                        if (!block_baseline(blk, c)) return false;
                        idct_block(C.data.data() + (size_t)C.w2 * j * 8 + i * 8, C.w2, blk);
                    } else {
                        int16_t* q = C.coeff.data() + 64 * ((size_t)i + (size_t)j * C.coeff_w);
                        if (!(spec_start == 0 ? block_prog_dc(q, c) : block_prog_ac(q, c))) return false;
                    }
                    if (!restart_or_stop()) return true;
                }
            return true;
        }
        for (int j = 0; j < mcu_y; ++j)   // interleaved MCUs
            for (int i = 0; i < mcu_x; ++i) {
                for (int k = 0; k < scan_n; ++k) {
                    const int c = order[k];
                    Comp& C = comp[c];
                    for (int y = 0; y < C.v; ++y)
                        for (int x = 0; x < C.h; ++x) {
                            const int bx = i * C.h + x, by = j * C.v + y;
                            if (!progressive) {
                                if (!block_baseline(blk, c)) return false;
                                idct_block(C.data.data() + (size_t)C.w2 * by * 8 + bx * 8, C.w2, blk);
                            } else {
                                int16_t* q = C.coeff.data() + 64 * ((size_t)bx + (size_t)by * C.coeff_w);
                                if (!block_prog_dc(q, c)) return false;
                            }
                        }
                }
                if (!restart_or_stop()) return true;
            }
        return true;
    }

    // ---- markers -------------------------------------------------------------------------
    bool table_marker(int m) {
        switch (m) {
            case kNoMarker: return fail("expected marker");
            case 0xdd:   // DRI
                if (get16() != 4) return fail("bad DRI len");
                restart_interval = get16();
                return true;
            case 0xdb: {   // DQT: 8-bit tables only
                int L = get16() - 2;
                while (L > 0) {
                    const int q = get8(), prec = q >> 4, t = q & 15;
                    if (prec != 0) return fail("bad DQT type");
                    if (t > 3) return fail("bad DQT table");
                    for (int i = 0; i < 64; ++i) dequant[t][kNatural[i]] = (uint8_t)get8();
                    L -= 65;
                }
                return L == 0 || fail("bad DQT len");
            }
            case 0xc4: {   // DHT
                int L = get16() - 2;
                while (L > 0) {
                    const int q = get8(), tc = q >> 4, th = q & 15;
                    if (tc > 1 || th > 3) return fail("bad DHT header");
                    int count[16], n = 0;
                    for (int i = 0; i < 16; ++i) n += (count[i] = get8());
                    L -= 17;
                    Huff& h = tc == 0 ? huff_dc[th] : huff_ac[th];
                    if (!build_huff(h, count)) return fail("bad code lengths");
                    for (int i = 0; i < n; ++i) h.values[i] = (uint8_t)get8();
                    h.defined = true;
                    L -= n;
                }
                return L == 0 || fail("bad DHT len");
            }
        }
        if ((m >= 0xe0 && m <= 0xef) || m == 0xfe) {   // APPn, COM
            skip(get16() - 2);
            return true;
        }
        return fail("unsupported marker");
    }

    bool frame_header(bool load) {
        const int Lf = get16();
        if (Lf < 11) return fail("bad SOF len");
        if (get8() != 8) return fail("only 8-bit JPEG is supported");
        img_y = get16();
        if (img_y == 0) return fail("no header height");
        img_x = get16();
        if (img_x == 0) return fail("0 width");
        img_n = get8();
        if (img_n != 3 && img_n != 1) return fail("bad component count");
        if (Lf != 8 + 3 * img_n) return fail("bad SOF len");
        for (int i = 0; i < img_n; ++i) {
            Comp& C = comp[i];
            C.id = get8();
            if (C.id != i + 1 && C.id != i) return fail("bad component ID");
            const int q = get8();
            C.h = q >> 4;
            C.v = q & 15;
            if (C.h < 1 || C.h > 4) return fail("bad H");
            if (C.v < 1 || C.v > 4) return fail("bad V");
            C.tq = get8();
            if (C.tq > 3) return fail("bad TQ");
        }
        if (!load) return true;
        if ((1 << 30) / img_x / img_n < img_y) return fail("image too large to decode");
        h_max = v_max = 1;
        for (int i = 0; i < img_n; ++i) {
            h_max = std::max(h_max, comp[i].h);
            v_max = std::max(v_max, comp[i].v);
        }
        // non-integer sampling ratios (e.g. H 3 beside H 2): stb 2.06 reads past its component
        // planes there; rejected, as later stb versions do (valid files are unaffected)
        for (int i = 0; i < img_n; ++i) {
            if (h_max % comp[i].h != 0) return fail("bad H");
            if (v_max % comp[i].v != 0) return fail("bad V");
        }
        mcu_x = (img_x + h_max * 8 - 1) / (h_max * 8);
        mcu_y = (img_y + v_max * 8 - 1) / (v_max * 8);
        for (int i = 0; i < img_n; ++i) {
            Comp& C = comp[i];
            C.x = (img_x * C.h + h_max - 1) / h_max;
            C.y = (img_y * C.v + v_max - 1) / v_max;
            C.w2 = mcu_x * C.h * 8;   // whole MCUs decoded, cropped at colour conversion
            C.h2 = mcu_y * C.v * 8;
            C.data.assign((size_t)C.w2 * C.h2, 0);
            if (progressive) {
                C.coeff_w = (C.w2 + 7) >> 3;
                C.coeff_h = (C.h2 + 7) >> 3;
                C.coeff.assign((size_t)C.coeff_w * C.coeff_h * 64, 0);
            }
        }
        return true;
    }

    bool scan_header() {
        const int Ls = get16();
        scan_n = get8();
        if (scan_n < 1 || scan_n > 4 || scan_n > img_n) return fail("bad SOS component count");
        if (Ls != 6 + 2 * scan_n) return fail("bad SOS len");
        for (int i = 0; i < scan_n; ++i) {
            const int id = get8(), q = get8();
            int which = 0;
            while (which < img_n && comp[which].id != id) ++which;
            if (which == img_n) return fail("bad SOS component");
            comp[which].hd = q >> 4;
            comp[which].ha = q & 15;
            if (comp[which].hd > 3) return fail("bad DC huff");
            if (comp[which].ha > 3) return fail("bad AC huff");
            order[i] = which;
        }
        spec_start = get8();
        spec_end = get8();
        const int aa = get8();
        succ_high = aa >> 4;
        succ_low = aa & 15;
        if (progressive) {
            if (spec_start > 63 || spec_end > 63 || spec_start > spec_end || succ_high > 13 || succ_low > 13)
                return fail("bad SOS");
        } else {
            if (spec_start != 0 || succ_high != 0 || succ_low != 0) return fail("bad SOS");
            spec_end = 63;
        }
        return true;
    }

    static bool is_sof(int m) { return m == 0xc0 || m == 0xc1 || m == 0xc2; }

    bool header(bool load) {
        marker = kNoMarker;
        if (next_marker() != 0xd8) return fail("no SOI (not a JPEG file)");
        int m = next_marker();
        while (!is_sof(m)) {
            if (!table_marker(m)) return false;
            m = next_marker();
            while (m == kNoMarker) {   // padding after a segment
                if (at_eof()) return fail("no SOF");
                m = next_marker();
            }
        }
        progressive = m == 0xc2;
        return frame_header(load);
    }

    bool decode_image() {
        restart_interval = 0;
        if (!header(true)) return false;
        int m = next_marker();
        while (m != 0xd9) {   // EOI
            if (m == 0xda) {   // SOS
                if (!scan_header() || !scan_data()) return false;
                if (marker == kNoMarker) {   // zero bytes before the next marker are tolerated
                    while (!at_eof()) {
                        const int x = get8();
                        if (x == 0xff) { marker = get8(); break; }
                        if (x != 0) return fail("junk before marker");
                    }
                }
            } else if (!table_marker(m)) {
                return false;
            }
            if (at_eof() && marker == kNoMarker) return fail("no EOI");
            m = next_marker();
        }
        if (progressive)   // dequantize + IDCT every block once all scans are in
            for (int c = 0; c < img_n; ++c) {
                Comp& C = comp[c];
                const int w = (C.x + 7) >> 3, h = (C.y + 7) >> 3;
                for (int j = 0; j < h; ++j)
                    for (int i = 0; i < w; ++i) {
                        int16_t* q = C.coeff.data() + 64 * ((size_t)i + (size_t)j * C.coeff_w);
                        for (int k = 0; k < 64; ++k) q[k] = (int16_t)(q[k] * dequant[C.tq][k]);
                        idct_block(C.data.data() + (size_t)C.w2 * j * 8 + i * 8, C.w2, q);
                    }
            }
        return true;
    }
};

// ---- upsampling (stb_image.h:2838-3039) ------------------------------------------------
using Resample = const uint8_t* (*)(uint8_t* out, const uint8_t* near_, const uint8_t* far_, int w, int hs);

const uint8_t* up_1(uint8_t*, const uint8_t* near_, const uint8_t*, int, int) { return near_; }
const uint8_t* up_v2(uint8_t* out, const uint8_t* near_, const uint8_t* far_, int w, int) {
    for (int i = 0; i < w; ++i) out[i] = (uint8_t)((3 * near_[i] + far_[i] + 2) >> 2);
    return out;
}
const uint8_t* up_h2(uint8_t* out, const uint8_t* in, const uint8_t*, int w, int) {
    if (w == 1) {
        out[0] = out[1] = in[0];
        return out;
    }
    out[0] = in[0];
    out[1] = (uint8_t)((in[0] * 3 + in[1] + 2) >> 2);
    int i = 1;
    for (; i < w - 1; ++i) {
        const int n = 3 * in[i] + 2;
        out[2 * i] = (uint8_t)((n + in[i - 1]) >> 2);
        out[2 * i + 1] = (uint8_t)((n + in[i + 1]) >> 2);
    }
    out[2 * i] = (uint8_t)((in[w - 2] * 3 + in[w - 1] + 2) >> 2);
    out[2 * i + 1] = in[w - 1];
    return out;
}
const uint8_t* up_hv2(uint8_t* out, const uint8_t* near_, const uint8_t* far_, int w, int) {
    if (w == 1) {
        out[0] = out[1] = (uint8_t)((3 * near_[0] + far_[0] + 2) >> 2);
        return out;
    }
    int cur = 3 * near_[0] + far_[0];   // vertical pass, then the horizontal triangle filter
    out[0] = (uint8_t)((cur + 2) >> 2);
    for (int i = 1; i < w; ++i) {
        const int prev = cur;
        cur = 3 * near_[i] + far_[i];
        out[2 * i - 1] = (uint8_t)((3 * prev + cur + 8) >> 4);
        out[2 * i] = (uint8_t)((3 * cur + prev + 8) >> 4);
    }
    out[2 * w - 1] = (uint8_t)((cur + 2) >> 2);
    return out;
}
const uint8_t* up_nearest(uint8_t* out, const uint8_t* near_, const uint8_t*, int w, int hs) {
    for (int i = 0; i < w; ++i)
        for (int j = 0; j < hs; ++j) out[i * hs + j] = near_[i];
    return out;
}

// reduced-precision YCbCr -> RGB (stb_image.h:3070-3096), 3 bytes per output pixel
int fix12(float x) { return ((int)(x * 4096.0f + 0.5f)) << 8; }
void ycbcr_row(uint8_t* out, const uint8_t* y, const uint8_t* cb, const uint8_t* cr, int count) {
    const int kr = fix12(1.40200f), kg_cr = -fix12(0.71414f), kg_cb = -fix12(0.34414f), kb = fix12(1.77200f);
    for (int i = 0; i < count; ++i) {
        const int yf = (y[i] << 20) + (1 << 19);
        const int dr = cr[i] - 128, db = cb[i] - 128;
        const int g_cb = (int)((uint32_t)(db * kg_cb) & 0xffff0000u);   // truncated Cb term of green
        out[3 * i + 0] = clamp255((yf + dr * kr) >> 20);
        out[3 * i + 1] = clamp255((yf + dr * kg_cr + g_cb) >> 20);
        out[3 * i + 2] = clamp255((yf + db * kb) >> 20);
    }
}

}  // namespace

// stbi_load(..., req_comp = 0) for JPEG data: width, height, components (1 or 3) and the
// interleaved 8-bit pixels, top row first.  pixels == nullptr: header only.
int decode_jpeg(const uint8_t* data, size_t size, int32_t* width, int32_t* height, int32_t* components,
                std::vector<uint8_t>* pixels) {
    Decoder z;
    z.p = data;
    z.end = data + size;
    if (!pixels) {
        if (!z.header(false)) return fail(PT_ERR_PARSE, "JPEG: " + z.err);
    } else {
        if (!z.decode_image()) return fail(PT_ERR_PARSE, "JPEG: " + z.err);
        const int n = z.img_n;
        pixels->assign((size_t)n * z.img_x * z.img_y, 0);
        struct Row {   // stbi__resample (stb_image.h:3282-3290)
            Resample fn = nullptr;
            const uint8_t *line0 = nullptr, *line1 = nullptr;
            int hs = 1, vs = 1, w_lores = 0, ystep = 0, ypos = 0;
            std::vector<uint8_t> buf;
        } rs[4];
        for (int k = 0; k < n; ++k) {
            Row& r = rs[k];
            r.hs = z.h_max / z.comp[k].h;
            r.vs = z.v_max / z.comp[k].v;
            r.ystep = r.vs >> 1;
            r.w_lores = (z.img_x + r.hs - 1) / r.hs;
            r.line0 = r.line1 = z.comp[k].data.data();
            r.buf.assign((size_t)r.w_lores * r.hs + 4, 0);
            r.fn = (r.hs == 1 && r.vs == 1)   ? up_1
                   : (r.hs == 1 && r.vs == 2) ? up_v2
                   : (r.hs == 2 && r.vs == 1) ? up_h2
                   : (r.hs == 2 && r.vs == 2) ? up_hv2
                                              : up_nearest;
        }
        const uint8_t* row[4] = {nullptr, nullptr, nullptr, nullptr};
        for (int j = 0; j < z.img_y; ++j) {
            uint8_t* out = pixels->data() + (size_t)n * z.img_x * j;
            for (int k = 0; k < n; ++k) {
                Row& r = rs[k];
                const bool bot = r.ystep >= (r.vs >> 1);   // output row nearer the next low-res row
                row[k] = r.fn(r.buf.data(), bot ? r.line1 : r.line0, bot ? r.line0 : r.line1, r.w_lores, r.hs);
                if (++r.ystep >= r.vs) {
                    r.ystep = 0;
                    r.line0 = r.line1;
                    if (++r.ypos < z.comp[k].y) r.line1 += z.comp[k].w2;
                }
            }
            if (n == 3) ycbcr_row(out, row[0], row[1], row[2], z.img_x);
            else std::memcpy(out, row[0], (size_t)z.img_x);
        }
    }
    *width = z.img_x;
    *height = z.img_y;
    *components = z.img_n;
    return PT_OK;
}

// Texture::load (sceneStructs.h:171-175) for a JSON scene's TEXTURE_FILE.
int load_texture_file(TextureHost& t) {
    std::FILE* f = std::fopen(t.path.c_str(), "rb");
    if (!f) return fail(PT_ERR_IO, "Texture load error: cannot open " + t.path);
    std::vector<uint8_t> bytes;
    uint8_t chunk[65536];
    size_t got;
    while ((got = std::fread(chunk, 1, sizeof chunk, f)) > 0) bytes.insert(bytes.end(), chunk, chunk + got);
    std::fclose(f);
    // Not a JPEG (no SOI marker): PNG/BMP/TGA/... files that the reference's stbi_load also reads
    // are left to the host — the texture keeps its path and no pixels, pt_scene_set_texture_pixels
    // fills it, and pt_create refuses a scene with an unfilled texture.
    if (bytes.size() < 2 || bytes[0] != 0xff || bytes[1] != 0xd8) return PT_OK;
    int32_t w = 0, h = 0, c = 0;
    if (decode_jpeg(bytes.data(), bytes.size(), &w, &h, &c, &t.pixels) != PT_OK)
        return fail(PT_ERR_IO, "Texture load error: " + t.path + ": " + g_err);
    t.width = w;
    t.height = h;
    t.components = c;
    return PT_OK;
}

}  // namespace pt

extern "C" int pt_decode_jpeg(const uint8_t* data, int64_t size, int32_t* width, int32_t* height,
                              int32_t* components, uint8_t* out, int64_t cap) {
    if (!data || size <= 0 || !width || !height || !components) return pt::fail(PT_ERR_ARG, "null argument");
    if (!out) return pt::decode_jpeg(data, (size_t)size, width, height, components, nullptr);
    std::vector<uint8_t> px;
    if (int rc = pt::decode_jpeg(data, (size_t)size, width, height, components, &px)) return rc;
    if ((int64_t)px.size() > cap) return pt::fail(PT_ERR_ARG, "output buffer too small");
    std::memcpy(out, px.data(), px.size());
    return PT_OK;
}
