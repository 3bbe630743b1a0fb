// film.cpp -- film output, the step after the hot path.
//
// SaveFloatImageToJpg (SceneRenderingHelper.cpp:57-70): per channel
// (unsigned char)(255 * pow(clamp(x, 0, 1), 0.6f)), then a quality-100 JPEG
// (stb_image_write, which at q100 uses 4:4:4 and all-ones quantisation).  This is
// an independent baseline JPEG encoder (JFIF, 4:4:4, quantiser 1, Annex K
// Huffman tables); .ppm and .pfm (raw float, bottom-up) are offered for lossless
// artefacts.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/tpt_host.h"

namespace {

unsigned char tonemap(float v) {  // SceneRenderingHelper.cpp:62-64
    return (unsigned char)(255 * std::pow(std::clamp(v, 0.f, 1.f), 0.6f));
}

struct BitWriter {
    std::vector<unsigned char>& out;
    uint32_t acc = 0;
    int n = 0;
    explicit BitWriter(std::vector<unsigned char>& o) : out(o) {}
    void put(uint32_t code, int len) {
        for (int i = len - 1; i >= 0; --i) {
            acc = (acc << 1) | ((code >> i) & 1u);
            if (++n == 8) {
                out.push_back((unsigned char)acc);
                if (acc == 0xff) out.push_back(0);  // byte stuffing
                acc = 0;
                n = 0;
            }
        }
    }
    void flush() {
        while (n) put(1, 1);
    }
};

// ITU-T T.81 Annex K.3 standard Huffman tables
const unsigned char kDcLumBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const unsigned char kDcLumVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const unsigned char kDcChrBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const unsigned char kDcChrVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const unsigned char kAcLumBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
const unsigned char kAcLumVal[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71, 0x14,
    0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09,
    0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a,
    0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65,
    0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88,
    0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9,
    0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
    0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea,
    0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
const unsigned char kAcChrBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
const unsigned char kAcChrVal[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22, 0x32,
    0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16,
    0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39,
    0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
    0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86,
    0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7,
    0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8,
    0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9,
    0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
const int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                         41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                         30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huff {
    uint16_t code[256];
    uint8_t len[256];
    Huff(const unsigned char* bits, const unsigned char* val) {
        for (int i = 0; i < 256; ++i) { code[i] = 0; len[i] = 0; }
        int k = 0;
        uint16_t c = 0;
        for (int l = 1; l <= 16; ++l) {
            for (int i = 0; i < bits[l - 1]; ++i) { code[val[k]] = c++; len[val[k]] = (uint8_t)l; ++k; }
            c <<= 1;
        }
    }
};

int nbits(int v) {
    v = v < 0 ? -v : v;
    int n = 0;
    while (v) { ++n; v >>= 1; }
    return n;
}

void encode_block(BitWriter& bw, const float in[64], int& prev_dc, const Huff& dc, const Huff& ac) {
    static double cosv[8][8];
    static bool init = false;
    if (!init) {
        for (int x = 0; x < 8; ++x)
            for (int u = 0; u < 8; ++u) cosv[x][u] = std::cos((2 * x + 1) * u * M_PI / 16.0);
        init = true;
    }
    int q[64];
    for (int v = 0; v < 8; ++v)
        for (int u = 0; u < 8; ++u) {
            double s = 0;
            for (int y = 0; y < 8; ++y)
                for (int x = 0; x < 8; ++x) s += in[y * 8 + x] * cosv[x][u] * cosv[y][v];
            double cu = u == 0 ? M_SQRT1_2 : 1.0, cv = v == 0 ? M_SQRT1_2 : 1.0;
            q[v * 8 + u] = (int)std::lround(0.25 * cu * cv * s);  // quantiser = 1 (quality 100)
        }
    int diff = q[0] - prev_dc;
    prev_dc = q[0];
    int nb = nbits(diff);
    bw.put(dc.code[nb], dc.len[nb]);
    if (nb) bw.put((uint32_t)(diff < 0 ? diff + (1 << nb) - 1 : diff), nb);
    int run = 0;
    for (int k = 1; k < 64; ++k) {
        int v = q[kZigzag[k]];
        if (v == 0) { ++run; continue; }
        while (run > 15) { bw.put(ac.code[0xf0], ac.len[0xf0]); run -= 16; }
        int s = nbits(v);
        int sym = (run << 4) | s;
        bw.put(ac.code[sym], ac.len[sym]);
        bw.put((uint32_t)(v < 0 ? v + (1 << s) - 1 : v), s);
        run = 0;
    }
    if (run) bw.put(ac.code[0], ac.len[0]);
}

bool write_jpeg(const std::vector<unsigned char>& rgb, int w, int h, const std::string& path) {
    std::vector<unsigned char> o;
    auto w16 = [&](int v) { o.push_back((unsigned char)(v >> 8)); o.push_back((unsigned char)v); };
    o.insert(o.end(), {0xff, 0xd8, 0xff, 0xe0});
    w16(16);
    o.insert(o.end(), {'J', 'F', 'I', 'F', 0, 1, 1, 0});
    w16(1); w16(1);
    o.insert(o.end(), {0, 0});
    for (int t = 0; t < 2; ++t) {  // DQT: all ones
        o.insert(o.end(), {0xff, 0xdb});
        w16(67);
        o.push_back((unsigned char)t);
        for (int i = 0; i < 64; ++i) o.push_back(1);
    }
    o.insert(o.end(), {0xff, 0xc0});
    w16(17);
    o.push_back(8); w16(h); w16(w); o.push_back(3);
    o.insert(o.end(), {1, 0x11, 0, 2, 0x11, 1, 3, 0x11, 1});
    auto dht = [&](int cls_id, const unsigned char* bits, const unsigned char* val) {
        int n = 0;
        for (int i = 0; i < 16; ++i) n += bits[i];
        o.insert(o.end(), {0xff, 0xc4});
        w16(19 + n);
        o.push_back((unsigned char)cls_id);
        o.insert(o.end(), bits, bits + 16);
        o.insert(o.end(), val, val + n);
    };
    dht(0x00, kDcLumBits, kDcLumVal);
    dht(0x10, kAcLumBits, kAcLumVal);
    dht(0x01, kDcChrBits, kDcChrVal);
    dht(0x11, kAcChrBits, kAcChrVal);
    o.insert(o.end(), {0xff, 0xda});
    w16(12);
    o.insert(o.end(), {3, 1, 0x00, 2, 0x11, 3, 0x11, 0, 63, 0});
    Huff dcl(kDcLumBits, kDcLumVal), acl(kAcLumBits, kAcLumVal), dcc(kDcChrBits, kDcChrVal), acc(kAcChrBits, kAcChrVal);
    BitWriter bw(o);
    int pdc[3] = {0, 0, 0};
    float blk[3][64];
    for (int by = 0; by < h; by += 8)
        for (int bx = 0; bx < w; bx += 8) {
            for (int y = 0; y < 8; ++y)
                for (int x = 0; x < 8; ++x) {
                    int sx = std::min(bx + x, w - 1), sy = std::min(by + y, h - 1);
                    const unsigned char* p = &rgb[3 * ((size_t)sy * w + sx)];
                    float r = p[0], g = p[1], b = p[2];
                    blk[0][y * 8 + x] = 0.299f * r + 0.587f * g + 0.114f * b - 128.f;
                    blk[1][y * 8 + x] = -0.168736f * r - 0.331264f * g + 0.5f * b;
                    blk[2][y * 8 + x] = 0.5f * r - 0.418688f * g - 0.081312f * b;
                }
            encode_block(bw, blk[0], pdc[0], dcl, acl);
            encode_block(bw, blk[1], pdc[1], dcc, acc);
            encode_block(bw, blk[2], pdc[2], dcc, acc);
        }
    bw.flush();
    o.insert(o.end(), {0xff, 0xd9});
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    bool ok = std::fwrite(o.data(), 1, o.size(), f) == o.size();
    return std::fclose(f) == 0 && ok;
}

bool ends_with(const std::string& s, const char* suf) {
    std::string t(suf);
    return s.size() >= t.size() && s.compare(s.size() - t.size(), t.size(), t) == 0;
}

}  // namespace

extern "C" int tpt_save_image(const float* rgb, int32_t w, int32_t h, const char* path_c) {
    if (!rgb || !path_c || w <= 0 || h <= 0) return TPT_E_INVALID;
    std::string path(path_c);
    if (ends_with(path, ".pfm")) {
        FILE* f = std::fopen(path.c_str(), "wb");
        if (!f) return TPT_E_INVALID;
        std::fprintf(f, "PF\n%d %d\n-1.0\n", w, h);
        for (int y = h - 1; y >= 0; --y) std::fwrite(rgb + 3 * (size_t)y * w, sizeof(float), 3 * (size_t)w, f);
        return std::fclose(f) == 0 ? TPT_OK : TPT_E_INVALID;
    }
    std::vector<unsigned char> px(3 * (size_t)w * h);
    for (size_t i = 0; i < px.size(); ++i) px[i] = tonemap(rgb[i]);
    if (ends_with(path, ".ppm")) {
        FILE* f = std::fopen(path.c_str(), "wb");
        if (!f) return TPT_E_INVALID;
        std::fprintf(f, "P6\n%d %d\n255\n", w, h);
        std::fwrite(px.data(), 1, px.size(), f);
        return std::fclose(f) == 0 ? TPT_OK : TPT_E_INVALID;
    }
    return write_jpeg(px, w, h, path) ? TPT_OK : TPT_E_INVALID;
}
