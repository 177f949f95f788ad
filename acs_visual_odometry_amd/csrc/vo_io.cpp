// vo_io.cpp -- image input of the trajectory loop: cv::imread(path, cv::IMREAD_GRAYSCALE)
// (VisualOdometry.cpp:65,76) for the formats a KITTI-style sequence comes in, without OpenCV.
//
//   PNG  (zlib inflate; every bit depth and colour type, Adam7 interlacing)
//   PGM  binary P5, maxval <= 255
//
// Conversion to 8-bit gray follows what OpenCV's PNG decoder asks libpng for under
// IMREAD_GRAYSCALE: gray 1/2/4-bit expanded to 8 bits, 16-bit samples reduced to their high
// byte (png_set_strip_16), palette expanded to RGB, alpha dropped, and RGB -> gray with
// png_set_rgb_to_gray(0.299, 0.587), i.e. the 15-bit fixed-point weights 9797 / 19234 / 3737.
// KITTI sequences and the repository fixtures are 8-bit gray PNGs, for which the decode is
// exact; the colour path is a restatement of libpng's arithmetic (libpng is absent here).
#include <zlib.h>

#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/vo_mi355x.h"

namespace {

bool read_file(const char* path, std::vector<uint8_t>& buf)
{
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (n < 0) { std::fclose(f); return false; }
    buf.resize((size_t)n);
    bool ok = n == 0 || std::fread(buf.data(), 1, (size_t)n, f) == (size_t)n;
    std::fclose(f);
    return ok;
}

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

int paeth(int a, int b, int c)
{
    int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

// undo the PNG filters of one pass (h rows of rowbytes bytes, bpp bytes per complete pixel)
bool unfilter(uint8_t* data, size_t rowbytes, int h, int bpp, std::vector<uint8_t>& out)
{
    out.assign(rowbytes * h, 0);
    const uint8_t* prev = nullptr;
    for (int y = 0; y < h; ++y) {
        const uint8_t* src = data + (size_t)y * (rowbytes + 1);
        uint8_t* dst = out.data() + (size_t)y * rowbytes;
        const int ft = src[0];
        ++src;
        for (size_t x = 0; x < rowbytes; ++x) {
            const int a = x >= (size_t)bpp ? dst[x - bpp] : 0;
            const int b = prev ? prev[x] : 0;
            const int c = (prev && x >= (size_t)bpp) ? prev[x - bpp] : 0;
            int v = src[x];
            switch (ft) {
            case 0: break;
            case 1: v += a; break;
            case 2: v += b; break;
            case 3: v += (a + b) >> 1; break;
            case 4: v += paeth(a, b, c); break;
            default: return false;
            }
            dst[x] = (uint8_t)v;
        }
        prev = dst;
    }
    return true;
}

struct PngInfo {
    int w = 0, h = 0, depth = 0, color = 0, interlace = 0;
    int channels = 1;
    std::vector<uint8_t> plte;   // RGB triples
};

// sample s (channel ch) of pixel x in an unfiltered row
inline uint32_t sample(const uint8_t* row, int x, int ch, const PngInfo& p)
{
    if (p.depth == 8) return row[(size_t)x * p.channels + ch];
    if (p.depth == 16) {
        const uint8_t* q = row + ((size_t)x * p.channels + ch) * 2;
        return (uint32_t)q[0] << 8 | q[1];
    }
    // 1/2/4-bit: one channel (gray or palette index), MSB first
    const int per = 8 / p.depth;
    const int shift = 8 - p.depth * (x % per + 1);
    return (row[x / per] >> shift) & ((1u << p.depth) - 1);
}

// one pixel of an unfiltered row -> 8-bit gray (IMREAD_GRAYSCALE as configured by OpenCV)
inline uint8_t to_gray(const uint8_t* row, int x, const PngInfo& p)
{
    uint32_t r, g, b;
    switch (p.color) {
    case 0:    // gray
    case 4: {  // gray + alpha (alpha stripped)
        uint32_t v = sample(row, x, 0, p);
        if (p.depth == 16) return (uint8_t)(v >> 8);
        if (p.depth < 8) return (uint8_t)(v * (255u / ((1u << p.depth) - 1)));
        return (uint8_t)v;
    }
    case 3: {  // palette -> RGB
        uint32_t i = sample(row, x, 0, p);
        if (3 * (size_t)i + 2 >= p.plte.size()) return 0;
        r = p.plte[3 * i]; g = p.plte[3 * i + 1]; b = p.plte[3 * i + 2];
        break;
    }
    default:   // RGB (2) / RGBA (6)
        r = sample(row, x, 0, p); g = sample(row, x, 1, p); b = sample(row, x, 2, p);
    }
    // png_do_rgb_to_gray without a gamma table (libpng 1.6 pngrtran.c): equal channels pass
    // through, else the 15-bit fixed-point sum -- truncated for 8-bit samples ("the historical
    // approach which simply truncates"), rounded for 16-bit ones, which png_set_strip_16 then
    // truncates to 8 bits.  A PNG whose gAMA / sRGB chunk makes libpng build gamma tables is
    // converted through those tables by libpng; that path is not modelled here.
    const uint32_t sum = 9797u * r + 19234u * g + 3737u * b;
    const uint32_t v = (r == g && g == b) ? r : (p.depth == 16 ? (sum + 16384u) >> 15 : sum >> 15);
    return (uint8_t)(p.depth == 16 ? v >> 8 : v);
}

int decode_png(const std::vector<uint8_t>& f, std::vector<uint8_t>& img, int& W, int& H)
{
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (f.size() < 8 || std::memcmp(f.data(), sig, 8) != 0) return VO_ERR_IO;
    PngInfo p;
    std::vector<uint8_t> idat;
    size_t pos = 8;
    bool have_hdr = false;
    while (pos + 12 <= f.size()) {
        const uint32_t len = be32(&f[pos]);
        if (len > f.size() - pos - 12) return VO_ERR_IO;
        const uint8_t* type = &f[pos + 4];
        const uint8_t* d = &f[pos + 8];
        if (!std::memcmp(type, "IHDR", 4) && len >= 13) {
            p.w = (int)be32(d); p.h = (int)be32(d + 4);
            p.depth = d[8]; p.color = d[9]; p.interlace = d[12];
            if (d[10] != 0 || d[11] != 0 || p.interlace > 1) return VO_ERR_IO;
            have_hdr = true;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            p.plte.assign(d, d + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), d, d + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        pos += 12 + (size_t)len;
    }
    if (!have_hdr || p.w <= 0 || p.h <= 0 || p.w > 65535 || p.h > 65535) return VO_ERR_IO;
    switch (p.color) {
    case 0: p.channels = 1; break;
    case 2: p.channels = 3; break;
    case 3: p.channels = 1; break;
    case 4: p.channels = 2; break;
    case 6: p.channels = 4; break;
    default: return VO_ERR_IO;
    }
    const int bits = p.channels * p.depth;
    if (!(p.depth == 1 || p.depth == 2 || p.depth == 4 || p.depth == 8 || p.depth == 16)) return VO_ERR_IO;
    if (p.depth < 8 && p.channels != 1) return VO_ERR_IO;
    if (p.color == 3 && p.depth == 16) return VO_ERR_IO;
    const int bpp = bits >= 8 ? bits / 8 : 1;

    // passes: Adam7 sub-images or the whole image
    struct Pass { int x0, y0, dx, dy; };
    static const Pass adam7[7] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                  {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
    const Pass whole = {0, 0, 1, 1};
    const int npass = p.interlace ? 7 : 1;
    size_t raw_size = 0;
    for (int k = 0; k < npass; ++k) {
        const Pass& ps = p.interlace ? adam7[k] : whole;
        const int pw = (p.w - ps.x0 + ps.dx - 1) / ps.dx, ph = (p.h - ps.y0 + ps.dy - 1) / ps.dy;
        if (pw > 0 && ph > 0) raw_size += ((size_t)pw * bits + 7) / 8 * ph + ph;
    }
    std::vector<uint8_t> raw(raw_size);
    uLongf got = (uLongf)raw_size;
    if (uncompress(raw.data(), &got, idat.data(), (uLong)idat.size()) != Z_OK || got != raw_size) return VO_ERR_IO;

    W = p.w; H = p.h;
    img.assign((size_t)W * H, 0);
    size_t off = 0;
    std::vector<uint8_t> rows;
    for (int k = 0; k < npass; ++k) {
        const Pass& ps = p.interlace ? adam7[k] : whole;
        const int pw = (p.w - ps.x0 + ps.dx - 1) / ps.dx, ph = (p.h - ps.y0 + ps.dy - 1) / ps.dy;
        if (pw <= 0 || ph <= 0) continue;
        const size_t rowbytes = ((size_t)pw * bits + 7) / 8;
        if (!unfilter(raw.data() + off, rowbytes, ph, bpp, rows)) return VO_ERR_IO;
        off += (rowbytes + 1) * ph;
        for (int y = 0; y < ph; ++y) {
            const uint8_t* row = rows.data() + (size_t)y * rowbytes;
            uint8_t* dst = img.data() + (size_t)(ps.y0 + y * ps.dy) * W;
            for (int x = 0; x < pw; ++x) dst[ps.x0 + x * ps.dx] = to_gray(row, x, p);
        }
    }
    return VO_OK;
}

int decode_pgm(const std::vector<uint8_t>& f, std::vector<uint8_t>& img, int& W, int& H)
{
    // P5 <ws> width <ws> height <ws> maxval <one ws> raster; '#' comments in the header
    size_t pos = 2;
    int vals[3];
    for (int k = 0; k < 3; ++k) {
        for (;;) {
            while (pos < f.size() && std::isspace(f[pos])) ++pos;
            if (pos < f.size() && f[pos] == '#') {
                while (pos < f.size() && f[pos] != '\n') ++pos;
                continue;
            }
            break;
        }
        long v = 0;
        size_t s = pos;
        while (pos < f.size() && f[pos] >= '0' && f[pos] <= '9' && v < 1000000) v = v * 10 + (f[pos++] - '0');
        if (pos == s) return VO_ERR_IO;
        vals[k] = (int)v;
    }
    if (pos >= f.size() || !std::isspace(f[pos])) return VO_ERR_IO;
    ++pos;
    W = vals[0]; H = vals[1];
    if (W <= 0 || H <= 0 || W > 65535 || H > 65535 || vals[2] <= 0 || vals[2] > 255) return VO_ERR_IO;
    if (f.size() - pos < (size_t)W * H) return VO_ERR_IO;
    img.assign(f.begin() + (long)pos, f.begin() + (long)pos + (long)W * H);
    return VO_OK;
}

}  // namespace

extern "C" int vo_imread_gray(const char* path, uint8_t* out, size_t cap, int* width, int* height)
{
    if (!path || !width || !height) return VO_ERR_ARG;
    *width = *height = 0;
    std::vector<uint8_t> f, img;
    if (!read_file(path, f)) return VO_ERR_IO;
    int W = 0, H = 0, rc;
    if (f.size() >= 2 && f[0] == 'P' && f[1] == '5') rc = decode_pgm(f, img, W, H);
    else rc = decode_png(f, img, W, H);
    if (rc) return rc;
    *width = W;
    *height = H;
    if (out) {
        if (cap < (size_t)W * H) return VO_ERR_CAPACITY;
        std::memcpy(out, img.data(), (size_t)W * H);
    }
    return VO_OK;
}
