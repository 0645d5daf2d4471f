// mcpt_image_io.hpp -- header-only framebuffer output for C++ callers of mcpt.h.
//
// encode_8bit_cv reproduces the reference's PNG encode (CVMCTracer/main.cpp:19-29,
// CUTracer.cu:383-396): cvSet2D(img, y, x, CvScalar(c.z*255, c.y*255, c.x*255))
// on an 8-bit image = channel*255 in float, cvRound (nearest, ties to even),
// saturate to [0,255]; NaN, +-inf and |v| >= 2^31 -> 0 (cvtsd2si's INT_MIN).  write_png writes 8-bit RGB with stored
// (uncompressed) deflate blocks, so no zlib/OpenCV is needed; write_pfm keeps
// the linear float image (bottom-up rows, little-endian).
#pragma once

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

namespace mcpt {
namespace image {

inline uint8_t encode_channel_cv(float c) {
    const double v = static_cast<double>(c * 255.0f);   // PWVector3f component * 255 (float), widened
    if (!(std::fabs(v) < 2147483648.0)) return 0;        // cvRound (cvtsd2si): NaN/inf/huge -> INT_MIN -> 0
    const double r = std::nearbyint(v);                  // default rounding mode: ties to even
    return static_cast<uint8_t>(r < 0.0 ? 0.0 : (r > 255.0 ? 255.0 : r));
}

// rgb: width*height*3 floats, row-major y*W+x (the reference's hostcolor)
inline std::vector<uint8_t> encode_8bit_cv(const float* rgb, int width, int height) {
    std::vector<uint8_t> out(static_cast<size_t>(width) * height * 3);
    for (size_t i = 0; i < out.size(); ++i) out[i] = encode_channel_cv(rgb[i]);
    return out;
}

namespace detail {
inline uint32_t crc32(const uint8_t* p, size_t n, uint32_t c = 0xFFFFFFFFu) {
    for (size_t i = 0; i < n; ++i) {
        c ^= p[i];
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    }
    return c;
}
inline void be32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back(uint8_t(x >> 24)); v.push_back(uint8_t(x >> 16)); v.push_back(uint8_t(x >> 8)); v.push_back(uint8_t(x));
}
inline void chunk(std::vector<uint8_t>& f, const char* tag, const std::vector<uint8_t>& data) {
    be32(f, static_cast<uint32_t>(data.size()));
    std::vector<uint8_t> td(tag, tag + 4);
    td.insert(td.end(), data.begin(), data.end());
    f.insert(f.end(), td.begin(), td.end());
    be32(f, crc32(td.data(), td.size()) ^ 0xFFFFFFFFu);
}
}  // namespace detail

// 8-bit RGB (width*height*3) -> PNG file; returns false on I/O failure
inline bool write_png(const std::string& path, const uint8_t* rgb8, int width, int height) {
    std::vector<uint8_t> raw;
    raw.reserve(static_cast<size_t>(height) * (1 + 3 * static_cast<size_t>(width)));
    for (int y = 0; y < height; ++y) {
        raw.push_back(0);                                // filter: none
        raw.insert(raw.end(), rgb8 + static_cast<size_t>(y) * width * 3, rgb8 + static_cast<size_t>(y + 1) * width * 3);
    }
    std::vector<uint8_t> z{0x78, 0x01};                  // zlib header, stored blocks
    uint32_t a = 1, b = 0;
    for (uint8_t x : raw) { a = (a + x) % 65521u; b = (b + a) % 65521u; }
    for (size_t off = 0; off < raw.size() || off == 0; off += 65535) {
        const size_t n = raw.size() - off < 65535 ? raw.size() - off : 65535;
        z.push_back(off + n >= raw.size() ? 1 : 0);
        z.push_back(uint8_t(n)); z.push_back(uint8_t(n >> 8));
        z.push_back(uint8_t(~n)); z.push_back(uint8_t(~n >> 8));
        z.insert(z.end(), raw.begin() + off, raw.begin() + off + n);
        if (raw.empty()) break;
    }
    detail::be32(z, (b << 16) | a);
    std::vector<uint8_t> f{0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    std::vector<uint8_t> ihdr;
    detail::be32(ihdr, static_cast<uint32_t>(width));
    detail::be32(ihdr, static_cast<uint32_t>(height));
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});
    detail::chunk(f, "IHDR", ihdr);
    detail::chunk(f, "IDAT", z);
    detail::chunk(f, "IEND", {});
    FILE* fp = std::fopen(path.c_str(), "wb");
    if (!fp) return false;
    const bool ok = std::fwrite(f.data(), 1, f.size(), fp) == f.size();
    return std::fclose(fp) == 0 && ok;
}

// float RGB hostcolor -> PNG with the reference's encode
inline bool write_png(const std::string& path, const float* rgb, int width, int height) {
    const std::vector<uint8_t> e = encode_8bit_cv(rgb, width, height);
    return write_png(path, e.data(), width, height);
}

inline bool write_pfm(const std::string& path, const float* rgb, int width, int height) {
    FILE* fp = std::fopen(path.c_str(), "wb");
    if (!fp) return false;
    std::fprintf(fp, "PF\n%d %d\n-1.0\n", width, height);
    bool ok = true;
    for (int y = height - 1; y >= 0; --y)
        ok = ok && std::fwrite(rgb + static_cast<size_t>(y) * width * 3, sizeof(float), static_cast<size_t>(width) * 3, fp) ==
                       static_cast<size_t>(width) * 3;
    return std::fclose(fp) == 0 && ok;
}

}  // namespace image
}  // namespace mcpt
