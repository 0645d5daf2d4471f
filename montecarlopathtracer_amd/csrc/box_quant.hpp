// box_quant.hpp -- conservative fixed-point child boxes (host side).
//
// Scenes served from global memory cull a child of an inner KD node when the
// ray segment (0, best] misses the child's box (the node's region clipped to
// its triangles' bounds, KDTree.hpp:154-155).  A sibling-pair record carries
// both children's boxes in 16 B (the 32-B record: two node words, two boxes),
// so a box is 8 B: one 32-bit word per corner, x in bits 0-10, y in 11-21, z
// in 22-31 -- codes on a fixed grid over the KD root box,
//   coordinate = fma(code, sc[a], lo[a])        (one IEEE fma, single rounding)
// with 2047 steps on x and y and 1023 on z.  The min corner is rounded down
// (the largest code whose coordinate <= the exact one), the max corner up, so
// the stored box always contains the exact one and the cull stays exact.  On
// the C4 mesh (oracle, 3 x 128^2 x 4 spp) the grid costs +0.8% inner visits and
// +1.3% triangle tests against fp16 corners, which needed 12 B per box (48-B
// records, three 16-B loads per descent step instead of two).  The oracle
// restates the grid and the rounding bit for bit (oracle/render_ref.c).
#pragma once

#include <cmath>
#include <cstdint>

namespace mcpt {

constexpr uint32_t kBoxQMax[3] = {2047u, 2047u, 1023u};   // codes 0..max per axis
constexpr int kBoxQShift[3] = {0, 11, 22};

struct BoxGrid {
    float lo[3], sc[3];
};

inline float box_dec(const BoxGrid& g, int a, uint32_t q) { return std::fma(static_cast<float>(q), g.sc[a], g.lo[a]); }

// the grid over the root box [bmin, bmax]: sc the smallest float with
// fma(max, sc, lo) >= bmax, so the top code reaches the root's max face
inline BoxGrid box_grid(const float bmin[3], const float bmax[3]) {
    BoxGrid g;
    for (int a = 0; a < 3; ++a) {
        const float mq = static_cast<float>(kBoxQMax[a]);
        g.lo[a] = bmin[a];
        float sc = (bmax[a] - bmin[a]) / mq;
        if (!(sc > 0.0f)) sc = 0.0f;          // flat root box: every code decodes to lo
        while (sc > 0.0f && std::fma(mq, sc, bmin[a]) < bmax[a]) sc = std::nextafter(sc, INFINITY);
        g.sc[a] = sc;
    }
    return g;
}

// largest code whose coordinate is <= v (v inside the root box)
inline uint32_t box_q_down(const BoxGrid& g, int a, float v) {
    if (!(g.sc[a] > 0.0f)) return 0;
    const double x = std::floor((static_cast<double>(v) - g.lo[a]) / g.sc[a]);
    int64_t q = x < 0 ? 0 : (x > kBoxQMax[a] ? kBoxQMax[a] : static_cast<int64_t>(x));
    while (q > 0 && box_dec(g, a, static_cast<uint32_t>(q)) > v) --q;
    while (q < int64_t(kBoxQMax[a]) && box_dec(g, a, static_cast<uint32_t>(q + 1)) <= v) ++q;
    return static_cast<uint32_t>(q);
}
// smallest code whose coordinate is >= v
inline uint32_t box_q_up(const BoxGrid& g, int a, float v) {
    if (!(g.sc[a] > 0.0f)) return 0;
    const double x = std::ceil((static_cast<double>(v) - g.lo[a]) / g.sc[a]);
    int64_t q = x < 0 ? 0 : (x > kBoxQMax[a] ? kBoxQMax[a] : static_cast<int64_t>(x));
    while (q < int64_t(kBoxQMax[a]) && box_dec(g, a, static_cast<uint32_t>(q)) < v) ++q;
    while (q > 0 && box_dec(g, a, static_cast<uint32_t>(q - 1)) >= v) --q;
    return static_cast<uint32_t>(q);
}

// a box's two corner words (min rounded down, max rounded up)
inline void box_pack(const BoxGrid& g, const float bmin[3], const float bmax[3], uint32_t out[2]) {
    out[0] = out[1] = 0;
    for (int a = 0; a < 3; ++a) {
        out[0] |= box_q_down(g, a, bmin[a]) << kBoxQShift[a];
        out[1] |= box_q_up(g, a, bmax[a]) << kBoxQShift[a];
    }
}

}  // namespace mcpt
