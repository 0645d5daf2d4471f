// leaf_box.hpp -- leaf boxes packed into the leaf node words of 8-B node
// images (scenes whose image the walk reads from LDS; host side).
//
// A leaf's node word is 64 bits, and the walk needs only the leaf flag
// (3 << 30), the first leaf ref and the count: the bits left over carry the
// leaf's KD box (its region clipped to its triangles' bounds,
// KDTree.hpp:154-155) as six codes of qb bits on a grid over the KD root box,
//   coordinate = fma(code, sc[a], lo[a])       (one IEEE fma, single rounding)
// min corner rounded down, max corner up, so the stored box contains the
// exact one.  A ray reaching a leaf tests the segment (0, best] against it
// (the child-box cull's slab test, trace_device.hpp box_hit) and skips the
// leaf's refs and triangles when it misses: exact, since a hit that could
// improve `best` lies inside the box.  scene01 (oracle, 4 x 128^2 x 4 spp of
// the 1024^2 frame): triangle tests per ray 8.96 -> 3.06 with 7-bit codes
// (2.66 with exact boxes, 3.35 with 6 bits).  No LDS byte is added.
//   w0 = 3 << 30 | y_hi << (30 - qb) | z_hi ... see leaf_word below;
//   w1 = x_lo | y_lo << qb | z_lo << 2qb | x_hi << 3qb
// with rb = bits of the ref count and cb = bits of the largest leaf count
// (the oracle, oracle/render_ref.c, restates the packing bit for bit).
#pragma once

#include <cmath>
#include <cstdint>

#include "host_model.hpp"

namespace mcpt {

struct LeafBoxPack {
    uint32_t qb = 0, rb = 0, cb = 0;     // box bits per coordinate (0: none), first-ref bits, count bits
    float lo[3] = {0, 0, 0}, sc[3] = {0, 0, 0};
};

inline uint32_t bit_length(uint32_t x) {
    uint32_t n = 0;
    while (x) { ++n; x >>= 1; }
    return n;
}

inline float leaf_dec(const LeafBoxPack& p, int a, uint32_t q) {
    return std::fma(static_cast<float>(q), p.sc[a], p.lo[a]);
}

// the packing for a scene: qb = min(8, (30 - rb - cb) / 2) (four codes in w1,
// two in w0 above the ref and count); qb < 4 turns the cull off
inline LeafBoxPack leaf_box_pack(const HostScene& hs) {
    LeafBoxPack p;
    if (hs.nodes.empty()) return p;
    uint32_t maxc = 0;
    for (const KdNode& n : hs.nodes)
        if (!n.axis && n.leaf_count > maxc) maxc = n.leaf_count;
    p.rb = bit_length(static_cast<uint32_t>(hs.leaf_ids.size()));
    p.cb = bit_length(maxc);
    if (p.rb + p.cb > 22) return LeafBoxPack{};
    const uint32_t qb = (30u - p.rb - p.cb) / 2u;
    p.qb = qb > 8u ? 8u : qb;
    const float mq = static_cast<float>((1u << p.qb) - 1u);
    for (int a = 0; a < 3; ++a) {
        const float lo = hs.nodes[0].bmin[a], hi = hs.nodes[0].bmax[a];
        float sc = (hi - lo) / mq;
        if (!(sc > 0.0f)) sc = 0.0f;                       // flat root box: every code decodes to lo
        while (sc > 0.0f && std::fma(mq, sc, lo) < hi) sc = std::nextafter(sc, INFINITY);
        p.lo[a] = lo;
        p.sc[a] = sc;
    }
    return p;
}

// largest code whose coordinate is <= v (dir < 0), smallest whose coordinate is >= v (dir > 0)
inline uint32_t leaf_q(const LeafBoxPack& p, int a, float v, int dir) {
    const int64_t mx = (int64_t(1) << p.qb) - 1;
    if (!(p.sc[a] > 0.0f)) return 0;
    double x = (static_cast<double>(v) - p.lo[a]) / p.sc[a];
    x = dir < 0 ? std::floor(x) : std::ceil(x);
    int64_t q = x < 0 ? 0 : (x > double(mx) ? mx : static_cast<int64_t>(x));
    if (dir < 0) {
        while (q > 0 && leaf_dec(p, a, static_cast<uint32_t>(q)) > v) --q;
        while (q < mx && leaf_dec(p, a, static_cast<uint32_t>(q + 1)) <= v) ++q;
    } else {
        while (q < mx && leaf_dec(p, a, static_cast<uint32_t>(q)) < v) ++q;
        while (q > 0 && leaf_dec(p, a, static_cast<uint32_t>(q - 1)) >= v) --q;
    }
    return static_cast<uint32_t>(q);
}

// the packed leaf word of a leaf with refs [first, first + count) and box [bmin, bmax]
inline void leaf_word(const LeafBoxPack& p, uint32_t first, uint32_t count, const float bmin[3], const float bmax[3],
                      uint32_t w[2]) {
    const uint32_t q = p.qb;
    const uint32_t xl = leaf_q(p, 0, bmin[0], -1), yl = leaf_q(p, 1, bmin[1], -1), zl = leaf_q(p, 2, bmin[2], -1);
    const uint32_t xh = leaf_q(p, 0, bmax[0], +1), yh = leaf_q(p, 1, bmax[1], +1), zh = leaf_q(p, 2, bmax[2], +1);
    w[0] = (3u << 30) | (zh << (30 - q)) | (yh << (30 - 2 * q)) | (count << p.rb) | first;
    w[1] = xl | (yl << q) | (zl << (2 * q)) | (xh << (3 * q));
}

}  // namespace mcpt
