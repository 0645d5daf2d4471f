// half_box.hpp -- conservative fp16 leaf boxes (host side).
//
// Scenes served from global memory cull a KD leaf before testing its
// triangles when the ray misses the leaf's box (the node AABB of the KD build:
// its region clipped to its triangles' bounds, KDTree.hpp:154-155).  The box
// is stored as IEEE binary16 rounded outward -- min toward -inf, max toward
// +inf -- so it always contains the exact box; the oracle restates the same
// conversion (oracle/render_ref.c, orc_f16_dir) bit for bit.
#pragma once

#include <cstdint>
#include <cstring>

namespace mcpt {

inline float f16_bits_to_f32(uint16_t h) {
    const uint32_t s = (h >> 15) & 1u, e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
    if (e == 0) {
        const float v = static_cast<float>(m) * 5.9604644775390625e-8f;   // m * 2^-24, exact
        return s ? -v : v;
    }
    uint32_t bits;
    if (e == 31) bits = (s << 31) | 0x7F800000u | (m << 13);
    else bits = (s << 31) | ((e - 15u + 127u) << 23) | (m << 13);
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
}

// binary16 of x rounded toward -inf (dir < 0) or +inf (dir > 0)
inline uint16_t f32_to_f16_dir(float x, int dir) {
    uint32_t u;
    std::memcpy(&u, &x, 4);
    const uint32_t sign = u >> 31;
    float a = x < 0 ? -x : x;
    uint32_t mag;                                   // magnitude, truncated toward zero
    if (!(a < 65520.0f)) {                          // beyond the largest finite: +-inf
        mag = 0x7C00u;
    } else if (a < 6.103515625e-05f) {              // below 2^-14: subnormal grid 2^-24
        mag = static_cast<uint32_t>(a * 16777216.0f);   // exact scaling, truncation
    } else {
        uint32_t ua;
        std::memcpy(&ua, &a, 4);
        const uint32_t e = (ua >> 23) - 127u + 15u;
        mag = (e << 10) | ((ua >> 13) & 0x3FFu);
        if (mag > 0x7BFFu) mag = 0x7BFFu;
    }
    const bool up_magnitude = (sign ? dir < 0 : dir > 0);
    if (mag < 0x7C00u && f16_bits_to_f32(static_cast<uint16_t>(mag)) != a && up_magnitude) mag += 1u;
    if (mag >= 0x7C00u && !up_magnitude) mag = 0x7BFFu;     // toward zero: largest finite
    if (mag == 0 && sign) return static_cast<uint16_t>(0x8000u);
    return static_cast<uint16_t>((sign << 15) | mag);
}

}  // namespace mcpt
