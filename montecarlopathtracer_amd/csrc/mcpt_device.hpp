// mcpt_device.hpp -- device building blocks of the path kernel (gfx950).
//
// Arithmetic contract (DESIGN.md "Determinism spec"): every float expression
// keeps the reference's operand order and is compiled with -ffp-contract=off;
// division and sqrt are IEEE correctly rounded (HIP default); sin/cos are a
// fixed float sequence, pow a fixed double one and the Fresnel x^5 three double
// multiplies -- add/mul/div/floor and bit casts only -- so the HIP kernel
// reproduces the CPU specification bit for bit.
//
// Reference lines restated here:
//   det()                 CVMCTracer/Framework/Math.hpp:169-175
//   Cramer test           CVMCTracer/CUDA/CUTracer.cu:54-92
//   sampleHemi/Phong/Fresnel  CVMCTracer/CUDA/Utils.hpp:46-137
//   normalize()           CVMCTracer/CUDA/Utils.hpp:27-34
//   TEA-16 / Park-Miller  MCRT/QuinEngine/Shader/rtx.hlsl:61-82 (path seeds: PCG hash)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mcpt {
namespace dev {

constexpr float kPwPi = 3.14159265359f;         // CV/stdafx.h:46
constexpr float kFltEps = 1.192092896e-07f;     // FLT_EPSILON
constexpr float kFltMax = 3.402823466e+38f;     // FLT_MAX
constexpr float kEpsHi = 1.000244140625f;       // ordered-traversal margins, 1 +/- 2^-12
constexpr float kEpsLo = 0.999755859375f;

struct V3 {
    float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ float dot3(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 vscale(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 vdiv(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
// Same-denominator division, bit-identical to IEEE f32 a / d: the quotient is
// RN_f32(a * r) with r a double reciprocal of d within ~2^-52.  A float quotient
// that is not exact lies more than 2^-49 (relative) from every f32 rounding
// midpoint (a - d*m is a multiple of a grid step >= 2^-49 |a| for 24-bit a, d and
// 25-bit m, and never 0), so the double error cannot change the rounding
// (tests/test_div_shared.py, tests/test_gpu_math.py).
// r = v_rcp_f64 + two Newton steps (error <= ~2^-52; 0, inf, NaN reciprocals
// passed through, so a / 0 and a / inf keep IEEE results; the IEEE double
// 1 / d measured 1.9% slower on C2)
__device__ __forceinline__ double recip_shared(float d) {
    const double dd = (double)d;
    const double r0 = __builtin_amdgcn_rcp(dd);
    double e = __builtin_fma(-dd, r0, 1.0);
    const double r1 = __builtin_fma(r0, e, r0);
    e = __builtin_fma(-dd, r1, 1.0);
    const double r2 = __builtin_fma(r1, e, r1);
    return (__builtin_isfinite(r0) && r0 != 0.0) ? r2 : r0;
}
__device__ __forceinline__ float div_shared(float a, double r) { return (float)((double)a * r); }

__device__ __forceinline__ void normalize_cu(V3& v) {   // Utils.hpp:27-34
    float len = __builtin_sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    if (fabsf(len) > kFltEps) { const double r = recip_shared(len); v.x = div_shared(v.x, r); v.y = div_shared(v.y, r); v.z = div_shared(v.z, r); }
}
// HLSL normalize(v) = v / length(v) (the D3D definition), no epsilon guard:
// QuinEngine's shading normal, Fresnel output and primary ray (rtx.hlsl:250,
// 340, 395).  Division as IEEE (shared reciprocal, bit-identical); a zero
// vector gives NaN like 0 / 0.
__device__ __forceinline__ void normalize_hlsl(V3& v) {
    const float len = __builtin_sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    const double r = recip_shared(len);
    v.x = div_shared(v.x, r); v.y = div_shared(v.y, r); v.z = div_shared(v.z, r);
}
// __builtin_sqrtf is correctly rounded under HIP defaults; __fsqrt_rn is NOT on gfx950
// (measured: ~14% of inputs off by 1 ulp, tests/test_gpu_math.py).
__device__ __forceinline__ float sqrt_rn(float x) { return __builtin_sqrtf(x); }

// ---------------- deterministic transcendentals (double sequences) ----------
__device__ __forceinline__ uint64_t d2u(double x) { return __builtin_bit_cast(uint64_t, x); }
__device__ __forceinline__ double u2d(uint64_t u) { return __builtin_bit_cast(double, u); }

// sin and cos in float arithmetic only: Cody-Waite pi/2 reduction in three
// parts (exact for the samplers' [0, 2pi)), Cephes sinf/cosf minimax
// polynomials on [-pi/4, pi/4]; <= 2 ulp (sin) / 1 ulp (cos) against libm on
// [0, 2pi).  The earlier double-precision (fdlibm) sequences cost 2.6% of the
// C2 frame.  Oracle: mc_sincos_f.
__device__ __forceinline__ void sincos_f(float x, float& s, float& c) {
    const float k = __builtin_floorf(x * 0.636619772367581343f + 0.5f);
    const float r = ((x - k * 1.5703125f) - k * 4.837512969970703125e-4f) - k * 7.54978995489188216e-8f;
    const float z = r * r;
    const float sr = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r + r;
    const float cr = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z -
                     0.5f * z + 1.0f;
    const int q = (int)(k - 4.0f * __builtin_floorf(k * 0.25f));   // k mod 4, exact
    s = q == 0 ? sr : (q == 1 ? cr : (q == 2 ? -sr : -cr));
    c = q == 0 ? cr : (q == 1 ? -sr : (q == 2 ? -cr : sr));
}
// x^5 of the Fresnel term (Utils.hpp:101) in double, rounded once to float
// (x^2 exact in double): within 1 ulp, three multiplies instead of log/exp
__device__ __forceinline__ float pow5_f(float x) {
    const double d = (double)x, d2 = d * d;
    return (float)(d2 * d2 * d);
}
__device__ __forceinline__ double log2_d(double x) {
    uint64_t b = d2u(x);
    int e = (int)((b >> 52) & 0x7FF) - 1022;
    double m = u2d((b & 0x000FFFFFFFFFFFFFull) | 0x3FE0000000000000ull);
    if (m < 0.70710678118654752440) { m = m * 2.0; e = e - 1; }
    double f = (m - 1.0) / (m + 1.0);
    double f2 = f * f;
    double p = 4.34782608695652173913e-02;
    p = 4.76190476190476190476e-02 + f2 * p;
    p = 5.26315789473684210526e-02 + f2 * p;
    p = 5.88235294117647058824e-02 + f2 * p;
    p = 6.66666666666666666667e-02 + f2 * p;
    p = 7.69230769230769230769e-02 + f2 * p;
    p = 9.09090909090909090909e-02 + f2 * p;
    p = 1.11111111111111111111e-01 + f2 * p;
    p = 1.42857142857142857143e-01 + f2 * p;
    p = 2.00000000000000000000e-01 + f2 * p;
    p = 3.33333333333333333333e-01 + f2 * p;
    double ln_m = 2.0 * f * (1.0 + f2 * p);
    return (double)e + ln_m * 1.44269504088896340736;
}
__device__ __forceinline__ double exp2_d(double z) {
    if (z < -1000.0) return 0.0;
    if (z > 1000.0) return __builtin_huge_val();
    double k = __builtin_floor(z + 0.5);
    double f = z - k;
    double t = f * 6.93147180559945309417e-01;
    double p = 1.60590438368216145994e-10;
    p = 2.08767569878680989792e-09 + t * p;
    p = 2.50521083854417187751e-08 + t * p;
    p = 2.75573192239858906526e-07 + t * p;
    p = 2.75573192239858906526e-06 + t * p;
    p = 2.48015873015873015873e-05 + t * p;
    p = 1.98412698412698412698e-04 + t * p;
    p = 1.38888888888888888889e-03 + t * p;
    p = 8.33333333333333333333e-03 + t * p;
    p = 4.16666666666666666667e-02 + t * p;
    p = 1.66666666666666666667e-01 + t * p;
    p = 5.00000000000000000000e-01 + t * p;
    p = 1.0 + t * p;
    p = 1.0 + t * p;
    int ki = (int)k;
    double scale = u2d((uint64_t)(ki + 1023) << 52);
    return p * scale;
}
__device__ __forceinline__ float pow_f(float x, float y) {
    if (x == 0.0f) return 0.0f;
    if (x == 1.0f) return 1.0f;
    if (!(x > 0.0f)) return __builtin_nanf("");
    return (float)exp2_d((double)y * log2_d((double)x));
}

// ---------------------------------- RNG -------------------------------------
__device__ __forceinline__ uint32_t tea16(uint32_t v0, uint32_t v1) {   // rtx.hlsl:61-72
    uint32_t sum = 0;
#pragma unroll
    for (int n = 0; n < 16; n++) {
        sum += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + sum) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    return v0;
}
// PCG hash (Jarzynski & Olano, "Hash Functions for GPU Rendering", JCGT 9(3),
// 2020: the PCG RXS-M-XS output permutation of one LCG step -- a bijection of
// 32-bit words with good avalanche at ~6 integer ops, where TEA needs many of
// its 16 rounds for the same quality)
__device__ __forceinline__ uint32_t pcg_hash(uint32_t x) {
    const uint32_t st = x * 747796405u + 2891336453u;
    const uint32_t w = ((st >> ((st >> 28u) + 4u)) ^ st) * 277803737u;
    return (w >> 22u) ^ w;
}
// Park-Miller start state of sample `sample` of pixel `pixel` (CVMCTracer mode;
// DESIGN.md section 3): stateless per (pixel, sample), so every sharding,
// chunking and kernel structure draws the same stream
__device__ __forceinline__ uint32_t rng_init(uint32_t pixel, uint32_t key, uint32_t sample) {
    return 1u + pcg_hash(pcg_hash(pixel ^ key) + sample) % 0x7FFFFFFEu;
}
__device__ __forceinline__ float rng_next(uint32_t& sd) {   // rtx.hlsl:74-82
    uint32_t s = sd;
    s = 16807u * (s % 127773u) - 2836u * (s / 127773u);
    if (s > 0x7FFFFFFFu) s += 0x7FFFFFFFu;
    sd = s;
    return (float)s * 4.656612873077392578125e-10f;
}

// ------------------------------- samplers -----------------------------------
// Diffuse (Utils.hpp:46-70 sampleHemi) and Phong (Utils.hpp:72-95) in one
// body -- the y-up local lobe rotated into the normal frame -- for a wave that
// holds lanes of both materials: each lane draws its two uniforms and forms
// (cos, sin) of its own lobe, then the sincos, the lobe vector and the frame
// rotation -- the bulk of both samplers -- run once for all of them.  Per lane
// the operations are exactly its sampler's: the rotation's y term is
// d.z / invlen for Phong and d.z * (1 / invlen) for the hemisphere.
// Returns the rotated lobe vector (the hemisphere direction, or Phong's half
// vector before the reflection).
__device__ __forceinline__ V3 sample_lobe_u(float x, float y, V3 n, bool phong, float ns1) {
    float cosT, sinT;
    if (phong) {
        cosT = pow_f(x, 1.0f / ns1);
        sinT = sqrt_rn(1 - cosT * cosT);
    } else {
        sinT = sqrt_rn(x);
        cosT = sqrt_rn(1 - x);
    }
    float phi = 2 * kPwPi * y;
    float sp, cp;
    sincos_f(phi, sp, cp);
    V3 h = v3(sinT * cp, cosT, sinT * sp);
    if (fabsf(n.y + 1) < kFltEps) {
        h = v3(-h.x, -h.y, -h.z);
    } else if (fabsf(n.y - 1) >= kFltEps) {
        V3 d = h;
        float invlen = 1.0f / sqrt_rn(1.0f - n.y * n.y);
        const float q = (phong ? d.z : 1.0f) / invlen;
        h.x = (n.z * d.x + n.x * n.y * d.z) * invlen + n.x * d.y;
        h.y = n.y * d.y - (phong ? q : d.z * q);
        h.z = (-n.x * d.x + n.z * n.y * d.z) * invlen + n.z * d.y;
    }
    return h;
}
__device__ __forceinline__ V3 sample_lobe(uint32_t& sd, V3 n, bool phong, float ns1) {
    float x = rng_next(sd);
    float y = rng_next(sd);
    return sample_lobe_u(x, y, n, phong, ns1);
}
// Fresnel: CVMCTracer normalizes only the refracted directions (epsilon-guarded
// Utils.hpp:27-34; Utils.hpp:97-137); QuinEngine normalizes every output, the
// mirror and total-internal-reflection branches included (rtx.hlsl:213-251)
template <bool QE = false>
__device__ __forceinline__ V3 sample_fresnel_u(float x, V3 n, V3 in, float Tr, float Ni) {
    float ndoti = dot3(in, n);
    Tr = Tr * (1 - pow5_f(1 - fabsf(ndoti)));
    // Entering (ndoti <= 0) and leaving refraction in one body: each lane forms
    // its branch's alpha terms -- the entering branch's six divisions by Ni as
    // RN(a * r) with one shared reciprocal r of Ni (bit-identical to IEEE a / Ni,
    // see recip_shared) -- then one sqrt, one n*alpha + in' and one normalize.
    const bool enter = ndoti <= 0;
    const float w = 1 - ndoti * ndoti;
    float a0, rad;
    V3 ins;
    if (enter) {
        const double rn = recip_shared(Ni);
        a0 = div_shared(-ndoti, rn);                       // -ndoti / Ni
        rad = 1 - div_shared(div_shared(w, rn), rn);       // 1 - (1 - ndoti^2) / Ni / Ni
        ins = v3(div_shared(in.x, rn), div_shared(in.y, rn), div_shared(in.z, rn));   // in / Ni
    } else {
        a0 = -ndoti * Ni;
        rad = 1 - w * Ni * Ni;                             // `test`: < 0 is total internal reflection
        ins = vscale(in, Ni);
    }
    V3 out;
    if (x < Tr && (enter || !(rad < 0))) {
        const float sq = sqrt_rn(rad);
        const float alpha = enter ? a0 - sq : a0 + sq;
        out = vadd(vscale(n, alpha), ins);
        if constexpr (!QE) normalize_cu(out);
    } else {
        out = vsub(in, vscale(vscale(n, dot3(in, n)), 2.0f));
    }
    if constexpr (QE) normalize_hlsl(out);
    return out;
}
template <bool QE = false>
__device__ __forceinline__ V3 sample_fresnel(uint32_t& sd, V3 n, V3 in, float Tr, float Ni) {
    float x = rng_next(sd);
    return sample_fresnel_u<QE>(x, n, in, Tr, Ni);
}

// -------------------------- ray / triangle ----------------------------------
__device__ __forceinline__ float det3(float m0, float m1, float m2, float m3, float m4, float m5,
                                      float m6, float m7, float m8) {   // Math.hpp:169-175
    float res1 = m0 * (m4 * m8 - m5 * m7);
    float res2 = -m1 * (m3 * m8 - m5 * m6);
    float res3 = m2 * (m3 * m7 - m4 * m6);
    return res1 + res2 + res3;
}

// det3 with its last minor (m3 * m7 - m4 * m6) supplied precomputed
__device__ __forceinline__ float det3_m(float m0, float m1, float m2, float m3, float m4, float m5,
                                        float m6, float m7, float m8, float minor_3746) {
    float res1 = m0 * (m4 * m8 - m5 * m7);
    float res2 = -m1 * (m3 * m8 - m5 * m6);
    float res3 = m2 * minor_3746;
    return res1 + res2 + res3;
}

}  // namespace dev
}  // namespace mcpt
