/*
 * render_ref.c -- oracle restatement of the reference per-pixel path tracer.
 * TEST INFRASTRUCTURE ONLY (see mcpt_oracle.h).
 *
 *   closest hit, brute force  CV/CUDA/CUTracer.cu:44-96, det() Math.hpp:169-175
 *   closest hit, KD (ref)     QE/Shader/rtx.hlsl:84-211 with CV's Cramer test
 *   closest hit, KD (ordered) the HIP kernel's traversal order
 *   samplers                  CV/CUDA/Utils.hpp:46-137
 *   path loop                 CV/CUDA/CUTracer.cu:98-177
 *   primary ray, accumulate   CV/CUDA/CUTracer.cu:179-218
 *   camera basis              CV/CUDA/CUTracer.cu:347-374, Math.hpp Vector3f
 * Every float expression keeps the reference's operand order; the library is
 * compiled with -ffp-contract=off and without -ffast-math.
 */
#include "oracle_internal.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define PW_PI 3.14159265359f        /* CV/stdafx.h:46 */
#define KD_EPS_HI 1.000244140625f   /* 1 + 2^-12 : ordered-traversal margins */
#define KD_EPS_LO 0.999755859375f   /* 1 - 2^-12 */

/* ======================= deterministic transcendentals ===================== */
/* The same operation sequences are compiled into the HIP kernel
 * (montecarlopathtracer_amd/csrc/mcpt_device.hpp); only IEEE add/mul/div,
 * floor and bit casts are used, so CPU and GPU agree bitwise.               */
static inline uint64_t d2u(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline double u2d(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

/* sin and cos in float arithmetic only: Cody-Waite pi/2 reduction in three
 * parts (exact for the samplers' [0, 2pi)), Cephes sinf/cosf minimax
 * polynomials on [-pi/4, pi/4].  <= 2 ulp (sin) / 1 ulp (cos) against libm
 * on [0, 2pi); mcpt_device.hpp sincos_f performs the same float operations. */
static void mc_sincos_f(float x, float* s, float* c) {
    const float k = floorf(x * 0.636619772367581343f + 0.5f);
    const float r = ((x - k * 1.5703125f) - k * 4.837512969970703125e-4f) - k * 7.54978995489188216e-8f;
    const float z = r * r;
    const float sr = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r + r;
    const float cr = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z -
                     0.5f * z + 1.0f;
    const int q = (int)(k - 4.0f * floorf(k * 0.25f));   /* k mod 4, exact */
    if (q == 0) { *s = sr; *c = cr; }
    else if (q == 1) { *s = cr; *c = -sr; }
    else if (q == 2) { *s = -sr; *c = -cr; }
    else { *s = -cr; *c = sr; }
}
float orc_sinf(float x) { float s, c; mc_sincos_f(x, &s, &c); return s; }
float orc_cosf(float x) { float s, c; mc_sincos_f(x, &s, &c); return c; }
/* x^5 of the Fresnel term (Utils.hpp:101) in double, rounded once to float:
 * x^2 is exact in double, so the result is within 1 ulp (mcpt_device.hpp pow5_f) */
float orc_pow5f(float x) {
    const double d = (double)x, d2 = d * d;
    return (float)(d2 * d2 * d);
}

static double mc_log2_d(double x) {   /* x: positive finite (from a float) */
    uint64_t b = d2u(x);
    int e = (int)((b >> 52) & 0x7FF) - 1022;
    double m = u2d((b & 0x000FFFFFFFFFFFFFull) | 0x3FE0000000000000ull);   /* [0.5,1) */
    if (m < 0.70710678118654752440) { m = m * 2.0; e = e - 1; }
    double f = (m - 1.0) / (m + 1.0);
    double f2 = f * f;
    double p = 4.34782608695652173913e-02;                 /* 1/23 */
    p = 4.76190476190476190476e-02 + f2 * p;               /* 1/21 */
    p = 5.26315789473684210526e-02 + f2 * p;               /* 1/19 */
    p = 5.88235294117647058824e-02 + f2 * p;               /* 1/17 */
    p = 6.66666666666666666667e-02 + f2 * p;               /* 1/15 */
    p = 7.69230769230769230769e-02 + f2 * p;               /* 1/13 */
    p = 9.09090909090909090909e-02 + f2 * p;               /* 1/11 */
    p = 1.11111111111111111111e-01 + f2 * p;               /* 1/9  */
    p = 1.42857142857142857143e-01 + f2 * p;               /* 1/7  */
    p = 2.00000000000000000000e-01 + f2 * p;               /* 1/5  */
    p = 3.33333333333333333333e-01 + f2 * p;               /* 1/3  */
    double ln_m = 2.0 * f * (1.0 + f2 * p);
    return (double)e + ln_m * 1.44269504088896340736;
}
static double mc_exp2_d(double z) {
    if (z < -1000.0) return 0.0;
    if (z > 1000.0) return INFINITY;
    double k = floor(z + 0.5);
    double f = z - k;                                       /* [-0.5, 0.5] */
    double t = f * 6.93147180559945309417e-01;
    double p = 1.60590438368216145994e-10;                  /* 1/13! */
    p = 2.08767569878680989792e-09 + t * p;                 /* 1/12! */
    p = 2.50521083854417187751e-08 + t * p;                 /* 1/11! */
    p = 2.75573192239858906526e-07 + t * p;                 /* 1/10! */
    p = 2.75573192239858906526e-06 + t * p;                 /* 1/9!  */
    p = 2.48015873015873015873e-05 + t * p;                 /* 1/8!  */
    p = 1.98412698412698412698e-04 + t * p;                 /* 1/7!  */
    p = 1.38888888888888888889e-03 + t * p;                 /* 1/6!  */
    p = 8.33333333333333333333e-03 + t * p;                 /* 1/5!  */
    p = 4.16666666666666666667e-02 + t * p;                 /* 1/4!  */
    p = 1.66666666666666666667e-01 + t * p;                 /* 1/3!  */
    p = 5.00000000000000000000e-01 + t * p;                 /* 1/2!  */
    p = 1.0 + t * p;
    p = 1.0 + t * p;
    int ki = (int)k;
    double scale = u2d((uint64_t)(ki + 1023) << 52);
    return p * scale;
}
float orc_powf(float x, float y) {
    if (x == 0.0f) return 0.0f;           /* y > 0 on every call site */
    if (x == 1.0f) return 1.0f;
    if (!(x > 0.0f)) return NAN;
    return (float)mc_exp2_d((double)y * mc_log2_d((double)x));
}

/* ================================ RNG ===================================== */
/* QE/Shader/rtx.hlsl:61-72 */
uint32_t orc_tea16(uint32_t v0, uint32_t v1) {
    uint32_t sum = 0;
    for (int n = 0; n < 16; n++) {
        sum += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + sum) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    return v0;
}
uint32_t orc_seed_key(uint64_t seed) { return orc_tea16((uint32_t)seed, (uint32_t)(seed >> 32)); }
/* Path seed of CVMCTracer mode (our determinism spec; the
 * reference seeds irreproducible cuRAND streams, CUTracer.cu:186-187): PCG hash
 * of (pixel ^ key) then of that + sample (Jarzynski & Olano, "Hash Functions for
 * GPU Rendering", JCGT 9(3) 2020), onto the Park-Miller range [1, 2^31 - 2] */
uint32_t orc_pcg_hash(uint32_t x) {
    uint32_t st = x * 747796405u + 2891336453u;
    uint32_t w = ((st >> ((st >> 28u) + 4u)) ^ st) * 277803737u;
    return (w >> 22u) ^ w;
}
uint32_t orc_rng_init(uint32_t pixel, uint32_t key, uint32_t sample) {
    return 1u + orc_pcg_hash(orc_pcg_hash(pixel ^ key) + sample) % 0x7FFFFFFEu;
}
/* QE/Shader/rtx.hlsl:74-82 (Park-Miller via Schrage); u = float(sd) / 2^31 */
float orc_rng_next(uint32_t* sd) {
    uint32_t s = *sd;
    s = 16807u * (s % 127773u) - 2836u * (s / 127773u);
    if (s > 0x7FFFFFFFu) s += 0x7FFFFFFFu;
    *sd = s;
    return (float)s * 4.656612873077392578125e-10f;
}

/* uniform source: Park-Miller stream or injected list (known-answer tests) */
typedef struct { uint32_t sd; const float* inj; int k; } usrc;
static inline float next_u(usrc* u) {
    if (u->inj) return u->inj[u->k++];
    return orc_rng_next(&u->sd);
}

/* ============================ vector helpers ============================== */
static inline orc_v3 v3(float x, float y, float z) { orc_v3 r = {x, y, z}; return r; }
static inline float dot3(orc_v3 a, orc_v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }   /* Utils.hpp:12-15 */
static inline orc_v3 vscale(orc_v3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline orc_v3 vadd(orc_v3 a, orc_v3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline orc_v3 vsub(orc_v3 a, orc_v3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline orc_v3 vdiv(orc_v3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
static inline void normalize_cu(orc_v3* v) {   /* Utils.hpp:27-34 */
    float len = sqrtf(v->x * v->x + v->y * v->y + v->z * v->z);
    if (fabsf(len) > FLT_EPSILON) { v->x /= len; v->y /= len; v->z /= len; }
}
/* HLSL normalize(v) = v / length(v), no epsilon guard (rtx.hlsl:250, 340, 395) */
static inline void normalize_hlsl(orc_v3* v) {
    float len = sqrtf(v->x * v->x + v->y * v->y + v->z * v->z);
    v->x /= len; v->y /= len; v->z /= len;
}

/* ============================== samplers =================================== */
/* Utils.hpp:46-70 */
static orc_v3 sample_hemi(usrc* u, orc_v3 n) {
    float x = next_u(u);
    float y = next_u(u);
    float sinT = sqrtf(x);
    float cosT = sqrtf(1 - x);
    float phi = 2 * PW_PI * y;
    orc_v3 out = v3(sinT * orc_cosf(phi), cosT, sinT * orc_sinf(phi));
    if (fabsf(n.y + 1) < FLT_EPSILON) {
        out = v3(-out.x, -out.y, -out.z);
    } else if (fabsf(n.y - 1) >= FLT_EPSILON) {
        orc_v3 d = out;
        float invlen = 1.0f / sqrtf(1.0f - n.y * n.y);
        float len = 1.0f / invlen;
        out.x = (n.z * d.x + n.x * n.y * d.z) * invlen + n.x * d.y;
        out.y = n.y * d.y - d.z * len;
        out.z = (-n.x * d.x + n.z * n.y * d.z) * invlen + n.z * d.y;
    }
    return out;
}
/* Utils.hpp:72-95 / rtx.hlsl:253-276.  ns1 = "Ns + 1" in the caller's type:
 * CVMCTracer passes Ns as unsigned int, (float)(Ns + 1u); QuinEngine keeps the
 * float, Ns + 1.0f */
static orc_v3 sample_phong(usrc* u, orc_v3 n, orc_v3 in, float ns1) {
    float x = next_u(u);
    float y = next_u(u);
    float cosT = orc_powf(x, 1.0f / ns1);
    float sinT = sqrtf(1 - cosT * cosT);
    float phi = 2 * PW_PI * y;
    orc_v3 h = v3(sinT * orc_cosf(phi), cosT, sinT * orc_sinf(phi));
    if (fabsf(n.y + 1) < FLT_EPSILON) {
        h = v3(-h.x, -h.y, -h.z);
    } else if (fabsf(n.y - 1) >= FLT_EPSILON) {
        orc_v3 d = h;
        float invlen = 1.0f / sqrtf(1.0f - n.y * n.y);
        h.x = (n.z * d.x + n.x * n.y * d.z) * invlen + n.x * d.y;
        h.y = n.y * d.y - d.z / invlen;
        h.z = (-n.x * d.x + n.z * n.y * d.z) * invlen + n.z * d.y;
    }
    return vsub(in, vscale(vscale(h, dot3(in, h)), 2));
}
/* Utils.hpp:97-137 (qe = 0): only the refracted directions are normalized
 * (epsilon-guarded); rtx.hlsl:213-251 (qe = 1): every output goes through
 * HLSL normalize, the mirror and total-internal-reflection branches included */
static orc_v3 sample_fresnel(usrc* u, orc_v3 n, orc_v3 in, float Tr, float Ni, int qe) {
    float x = next_u(u);
    orc_v3 out;
    float ndoti = dot3(in, n);
    Tr = Tr * (1 - orc_pow5f(1 - fabsf(ndoti)));
    if (x < Tr) {
        if (ndoti <= 0) {
            float alpha = -ndoti / Ni - sqrtf(1 - (1 - ndoti * ndoti) / Ni / Ni);
            out = vadd(vscale(n, alpha), vdiv(in, Ni));
            if (!qe) normalize_cu(&out);
        } else {
            float test = 1 - (1 - ndoti * ndoti) * Ni * Ni;
            if (test < 0) {
                out = vsub(in, vscale(vscale(n, dot3(in, n)), 2));
            } else {
                float alpha = -ndoti * Ni + sqrtf(test);
                out = vadd(vscale(n, alpha), vscale(in, Ni));
                if (!qe) normalize_cu(&out);
            }
        }
    } else {
        out = vsub(in, vscale(vscale(n, dot3(in, n)), 2));
    }
    if (qe) normalize_hlsl(&out);
    return out;
}

void orc_sample_hemi(const float* n, const float* u, float* out) {
    usrc s = {0, u, 0};
    orc_v3 r = sample_hemi(&s, v3(n[0], n[1], n[2]));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
void orc_sample_phong(const float* n, const float* in, uint32_t Ns, const float* u, float* out) {
    usrc s = {0, u, 0};
    orc_v3 r = sample_phong(&s, v3(n[0], n[1], n[2]), v3(in[0], in[1], in[2]), (float)(Ns + 1u));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
void orc_sample_fresnel(const float* n, const float* in, float Tr, float Ni, const float* u, float* out) {
    usrc s = {0, u, 0};
    orc_v3 r = sample_fresnel(&s, v3(n[0], n[1], n[2]), v3(in[0], in[1], in[2]), Tr, Ni, 0);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
/* QuinEngine samplers (rtx.hlsl:213-276): float Ns, normalized Fresnel output */
void orc_sample_phong_qe(const float* n, const float* in, float Ns, const float* u, float* out) {
    usrc s = {0, u, 0};
    orc_v3 r = sample_phong(&s, v3(n[0], n[1], n[2]), v3(in[0], in[1], in[2]), Ns + 1.0f);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
void orc_sample_fresnel_qe(const float* n, const float* in, float Tr, float Ni, const float* u, float* out) {
    usrc s = {0, u, 0};
    orc_v3 r = sample_fresnel(&s, v3(n[0], n[1], n[2]), v3(in[0], in[1], in[2]), Tr, Ni, 1);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

/* ========================= camera (CUTracer.cu:347-374) =================== */
static orc_v3 m_normal(orc_v3 v) {   /* Math::Vector3f::normal(): v / fmax(len, FLT_MIN) */
    float len = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    return vdiv(v, fmaxf(len, FLT_MIN));
}
static orc_v3 m_cross(orc_v3 a, orc_v3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
void orc_camera_basis(const float* eye, const float* dir, const float* up,
                      float* fwd_out, float* up_out, float* right_out) {
    (void)eye;
    orc_v3 d = m_normal(v3(dir[0], dir[1], dir[2]));      /* dir.normalize() */
    orc_v3 u = v3(up[0], up[1], up[2]);
    orc_v3 r = m_normal(m_cross(d, u));
    u = m_normal(m_cross(r, d));
    fwd_out[0] = d.x; fwd_out[1] = d.y; fwd_out[2] = d.z;
    up_out[0] = u.x; up_out[1] = u.y; up_out[2] = u.z;
    right_out[0] = r.x; right_out[1] = r.y; right_out[2] = r.z;
}
/* tan(projFOV * PW_PI / 360) (CUTracer.cu:189,202): float argument, tan in double, rounded */
float orc_tan_half_fov(float fov_deg) {
    float a = fov_deg * PW_PI / 360;
    return (float)tan((double)a);
}
/* yScale = cot(fovY/2), xScale = yScale / aspect (D3DXMatrixPerspectiveFovRH) */
void orc_qe_proj(float fovy_deg, int32_t width, int32_t height, float* p11, float* p22) {
    float a = fovy_deg * PW_PI / 360;
    float ys = (float)(1.0 / tan((double)a));
    *p22 = ys;
    *p11 = ys / ((float)width / (float)height);
}

/* ======================== closest-hit queries ============================= */
float orc_det3(const float* m) {   /* Math.hpp:169-175 */
    float res1 = m[0] * (m[4] * m[8] - m[5] * m[7]);
    float res2 = -m[1] * (m[3] * m[8] - m[5] * m[6]);
    float res3 = m[2] * (m[3] * m[7] - m[4] * m[6]);
    return res1 + res2 + res3;
}

typedef struct {
    int tri;      /* kd id, -1 miss */
    int geom;
    float beta, gamma, t;
    orc_v3 hp;
} hit_t;

/* Diagnostic hooks of the ordered walk and the path loop: no-ops here;
 * scripts/price_descent.c defines them to price traversal changes on the
 * oracle's exact visit sequence (test/diagnostic infrastructure only). */
#ifndef ORC_DIAG_FIELDS
#define ORC_DIAG_FIELDS
#define ORC_DIAG_RAY_BEGIN(q) do {} while (0)
#define ORC_DIAG_INNER(q, node) do {} while (0)
#define ORC_DIAG_LEAF(q, node) do {} while (0)
#define ORC_DIAG_POP(q) do {} while (0)
#define ORC_DIAG_ACCEPT(q, node) do {} while (0)
#define ORC_DIAG_AFTER_ISECT(q, depth) do {} while (0)
#endif

typedef struct {
    const orc_scene* s;
    const orc_v3 (*kv)[3];   /* vertices by kd id */
    int traversal;
    int node_boxes;          /* ordered walk: fp16 child-box cull */
    float best_init;         /* FLT_MAX (CUTracer.cu:46); 10000 in QE mode (rtx.hlsl:88) */
    orc_counters c;
    ORC_DIAG_FIELDS
} qctx;

/* CUTracer.cu:54-92: Cramer test of one triangle against the running tmin */
static inline int tri_test(const orc_v3* v, orc_v3 o, orc_v3 d, float* tmin, hit_t* h, int tri, int geom,
                           uint32_t prio, uint32_t* best_prio) {
    orc_v3 a = v[0], b = v[1], c = v[2];
    float betaM[9] = {a.x - o.x, a.x - c.x, d.x, a.y - o.y, a.y - c.y, d.y, a.z - o.z, a.z - c.z, d.z};
    float gammaM[9] = {a.x - b.x, a.x - o.x, d.x, a.y - b.y, a.y - o.y, d.y, a.z - b.z, a.z - o.z, d.z};
    float tM[9] = {a.x - b.x, a.x - c.x, a.x - o.x, a.y - b.y, a.y - c.y, a.y - o.y, a.z - b.z, a.z - c.z, a.z - o.z};
    float A[9] = {a.x - b.x, a.x - c.x, d.x, a.y - b.y, a.y - c.y, d.y, a.z - b.z, a.z - c.z, d.z};
    float detA = orc_det3(A);
    float beta = orc_det3(betaM) / detA;
    float gamma = orc_det3(gammaM) / detA;
    float t = orc_det3(tM) / detA;
    /* strict t < tmin (CUTracer.cu:82); exact ties resolved like the brute-force
     * loop order, i.e. lowest (geometry map order, index) rank wins          */
    if (beta + gamma < 1 && beta > 0 && gamma > 0 && t > 0 &&
        (t < *tmin || (t == *tmin && prio < *best_prio))) {
        *tmin = t;
        *best_prio = prio;
        h->tri = tri;
        h->geom = geom;
        h->beta = beta;
        h->gamma = gamma;
        h->t = t;
        h->hp.x = o.x + t * d.x;
        h->hp.y = o.y + t * d.y;
        h->hp.z = o.z + t * d.z;
        return 1;
    }
    return 0;
}

/* CUTracer.cu:44-96: every geometry, every triangle, strict t < tmin */
static hit_t isect_brute(qctx* q, orc_v3 o, orc_v3 d) {
    const orc_scene* s = q->s;
    hit_t h;
    memset(&h, 0, sizeof h);
    h.tri = -1; h.geom = -1;
    float tmin = q->best_init;
    for (int g = 0; g < s->ngeoms; g++) {
        uint32_t off = s->geoms[g].start;
        for (uint32_t i = 0; i < s->geoms[g].count; i++) {
            int cv = (int)(i + off);
            orc_v3 vv[3];
            const orc_tri* t = &s->model.tris[cv];
            vv[0] = s->model.verts[t->v[0]]; vv[1] = s->model.verts[t->v[1]]; vv[2] = s->model.verts[t->v[2]];
            q->c.tri_tests++;
            uint32_t bp = 0;   /* brute force: ties keep the first (prio 0 never beats) */
            tri_test(vv, o, d, &tmin, &h, cv, g, 0xFFFFFFFFu, &bp);
        }
    }
    return h;   /* h.tri is a CV index here; mapped by caller */
}

/* rtx.hlsl:84-142 */
static int aabb_ref(const orc_node* nd, orc_v3 from, orc_v3 dir, float curt) {
    float x_a = 1.0f / dir.x, y_a = 1.0f / dir.y, z_a = 1.0f / dir.z;
    if (dir.x == 0 && (from.x < nd->bmin[0] || from.x > nd->bmax[0])) return 0;
    if (dir.y == 0 && (from.y < nd->bmin[1] || from.y > nd->bmax[1])) return 0;
    if (dir.z == 0 && (from.z < nd->bmin[2] || from.z > nd->bmax[2])) return 0;
    float t_xmin, t_xmax, t_ymin, t_ymax, t_zmin, t_zmax;
    if (x_a >= 0) { t_xmin = (nd->bmin[0] - from.x) * x_a; t_xmax = (nd->bmax[0] - from.x) * x_a; }
    else { t_xmin = (nd->bmax[0] - from.x) * x_a; t_xmax = (nd->bmin[0] - from.x) * x_a; }
    if (y_a >= 0) { t_ymin = (nd->bmin[1] - from.y) * y_a; t_ymax = (nd->bmax[1] - from.y) * y_a; }
    else { t_ymin = (nd->bmax[1] - from.y) * y_a; t_ymax = (nd->bmin[1] - from.y) * y_a; }
    if (z_a >= 0) { t_zmin = (nd->bmin[2] - from.z) * z_a; t_zmax = (nd->bmax[2] - from.z) * z_a; }
    else { t_zmin = (nd->bmax[2] - from.z) * z_a; t_zmax = (nd->bmin[2] - from.z) * z_a; }
    float t_min = fmaxf(t_xmin, fmaxf(t_ymin, t_zmin));
    float t_max = fminf(t_xmax, fminf(t_ymax, t_zmax));
    return t_min <= t_max && t_min <= curt;
}

/* rtx.hlsl:144-211 (push left then right; no near-first order) */
static hit_t isect_kd_ref(qctx* q, orc_v3 o, orc_v3 d) {
    const orc_scene* s = q->s;
    hit_t h;
    memset(&h, 0, sizeof h);
    h.tri = -1; h.geom = -1;
    float tmin = q->best_init;
    uint32_t bprio = 0xFFFFFFFFu;
    uint32_t stack[96];
    int top = 0;
    stack[top++] = 0;
    while (top) {
        uint32_t ni = stack[--top];
        const orc_node* nd = &s->nodes[ni];
        if (nd->axis) q->c.inner_visits++; else q->c.leaf_visits++;
        if (!aabb_ref(nd, o, d, tmin)) continue;
        if (nd->axis == 0) {
            for (uint32_t i = 0; i < nd->tri_count; i++) {
                uint32_t k = s->leaf_ids[nd->tri_begin + i];
                q->c.leaf_refs++;
                q->c.tri_tests++;
                tri_test(q->kv[k], o, d, &tmin, &h, (int)k, s->tri_geom[s->kd_tris[k]], s->kd_prio[k], &bprio);
            }
        } else {
            stack[top++] = nd->left;
            stack[top++] = nd->right;
        }
    }
    return h;
}

/* Ordered front-to-back traversal used by the HIP kernel:
 * split-plane intervals, conservative 2^-12 margins, full stack (<= depth). */

/* ====================== fp16 leaf boxes (kernel mirror) =================== */
float orc_f16_to_f32(uint16_t h) {
    uint32_t sg = (h >> 15) & 1u, e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
    if (e == 0) {
        float v = (float)m * 5.9604644775390625e-8f;
        return sg ? -v : v;
    }
    uint32_t bits = e == 31 ? ((sg << 31) | 0x7F800000u | (m << 13)) : ((sg << 31) | ((e - 15u + 127u) << 23) | (m << 13));
    float f;
    memcpy(&f, &bits, 4);
    return f;
}
uint16_t orc_f16_dir(float x, int dir) {
    uint32_t u;
    memcpy(&u, &x, 4);
    uint32_t sg = u >> 31, mag;
    float a = x < 0 ? -x : x;
    if (!(a < 65520.0f)) {
        mag = 0x7C00u;
    } else if (a < 6.103515625e-05f) {
        mag = (uint32_t)(a * 16777216.0f);
    } else {
        uint32_t ua;
        memcpy(&ua, &a, 4);
        mag = (((ua >> 23) - 127u + 15u) << 10) | ((ua >> 13) & 0x3FFu);
        if (mag > 0x7BFFu) mag = 0x7BFFu;
    }
    int up = sg ? dir < 0 : dir > 0;
    if (mag < 0x7C00u && orc_f16_to_f32((uint16_t)mag) != a && up) mag += 1u;
    if (mag >= 0x7C00u && !up) mag = 0x7BFFu;
    if (mag == 0 && sg) return (uint16_t)0x8000u;
    return (uint16_t)((sg << 15) | mag);
}
/* does the ray segment (0, best] meet the node's fp16 box?  (trace_device.hpp box_hit) */
static int box_hit(const orc_node* nd, const float* oo, const float* dd, const float* inv, float best) {
    float lo = 0.0f, hi = best;
    /* slab ends ordered by the direction's sign; inv = +-inf for a zero
     * component makes each bound's term -inf / +inf inside / outside and NaN
     * on it, which the comparisons pass over (the containment test) */
    for (int a = 0; a < 3; a++) {
        float blo = orc_f16_to_f32(orc_f16_dir(nd->bmin[a], -1));
        float bhi = orc_f16_to_f32(orc_f16_dir(nd->bmax[a], +1));
        int neg = signbit(dd[a]) != 0;
        float t0 = ((neg ? bhi : blo) - oo[a]) * inv[a], t1 = ((neg ? blo : bhi) - oo[a]) * inv[a];
        lo = t0 > lo ? t0 : lo;
        hi = t1 < hi ? t1 : hi;
    }
    return !(lo * KD_EPS_LO > hi * KD_EPS_HI);
}

static hit_t isect_kd_ordered(qctx* q, orc_v3 o, orc_v3 d) {
    const orc_scene* s = q->s;
    hit_t h;
    memset(&h, 0, sizeof h);
    h.tri = -1; h.geom = -1;
    float best = q->best_init;
    uint32_t bprio = 0xFFFFFFFFu;
    ORC_DIAG_RAY_BEGIN(q);
    float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    float inv[3] = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    const orc_node* root = &s->nodes[0];
    float tmin = 0.0f, tmax = FLT_MAX;
    for (int a = 0; a < 3; a++) {
        if (dd[a] == 0.0f) {
            if (oo[a] < root->bmin[a] || oo[a] > root->bmax[a]) return h;
        } else {
            float t0 = (root->bmin[a] - oo[a]) * inv[a];
            float t1 = (root->bmax[a] - oo[a]) * inv[a];
            float lo = dd[a] < 0.0f ? t1 : t0;
            float hi = dd[a] < 0.0f ? t0 : t1;
            tmin = lo > tmin ? lo : tmin;
            tmax = hi < tmax ? hi : tmax;
        }
    }
    if (tmin > tmax * KD_EPS_HI) return h;
    uint32_t st_node[40];
    float st_lo[40], st_hi[40];
    int sp = 0;
    uint32_t node = 0;
    for (;;) {
        const orc_node* nd = &s->nodes[node];
        while (nd->axis) {
            q->c.inner_visits++;
            ORC_DIAG_INNER(q, node);
            int a = (int)nd->axis - 1;
            float sv = nd->split;
            float t = (sv - oo[a]) * inv[a];
            int below = (oo[a] < sv) || (oo[a] == sv && dd[a] <= 0.0f);
            uint32_t nearc = below ? nd->left : nd->right;
            uint32_t farc = below ? nd->right : nd->left;
            /* child-box cull (scenes the kernel serves from global memory) */
            int nhit = 1, fhit = 1;
            if (q->node_boxes) {
                nhit = box_hit(&s->nodes[nearc], oo, dd, inv, best);
                fhit = box_hit(&s->nodes[farc], oo, dd, inv, best);
            }
            if (dd[a] == 0.0f && oo[a] == sv) {
                if (fhit) { st_node[sp] = farc; st_lo[sp] = tmin; st_hi[sp] = tmax; sp++; }
                node = nearc;
            } else if (!(t > 0.0f) || t > tmax * KD_EPS_HI) {
                node = nearc;
            } else if (t * KD_EPS_HI < tmin) {
                node = farc;
            } else {
                if (fhit) { st_node[sp] = farc; st_lo[sp] = t > tmin ? t : tmin; st_hi[sp] = tmax; sp++; }
                node = nearc;
                tmax = t < tmax ? t : tmax;
            }
            if (!(node == nearc ? nhit : fhit)) {   /* chosen child missed: next interval */
                ORC_DIAG_POP(q);
                if (sp == 0) return h;
                sp--;
                node = st_node[sp]; tmin = st_lo[sp]; tmax = st_hi[sp];
                if (best <= tmin * KD_EPS_LO) return h;
            }
            if ((uint64_t)sp > q->c.stack_max) q->c.stack_max = (uint64_t)sp;
            nd = &s->nodes[node];
        }
        q->c.leaf_visits++;
        ORC_DIAG_LEAF(q, node);
        for (uint32_t i = 0; i < nd->tri_count; i++) {
            uint32_t k = s->leaf_ids[nd->tri_begin + i];
            q->c.leaf_refs++;
            q->c.tri_tests++;
            if (tri_test(q->kv[k], o, d, &best, &h, (int)k, s->tri_geom[s->kd_tris[k]], s->kd_prio[k], &bprio))
                ORC_DIAG_ACCEPT(q, node);
        }
        if (sp == 0) break;
        sp--;
        node = st_node[sp]; tmin = st_lo[sp]; tmax = st_hi[sp];
        if (best <= tmin * KD_EPS_LO) break;
    }
    return h;
}

static hit_t intersect(qctx* q, orc_v3 o, orc_v3 d) {
    q->c.rays++;
    if (q->traversal == 0) {
        hit_t h = isect_brute(q, o, d);
        if (h.tri >= 0) {
            /* brute force reports the CV index; convert to kd id for shading lookups */
            int lo = 0, hi = q->s->nkd - 1;
            while (lo < hi) { int mid = (lo + hi) / 2; if (q->s->kd_tris[mid] < h.tri) lo = mid + 1; else hi = mid; }
            h.tri = lo;
        }
        return h;
    }
    if (q->traversal == 1) return isect_kd_ref(q, o, d);
    return isect_kd_ordered(q, o, d);
}

void orc_intersect_batch(const orc_scene* s, int traversal, int64_t n,
                         const float* o, const float* d, int32_t* tri_out,
                         int32_t* geom_out, float* hit_out, orc_counters* c) {
    qctx q;
    memset(&q, 0, sizeof q);
    q.s = s;
    q.traversal = traversal;
    q.best_init = FLT_MAX;
    orc_v3(*kv)[3] = malloc(sizeof(orc_v3[3]) * (size_t)(s->nkd ? s->nkd : 1));
    for (int k = 0; k < s->nkd; k++)
        for (int j = 0; j < 3; j++) kv[k][j] = s->model.verts[s->model.tris[s->kd_tris[k]].v[j]];
    q.kv = (const orc_v3(*)[3])kv;
    for (int64_t i = 0; i < n; i++) {
        hit_t h = intersect(&q, v3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), v3(d[3 * i], d[3 * i + 1], d[3 * i + 2]));
        tri_out[i] = h.tri;
        geom_out[i] = h.geom;
        if (hit_out) {
            float* ho = hit_out + 6 * i;
            if (h.tri >= 0) { ho[0] = h.beta; ho[1] = h.gamma; ho[3] = h.hp.x; ho[4] = h.hp.y; ho[5] = h.hp.z; ho[2] = h.t; }
            else memset(ho, 0, 6 * sizeof(float));
        }
    }
    free(kv);
    if (c) *c = q.c;
}

/* Same, with the ordered walk's fp16 child-box cull selectable and the rays
 * split into contiguous ranges over `threads` pthreads (test infrastructure:
 * brute force over a 70k-triangle mesh takes ~1 ms per ray on one core). */
typedef struct {
    const orc_scene* s;
    const orc_v3 (*kv)[3];
    int traversal, node_boxes;
    int64_t b, e;
    const float *o, *d;
    int32_t *tri_out, *geom_out;
    float* hit_out;
    orc_counters c;
} ibjob;

static void* ib_worker(void* arg) {
    ibjob* j = (ibjob*)arg;
    qctx q;
    memset(&q, 0, sizeof q);
    q.s = j->s;
    q.kv = j->kv;
    q.traversal = j->traversal;
    q.node_boxes = j->node_boxes;
    q.best_init = FLT_MAX;
    for (int64_t i = j->b; i < j->e; i++) {
        hit_t h = intersect(&q, v3(j->o[3 * i], j->o[3 * i + 1], j->o[3 * i + 2]),
                            v3(j->d[3 * i], j->d[3 * i + 1], j->d[3 * i + 2]));
        j->tri_out[i] = h.tri;
        j->geom_out[i] = h.geom;
        if (j->hit_out) {
            float* ho = j->hit_out + 6 * i;
            if (h.tri >= 0) { ho[0] = h.beta; ho[1] = h.gamma; ho[3] = h.hp.x; ho[4] = h.hp.y; ho[5] = h.hp.z; ho[2] = h.t; }
            else memset(ho, 0, 6 * sizeof(float));
        }
    }
    j->c = q.c;
    return NULL;
}

void orc_intersect_batch_mt(const orc_scene* s, int traversal, int node_boxes, int threads, int64_t n,
                            const float* o, const float* d, int32_t* tri_out, int32_t* geom_out, float* hit_out,
                            orc_counters* c) {
    int nt = threads > 0 ? threads : 1;
    if (nt > 256) nt = 256;
    orc_v3(*kv)[3] = malloc(sizeof(orc_v3[3]) * (size_t)(s->nkd ? s->nkd : 1));
    for (int k = 0; k < s->nkd; k++)
        for (int j = 0; j < 3; j++) kv[k][j] = s->model.verts[s->model.tris[s->kd_tris[k]].v[j]];
    ibjob jobs[256];
    pthread_t th[256];
    for (int t = 0; t < nt; t++) {
        ibjob* j = &jobs[t];
        memset(j, 0, sizeof *j);
        j->s = s; j->kv = (const orc_v3(*)[3])kv; j->traversal = traversal; j->node_boxes = node_boxes;
        j->b = n * t / nt; j->e = n * (t + 1) / nt;
        j->o = o; j->d = d; j->tri_out = tri_out; j->geom_out = geom_out; j->hit_out = hit_out;
        pthread_create(&th[t], NULL, ib_worker, j);
    }
    orc_counters tot;
    memset(&tot, 0, sizeof tot);
    for (int t = 0; t < nt; t++) {
        pthread_join(th[t], NULL);
        const orc_counters* q = &jobs[t].c;
        tot.rays += q->rays; tot.paths += q->paths; tot.inner_visits += q->inner_visits;
        tot.leaf_visits += q->leaf_visits; tot.leaf_refs += q->leaf_refs; tot.tri_tests += q->tri_tests;
        tot.shades += q->shades;
        if (q->stack_max > tot.stack_max) tot.stack_max = q->stack_max;
    }
    free(kv);
    if (c) *c = tot;
}

/* =========================== path (CUTracer.cu:98-177) ==================== */
static orc_v3 sample_mc(qctx* q, usrc* u, orc_v3 pos, orc_v3 dir, int max_depth, float illum, int fresnel_kd) {
    const orc_scene* s = q->s;
    orc_v3 color = v3(1, 1, 1);
    int depth;
    q->c.paths++;
    for (depth = 0; depth < max_depth; depth++) {
        hit_t hit = intersect(q, pos, dir);
        ORC_DIAG_AFTER_ISECT(q, depth);
        if (hit.geom == -1) return v3(0, 0, 0);
        const orc_geom* g = &s->geoms[hit.geom];
        if (g->Ka.x > 0 || g->Ka.y > 0 || g->Ka.z > 0) {
            color.x *= g->Ka.x * illum;
            color.y *= g->Ka.y * illum;
            color.z *= g->Ka.z * illum;
            return color;
        }
        q->c.shades++;
        const orc_tri* t = &s->model.tris[s->kd_tris[hit.tri]];
        orc_v3 n1 = s->model.normals[t->n[0]];
        orc_v3 n2 = s->model.normals[t->n[1]];
        orc_v3 n3 = s->model.normals[t->n[2]];
        orc_v3 normal = vadd(vadd(vscale(n1, 1.0f - hit.beta - hit.gamma), vscale(n2, hit.beta)), vscale(n3, hit.gamma));
        normalize_cu(&normal);
        if (g->Tr > 0) {
            dir = sample_fresnel(u, normal, dir, g->Tr, g->Ni, 0);
            if (fresnel_kd) { color.x *= g->Kd.x; color.y *= g->Kd.y; color.z *= g->Kd.z; }
            pos = vadd(hit.hp, vscale(dir, 0.01f));
        } else if (g->Ns > 1) {
            dir = sample_phong(u, normal, dir, (float)((uint32_t)g->Ns + 1u));
            color.x *= g->Ks.x; color.y *= g->Ks.y; color.z *= g->Ks.z;
            pos = vadd(hit.hp, vscale(dir, 0.01f));
        } else {
            color.x *= g->Kd.x; color.y *= g->Kd.y; color.z *= g->Kd.z;
            if (dot3(dir, normal) > 0) {
                orc_v3 h = sample_hemi(u, normal);
                dir = v3(-h.x, -h.y, -h.z);
            } else {
                dir = sample_hemi(u, normal);
            }
            pos = vadd(hit.hp, vscale(dir, 0.01f));
        }
    }
    {
        hit_t hit = intersect(q, pos, dir);
        ORC_DIAG_AFTER_ISECT(q, max_depth);
        if (hit.geom != -1) {
            const orc_geom* g = &s->geoms[hit.geom];
            color.x *= g->Ka.x * illum;
            color.y *= g->Ka.y * illum;
            color.z *= g->Ka.z * illum;
        } else {
            color = v3(0, 0, 0);
        }
    }
    return color;
}


/* ===================== QuinEngine path (rtx.hlsl:304-371) ================= */
#define QE_T_BEST 10000.0f
static orc_v3 sample_mc_qe(qctx* q, usrc* u, orc_v3 pos, orc_v3 dir, int depth_lim) {
    const orc_scene* s = q->s;
    orc_v3 color = v3(1, 1, 1);
    uint32_t bounce = 0;
    q->c.paths++;
    hit_t hit = intersect(q, pos, dir);
    while (hit.geom != -1) {
        if (bounce >= (uint32_t)depth_lim * 3u) return v3(0, 0, 0);
        if (bounce >= (uint32_t)depth_lim) {                  /* Russian roulette, :314-325 */
            float illum = fmaxf(fmaxf(color.x, color.y), color.z);
            if (illum > next_u(u)) color = vdiv(color, illum);
            else return v3(0, 0, 0);
        }
        const orc_geom* g = &s->geoms[hit.geom];
        if (g->Ka.x > 0 || g->Ka.y > 0 || g->Ka.z > 0) {     /* :327-331, no ILLUM */
            color.x *= g->Ka.x * 1.0f; color.y *= g->Ka.y * 1.0f; color.z *= g->Ka.z * 1.0f;
            return color;
        }
        q->c.shades++;
        const orc_tri* t = &s->model.tris[s->kd_tris[hit.tri]];
        orc_v3 n1 = s->model.normals[t->n[0]];
        orc_v3 n2 = s->model.normals[t->n[1]];
        orc_v3 n3 = s->model.normals[t->n[2]];
        orc_v3 normal = vadd(vadd(vscale(n1, 1.0f - hit.beta - hit.gamma), vscale(n2, hit.beta)), vscale(n3, hit.gamma));
        normalize_hlsl(&normal);                              /* :340 */
        if (g->Tr > 0) {                                      /* :341-345, no Kd tint */
            dir = sample_fresnel(u, normal, dir, g->Tr, g->Ni, 1);
        } else if (g->Ns > 1) {
            dir = sample_phong(u, normal, dir, g->Ns + 1.0f);
            color.x *= g->Ks.x; color.y *= g->Ks.y; color.z *= g->Ks.z;
        } else {
            color.x *= g->Kd.x; color.y *= g->Kd.y; color.z *= g->Kd.z;
            if (dot3(dir, normal) > 0) {
                orc_v3 h = sample_hemi(u, normal);
                dir = v3(-h.x, -h.y, -h.z);
            } else {
                dir = sample_hemi(u, normal);
            }
        }
        pos = vadd(hit.hp, vscale(dir, 0.01f));
        hit = intersect(q, pos, dir);
        ++bounce;
    }
    return v3(0, 0, 0);
}

/* QE primary ray (rtx.hlsl:380-397): TEA-16(pixel, frame seed), two warm-up
 * draws, +-0.5 px jitter, near-plane origin, view->world by the camera basis */
static void qe_primary(const orc_params* p, uint32_t pix, int x, int y, uint32_t sample, usrc* u,
                       orc_v3* o, orc_v3* d) {
    u->sd = orc_tea16(pix, (uint32_t)p->seed + p->spp_offset + sample);
    u->inj = NULL; u->k = 0;
    next_u(u);
    next_u(u);
    float bx = (float)(uint32_t)x + (next_u(u) - 0.5f);
    float by = (float)(uint32_t)y + (next_u(u) - 0.5f);
    float vx = (2.0f * bx / (float)(uint32_t)p->width - 1.0f) / p->proj11;
    float vy = (1.0f - 2.0f * by / (float)(uint32_t)p->height) / p->proj22;
    float vz = -1.0f;
    orc_v3 w;
    w.x = p->right[0] * vx + p->up[0] * vy - p->fwd[0] * vz;
    w.y = p->right[1] * vx + p->up[1] * vy - p->fwd[1] * vz;
    w.z = p->right[2] * vx + p->up[2] * vy - p->fwd[2] * vz;
    *o = v3(w.x + p->eye[0], w.y + p->eye[1], w.z + p->eye[2]);
    normalize_hlsl(&w);                                       /* :395 */
    *d = w;
}

/* gamma-space running mean (rtx.hlsl:401-402) with the deterministic pow */
#define QE_GAMMA 2.2f
#define QE_INV_GAMMA 0.454545454545f
static float qe_blend(float old, float c, uint32_t prev) {
    if (prev == 0) return orc_powf(c, QE_INV_GAMMA);
    float pc = (float)prev, pc1 = (float)(prev + 1u);
    return orc_powf((orc_powf(old, QE_GAMMA) * pc + c) / pc1, QE_INV_GAMMA);
}

/* ========================= render (CUTracer.cu:179-218) =================== */
typedef struct {
    const orc_scene* s;
    const orc_params* p;
    float* out;
    const orc_v3 (*kv)[3];
    int next_row;
    pthread_mutex_t mu;
    orc_counters total;
} rjob;

static void render_pixel(qctx* q, const orc_params* p, uint32_t key, int x, int y, float* px) {
    uint32_t W = (uint32_t)p->width, H = (uint32_t)p->height;
    uint32_t pix = (uint32_t)y * W + (uint32_t)x;
    uint32_t chunk = p->spp_chunk ? p->spp_chunk : p->spp;
    if (chunk == 0) chunk = 1;
    orc_v3 sum = v3(0, 0, 0);
    orc_v3 right = v3(p->right[0], p->right[1], p->right[2]);
    orc_v3 up = v3(p->up[0], p->up[1], p->up[2]);
    orc_v3 fwd = v3(p->fwd[0], p->fwd[1], p->fwd[2]);
    orc_v3 eye = v3(p->eye[0], p->eye[1], p->eye[2]);
    for (uint32_t c0 = 0; c0 < p->spp; c0 += chunk) {
        orc_v3 part = v3(0, 0, 0);
        uint32_t c1 = c0 + chunk < p->spp ? c0 + chunk : p->spp;
        for (uint32_t i = c0; i < c1; i++) {
            if (p->mode == 1) {
                usrc u;
                orc_v3 o, d;
                qe_primary(p, pix, x, y, i, &u, &o, &d);
                part = vadd(part, sample_mc_qe(q, &u, o, d, p->max_depth));
                continue;
            }
            usrc u = {orc_rng_init(pix, key, p->spp_offset + i), NULL, 0};
            float biasx = (float)(uint32_t)x + (next_u(&u) * 2.0f - 1.0f);
            float biasy = (float)(uint32_t)y + (next_u(&u) * 2.0f - 1.0f);
            double th = (double)p->tan_half_fov;
            orc_v3 idir = v3((float)((2.0 * (double)biasx / (double)W - 1) * th),
                             (float)((1.0 * (double)H / (double)W - 2.0 * (double)biasy / (double)W) * th),
                             -1.0f);
            orc_v3 wr;
            wr.x = right.x * idir.x + up.x * idir.y - fwd.x * idir.z;
            wr.y = right.y * idir.x + up.y * idir.y - fwd.y * idir.z;
            wr.z = right.z * idir.x + up.z * idir.y - fwd.z * idir.z;
            normalize_cu(&wr);
            orc_v3 L = sample_mc(q, &u, eye, wr, p->max_depth, p->illum, p->fresnel_kd);
            part = vadd(part, L);
        }
        sum = vadd(sum, part);
    }
    orc_v3 mean = vdiv(sum, (float)p->spp);
    if (p->mode == 1) {
        px[0] = qe_blend(px[0], mean.x, p->prev_count);
        px[1] = qe_blend(px[1], mean.y, p->prev_count);
        px[2] = qe_blend(px[2], mean.z, p->prev_count);
    } else if (p->prev_count == 0) {
        px[0] = mean.x; px[1] = mean.y; px[2] = mean.z;
    } else {
        float pc = (float)p->prev_count, pc1 = (float)(p->prev_count + 1);
        px[0] = (px[0] * pc + mean.x) / pc1;
        px[1] = (px[1] * pc + mean.y) / pc1;
        px[2] = (px[2] * pc + mean.z) / pc1;
    }
}

static void* render_worker(void* arg) {
    rjob* j = (rjob*)arg;
    const orc_params* p = j->p;
    qctx q;
    memset(&q, 0, sizeof q);
    q.s = j->s;
    q.kv = j->kv;
    q.traversal = p->traversal;
    q.node_boxes = p->node_boxes;
    q.best_init = p->mode == 1 ? QE_T_BEST : FLT_MAX;
    uint32_t key = orc_seed_key(p->seed);
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int y = j->next_row++;
        pthread_mutex_unlock(&j->mu);
        if (y >= p->y1) break;
        for (int x = p->x0; x < p->x1; x++)
            render_pixel(&q, p, key, x, y, j->out + 3 * ((size_t)y * (size_t)p->width + (size_t)x));
    }
    pthread_mutex_lock(&j->mu);
    j->total.rays += q.c.rays; j->total.paths += q.c.paths;
    j->total.inner_visits += q.c.inner_visits; j->total.leaf_visits += q.c.leaf_visits;
    j->total.leaf_refs += q.c.leaf_refs; j->total.tri_tests += q.c.tri_tests;
    j->total.shades += q.c.shades;
    if (q.c.stack_max > j->total.stack_max) j->total.stack_max = q.c.stack_max;
    pthread_mutex_unlock(&j->mu);
    return NULL;
}

int orc_render(const orc_scene* s, const orc_params* p, float* out, orc_counters* c) {
    if (!s || !p || !out || p->width <= 0 || p->height <= 0 || p->spp == 0) return -1;
    if (p->x0 < 0 || p->y0 < 0 || p->x1 > p->width || p->y1 > p->height) return -1;
    rjob j;
    memset(&j, 0, sizeof j);
    j.s = s; j.p = p; j.out = out; j.next_row = p->y0;
    pthread_mutex_init(&j.mu, NULL);
    orc_v3(*kv)[3] = malloc(sizeof(orc_v3[3]) * (size_t)(s->nkd ? s->nkd : 1));
    for (int k = 0; k < s->nkd; k++)
        for (int i = 0; i < 3; i++) kv[k][i] = s->model.verts[s->model.tris[s->kd_tris[k]].v[i]];
    j.kv = (const orc_v3(*)[3])kv;
    int nt = p->threads > 0 ? p->threads : 1;
    if (nt == 1) {
        render_worker(&j);
    } else {
        pthread_t* th = malloc(sizeof(pthread_t) * (size_t)nt);
        for (int i = 0; i < nt; i++) pthread_create(&th[i], NULL, render_worker, &j);
        for (int i = 0; i < nt; i++) pthread_join(th[i], NULL);
        free(th);
    }
    free(kv);
    pthread_mutex_destroy(&j.mu);
    if (c) *c = j.total;
    return 0;
}

/* ============================ scene assembly ============================== */
orc_scene* orc_scene_load(const char* path, char* err, int errlen) { return orc_scene_load_ex(path, 0, err, errlen); }

orc_scene* orc_scene_load_ex(const char* path, int flavor, char* err, int errlen) {
    return orc_scene_load_kd(path, flavor, 0, err, errlen);
}

orc_scene* orc_scene_load_kd(const char* path, int flavor, int kd_build, char* err, int errlen) {
    char dummy[256];
    if (!err) { err = dummy; errlen = sizeof dummy; }
    err[0] = 0;
    orc_scene* s = calloc(1, sizeof(orc_scene));
    if (!(flavor == 1 ? orc_model_read_tinyobj : orc_model_read)(&s->model, path, err, errlen)) {
        orc_scene_free(s);
        return NULL;
    }
    orc_model* m = &s->model;
    /* CreateGeometry (CUTracer.cu:277-311): non-empty groups in map order */
    s->geoms = calloc((size_t)(m->ngroups ? m->ngroups : 1), sizeof(orc_geom));
    for (int g = 0; g < m->ngroups; g++) {
        const orc_group* gr = &m->groups[g];
        if (gr->ntris == 0) continue;
        orc_geom* ge = &s->geoms[s->ngeoms++];
        ge->start = (uint32_t)gr->tris[0];
        ge->count = (uint32_t)gr->ntris;
        const orc_mat* mt = &m->mats[m->tris[gr->tris[0]].mat];
        ge->Ka = mt->Ka; ge->Kd = mt->Kd; ge->Ks = mt->Ks;
        ge->Ns = (float)mt->Ns; ge->Tr = (float)mt->Tr; ge->Ni = (float)mt->Ni;
    }
    s->tri_geom = malloc(sizeof(int) * (size_t)m->ntris);
    for (int i = 0; i < m->ntris; i++) s->tri_geom[i] = -1;
    for (int g = 0; g < s->ngeoms; g++) {
        for (uint32_t i = 0; i < s->geoms[g].count; i++) {
            uint32_t cv = s->geoms[g].start + i;
            if (cv >= (uint32_t)m->ntris) {
                snprintf(err, errlen, "geometry %d range exceeds triangle count", g);
                orc_scene_free(s);
                return NULL;
            }
            if (s->tri_geom[cv] < 0) s->tri_geom[cv] = g;
        }
    }
    s->kd_tris = malloc(sizeof(int) * (size_t)m->ntris);
    for (int i = 0; i < m->ntris; i++) {
        if (s->tri_geom[i] < 0) continue;
        const orc_tri* t = &m->tris[i];
        for (int j = 0; j < 3; j++) {
            if (t->v[j] < 0 || t->v[j] >= m->nverts || t->n[j] < 0 || t->n[j] >= m->nnormals) {
                snprintf(err, errlen, "triangle %d has an out-of-range index", i);
                orc_scene_free(s);
                return NULL;
            }
        }
        s->kd_tris[s->nkd++] = i;
    }
    /* brute-force iteration rank of each kd triangle (CUTracer.cu:49-54) */
    s->kd_prio = malloc(sizeof(uint32_t) * (size_t)(s->nkd ? s->nkd : 1));
    {
        int* cv2kd = malloc(sizeof(int) * (size_t)m->ntris);
        for (int i = 0; i < m->ntris; i++) cv2kd[i] = -1;
        for (int k = 0; k < s->nkd; k++) cv2kd[s->kd_tris[k]] = k;
        uint32_t rank = 0;
        for (int g = 0; g < s->ngeoms; g++)
            for (uint32_t i = 0; i < s->geoms[g].count; i++) {
                uint32_t cv = s->geoms[g].start + i;
                if (s->tri_geom[cv] == g) s->kd_prio[cv2kd[cv]] = rank;
                rank++;
            }
        free(cv2kd);
    }
    orc_kd_build(s, kd_build);
    return s;
}

void orc_scene_free(orc_scene* s) {
    if (!s) return;
    orc_model_free(&s->model);
    free(s->geoms); free(s->tri_geom); free(s->kd_tris); free(s->kd_prio); free(s->nodes); free(s->leaf_ids);
    free(s);
}

void orc_scene_info(const orc_scene* s, int64_t* info) {
    info[0] = s->model.nverts; info[1] = s->model.nnormals; info[2] = s->model.ntris;
    info[3] = s->model.nmats; info[4] = s->model.ngroups; info[5] = s->ngeoms;
    info[6] = s->nkd; info[7] = s->nnodes; info[8] = s->nleaf_ids; info[9] = s->kd_depth;
}
void orc_copy_vertices(const orc_scene* s, float* out) {
    for (int i = 0; i < s->model.nverts; i++) { out[3 * i] = s->model.verts[i].x; out[3 * i + 1] = s->model.verts[i].y; out[3 * i + 2] = s->model.verts[i].z; }
}
void orc_copy_normals(const orc_scene* s, float* out) {
    for (int i = 0; i < s->model.nnormals; i++) { out[3 * i] = s->model.normals[i].x; out[3 * i + 1] = s->model.normals[i].y; out[3 * i + 2] = s->model.normals[i].z; }
}
void orc_copy_triangles(const orc_scene* s, int32_t* out) {
    for (int i = 0; i < s->model.ntris; i++) {
        const orc_tri* t = &s->model.tris[i];
        for (int j = 0; j < 3; j++) { out[10 * i + j] = t->v[j]; out[10 * i + 3 + j] = t->t[j]; out[10 * i + 6 + j] = t->n[j]; }
        out[10 * i + 9] = t->mat;
    }
}
void orc_copy_materials(const orc_scene* s, double* out) {
    for (int i = 0; i < s->model.nmats; i++) {
        const orc_mat* m = &s->model.mats[i];
        double* o = out + 12 * i;
        o[0] = m->Ka.x; o[1] = m->Ka.y; o[2] = m->Ka.z; o[3] = m->Kd.x; o[4] = m->Kd.y; o[5] = m->Kd.z;
        o[6] = m->Ks.x; o[7] = m->Ks.y; o[8] = m->Ks.z; o[9] = m->Ns; o[10] = m->Tr; o[11] = m->Ni;
    }
}
const char* orc_group_name(const orc_scene* s, int g) { return s->model.groups[g].name; }
int orc_group_ntris(const orc_scene* s, int g) { return s->model.groups[g].ntris; }
void orc_group_tris(const orc_scene* s, int g, int32_t* out) {
    for (int i = 0; i < s->model.groups[g].ntris; i++) out[i] = s->model.groups[g].tris[i];
}
void orc_copy_geoms(const orc_scene* s, float* out) {
    for (int g = 0; g < s->ngeoms; g++) {
        const orc_geom* e = &s->geoms[g];
        float* o = out + 14 * g;
        o[0] = e->Ka.x; o[1] = e->Ka.y; o[2] = e->Ka.z; o[3] = e->Kd.x; o[4] = e->Kd.y; o[5] = e->Kd.z;
        o[6] = e->Ks.x; o[7] = e->Ks.y; o[8] = e->Ks.z; o[9] = e->Ns; o[10] = e->Tr; o[11] = e->Ni;
        o[12] = (float)e->start; o[13] = (float)e->count;
    }
}
void orc_copy_kd_tris(const orc_scene* s, int32_t* out) { memcpy(out, s->kd_tris, sizeof(int) * (size_t)s->nkd); }
void orc_copy_kd_nodes(const orc_scene* s, uint32_t* out) {
    for (int i = 0; i < s->nnodes; i++) {
        const orc_node* n = &s->nodes[i];
        uint32_t* o = out + 12 * i;
        o[0] = n->left; o[1] = n->right; o[2] = n->axis;
        memcpy(&o[3], &n->split, 4);
        memcpy(&o[4], n->bmin, 12);
        memcpy(&o[7], n->bmax, 12);
        o[10] = n->tri_begin; o[11] = n->tri_count;
    }
}
void orc_copy_kd_leaf_ids(const orc_scene* s, uint32_t* out) {
    memcpy(out, s->leaf_ids, sizeof(uint32_t) * (size_t)s->nleaf_ids);
}
