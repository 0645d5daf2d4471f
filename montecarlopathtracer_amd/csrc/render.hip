// render.hip -- MI355X (gfx950) path-tracing megakernel and its host launcher.
//
// Replaces rayTraceKernel (CVMCTracer/CUDA/CUTracer.cu:179-218, one thread per
// pixel, brute-force intersect :44-96) with:
//   * persistent workgroups (one 1024-thread workgroup per CU when the scene
//     image fits in LDS) that pull work units (pixel, sample-chunk) from a
//     device counter, one atomic per wave per refill (__ballot / popcount);
//   * path regeneration: a lane whose path ends immediately starts the next
//     sample of its unit, so every lane traces one ray per loop iteration;
//   * the scene image (triangles, KD nodes, leaf ids, materials) copied into
//     LDS once per workgroup; the KD traversal stack keeps its top S entries in
//     LDS (lane-strided, conflict-free) and spills deeper ones to global memory;
//   * ordered front-to-back KD traversal (split-plane intervals, conservative
//     2^-12 margins) returning the brute-force closest hit (ties broken in the
//     brute-force loop order), see DESIGN.md;
//   * per-unit partial sums in HBM reduced in chunk order by a second kernel:
//     results are deterministic and independent of scheduling.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>

#include "mcpt_device.hpp"
#include "render_launch.hpp"

namespace mcpt {

using namespace dev;

namespace {

struct Counters {
    uint32_t rays, paths, inner, leaf, refs, tests, shades, spills;
};

__device__ __forceinline__ float sel3(int a, float x, float y, float z) {
    return a == 0 ? x : (a == 1 ? y : z);
}

// lane modes of the persistent loop
constexpr int kDead = 0;    // no more work
constexpr int kTrav = 1;    // traversing its current ray
constexpr int kReady = 2;   // closest hit known, waiting for a shading round
constexpr int kNeed = 3;    // needs a work unit

// Per-lane ray + traversal state.  The traversal is the ordered front-to-back
// KD walk of oracle/render_ref.c isect_kd_ordered(), split into resumable
// iterations (descend to a leaf, test its triangles, pop).
struct RayState {
    V3 o, d;
    float ix, iy, iz;
    float tmin, tmax, best;
    uint32_t nw0, nw1, bprio;            // current node record
    int32_t sp, htri;
    float hbeta, hgamma;
};

// root interval (oracle: isect_kd_ordered prologue); returns false on a miss
__device__ __forceinline__ bool begin_ray(RayState& r, const GpuScene& sc) {
    r.ix = 1.0f / r.d.x;
    r.iy = 1.0f / r.d.y;
    r.iz = 1.0f / r.d.z;
    r.htri = -1;
    r.hbeta = r.hgamma = 0.0f;
    r.best = kFltMax;
    r.bprio = 0xFFFFFFFFu;
    r.nw0 = sc.root_w[0];
    r.nw1 = sc.root_w[1];
    r.sp = 0;
    float tmin = 0.0f, tmax = kFltMax;
    const float oo[3] = {r.o.x, r.o.y, r.o.z}, dd[3] = {r.d.x, r.d.y, r.d.z}, inv[3] = {r.ix, r.iy, r.iz};
    bool miss = false;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        if (dd[a] == 0.0f) {
            miss = miss || (oo[a] < sc.root_min[a] || oo[a] > sc.root_max[a]);
        } else {
            const float t0 = (sc.root_min[a] - oo[a]) * inv[a];
            const float t1 = (sc.root_max[a] - oo[a]) * inv[a];
            const float lo = dd[a] < 0.0f ? t1 : t0;
            const float hi = dd[a] < 0.0f ? t0 : t1;
            tmin = lo > tmin ? lo : tmin;
            tmax = hi < tmax ? hi : tmax;
        }
    }
    r.tmin = tmin;
    r.tmax = tmax;
    return !miss && !(tmin > tmax * kEpsHi);
}

// Cramer test (CUTracer.cu:54-92) with an exact-result-preserving prefilter:
// the three IEEE divisions run only when the signs of the determinants allow
// beta, gamma, t > 0 and the magnitudes do not already rule out beta+gamma < 1
// or t < best (2^-20 margins cover every rounding of the exact path).
__device__ __forceinline__ void test_tri(RayState& r, const float4* __restrict__ tris, uint32_t k) {
    const float4 A0 = tris[3 * k], A1 = tris[3 * k + 1], A2 = tris[3 * k + 2];
    const float aox = A0.x - r.o.x, aoy = A0.y - r.o.y, aoz = A0.z - r.o.z;
    const float detA = det3(A1.x, A2.x, r.d.x, A1.y, A2.y, r.d.y, A1.z, A2.z, r.d.z);
    const float qb = det3(aox, A2.x, r.d.x, aoy, A2.y, r.d.y, aoz, A2.z, r.d.z);
    const float qg = det3(A1.x, aox, r.d.x, A1.y, aoy, r.d.y, A1.z, aoz, r.d.z);
    const float qt = det3(A1.x, A2.x, aox, A1.y, A2.y, aoy, A1.z, A2.z, aoz);
    // sign-normalised numerators: beta, gamma, t > 0 needs all three > 0 (a NaN
    // anywhere means no hit, so min3 may drop it); detA == 0 fails the magnitude test
    const uint32_t sA = __float_as_uint(detA) & 0x80000000u;
    const float xb = __uint_as_float(__float_as_uint(qb) ^ sA);
    const float xg = __uint_as_float(__float_as_uint(qg) ^ sA);
    const float xt = __uint_as_float(__float_as_uint(qt) ^ sA);
    const bool signs_ok = __builtin_fminf(__builtin_fminf(xb, xg), xt) > 0.0f;
    const float adet = fabsf(detA) * 1.00000095367431640625f;   // 1 + 2^-20
    const bool mags_ok = !(xb + xg > adet) & !(xt > r.best * adet);
    if (signs_ok & mags_ok) {
        const float beta = qb / detA;
        const float gamma = qg / detA;
        const float t = qt / detA;
        const uint32_t prio = __float_as_uint(A0.w);
        if (beta + gamma < 1.0f && beta > 0.0f && gamma > 0.0f && t > 0.0f &&
            (t < r.best || (t == r.best && prio < r.bprio))) {
            r.best = t;
            r.bprio = prio;
            r.htri = (int32_t)k;
            r.hbeta = beta;
            r.hgamma = gamma;
        }
    }
}

// One resumable traversal iteration: descend to a leaf, test it, pop.
// Returns true when the ray's closest hit is final.  The children of the
// current node are read as one 16-B sibling-pair record whose address is known
// before the split-plane decision, so the LDS latency overlaps the decision;
// stack entries carry the far child's record (16 B: w0, w1, lo, hi), so a pop
// needs no node re-read.
template <int S>
__device__ __forceinline__ bool trav_iter(RayState& r, const float4* __restrict__ tris,
                                          const uint2* __restrict__ nodes1, const uint32_t* __restrict__ leafs,
                                          uint4* st, int stride, uint4* __restrict__ spill, uint32_t spill_stride,
                                          Counters& c) {
    uint32_t w0 = r.nw0, w1 = r.nw1;
    while ((w0 >> 30) != 3u) {
        c.inner++;
        const uint32_t left = w0 & 0x3FFFFFFFu;
        const uint4 pr = *reinterpret_cast<const uint4*>(nodes1 + left);   // children left, left+1
        const int a = (int)(w0 >> 30);
        const float sv = __uint_as_float(w1);
        const float oa = sel3(a, r.o.x, r.o.y, r.o.z);
        const float da = sel3(a, r.d.x, r.d.y, r.d.z);
        const float ia = sel3(a, r.ix, r.iy, r.iz);
        const float t = (sv - oa) * ia;
        const bool below = (oa < sv) || (oa == sv && da <= 0.0f);
        // if/else chain of the oracle, evaluated branch-free
        const bool pp = (da == 0.0f) & (oa == sv);                  // ray inside the plane: both
        const bool no = !(t > 0.0f) | (t > r.tmax * kEpsHi);        // near child only
        const bool fo = t * kEpsHi < r.tmin;                        // far child only
        const bool go_far = !pp & !no & fo;
        const bool push_it = pp | (!no & !fo);
        const uint32_t n0 = below ? pr.x : pr.z, n1 = below ? pr.y : pr.w;     // near child record
        const uint32_t f0 = below ? pr.z : pr.x, f1 = below ? pr.w : pr.y;     // far child record
        if (push_it) {
            const float plo = pp ? r.tmin : (t > r.tmin ? t : r.tmin);
            uint4* slot = st + (r.sp & (S - 1)) * stride;
            if (r.sp >= S) {
                spill[(uint32_t)(r.sp - S) * spill_stride] = *slot;
                c.spills++;
            }
            *slot = make_uint4(f0, f1, __float_as_uint(plo), __float_as_uint(r.tmax));
            r.sp++;
            if (!pp) r.tmax = t < r.tmax ? t : r.tmax;
        }
        w0 = go_far ? f0 : n0;
        w1 = go_far ? f1 : n1;
    }
    c.leaf++;
    const uint32_t begin = w0 & 0x3FFFFFFFu;
    const uint32_t cnt = w1;
    for (uint32_t i = 0; i < cnt; i++) {
        c.refs++;
        c.tests++;
        test_tri(r, tris, leafs[begin + i]);
    }
    if (r.sp == 0) return true;
    r.sp--;
    uint4* slot = st + (r.sp & (S - 1)) * stride;
    const uint4 e = *slot;
    r.nw0 = e.x;
    r.nw1 = e.y;
    r.tmin = __uint_as_float(e.z);
    r.tmax = __uint_as_float(e.w);
    if (r.sp >= S) *slot = spill[(uint32_t)(r.sp - S) * spill_stride];
    return r.best <= r.tmin * kEpsLo;
}

// work unit v (packed owned-pixel index) -> image pixel; false outside the image
__device__ __forceinline__ bool unit_pixel(const KernelParams& kp, uint32_t v, int& x, int& y) {
    const uint32_t tt = (uint32_t)(kp.tile * kp.tile);
    const uint32_t k = v / tt, w = v - k * tt;
    const uint32_t t = (uint32_t)kp.shard_index + k * (uint32_t)kp.shard_count;
    const uint32_t ty = t / (uint32_t)kp.tiles_x, tx = t - ty * (uint32_t)kp.tiles_x;
    const uint32_t wy = w / (uint32_t)kp.tile, wx = w - wy * (uint32_t)kp.tile;
    x = (int)(tx * (uint32_t)kp.tile + wx);
    y = (int)(ty * (uint32_t)kp.tile + wy);
    return x < kp.width && y < kp.height;
}

// primary ray of sample s of pixel (px, py) (CUTracer.cu:186-211)
__device__ __forceinline__ void primary_ray(const KernelParams& kp, uint32_t pix, int px, int py, uint32_t s,
                                            uint32_t& sd, V3& dir) {
    sd = rng_init(pix, kp.key, kp.spp_offset + s);
    const float biasx = (float)(uint32_t)px + (rng_next(sd) * 2.0f - 1.0f);
    const float biasy = (float)(uint32_t)py + (rng_next(sd) * 2.0f - 1.0f);
    const double th = (double)kp.tan_half_fov;
    const double W = (double)(uint32_t)kp.width, H = (double)(uint32_t)kp.height;
    const float idx = (float)((2.0 * (double)biasx / W - 1) * th);
    const float idy = (float)((1.0 * H / W - 2.0 * (double)biasy / W) * th);
    const float idz = -1.0f;
    V3 wr;
    wr.x = kp.right[0] * idx + kp.up[0] * idy - kp.fwd[0] * idz;
    wr.y = kp.right[1] * idx + kp.up[1] * idy - kp.fwd[1] * idz;
    wr.z = kp.right[2] * idx + kp.up[2] * idy - kp.fwd[2] * idz;
    normalize_cu(wr);
    dir = wr;
}

template <bool IN_LDS, int S, int BLOCK, bool DBG>
__global__ void __launch_bounds__(BLOCK) path_kernel(const KernelParams kp) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = (int)threadIdx.x;
    const int lane = tid & 63;
    const GpuScene& sc = kp.scene;

    const float4* tris;
    const uint2* nodes;
    const uint32_t* leafs;
    const GpuGeom* geoms;
    if constexpr (IN_LDS) {
        const uint4* src = reinterpret_cast<const uint4*>(sc.image);
        uint4* dst = reinterpret_cast<uint4*>(smem);
        const uint32_t n16 = sc.image_bytes / 16u;
        for (uint32_t i = (uint32_t)tid; i < n16; i += BLOCK) dst[i] = src[i];
        __syncthreads();
        tris = reinterpret_cast<const float4*>(smem + sc.off_tris);
        nodes = reinterpret_cast<const uint2*>(smem + sc.off_nodes) + 1;   // node i at slot i+1
        leafs = reinterpret_cast<const uint32_t*>(smem + sc.off_leafs);
        geoms = reinterpret_cast<const GpuGeom*>(smem + sc.off_geoms);
    } else {
        tris = reinterpret_cast<const float4*>(sc.image + sc.off_tris);
        nodes = reinterpret_cast<const uint2*>(sc.image + sc.off_nodes) + 1;
        leafs = reinterpret_cast<const uint32_t*>(sc.image + sc.off_leafs);
        geoms = reinterpret_cast<const GpuGeom*>(sc.image + sc.off_geoms);
    }
    uint4* st = reinterpret_cast<uint4*>(smem + kp.lds_stack_off) + tid;   // [S][BLOCK] x 16 B
    const uint32_t gl = blockIdx.x * BLOCK + (uint32_t)tid;
    uint4* spill = kp.spill + gl;
    const uint32_t spill_stride = kp.total_lanes;
    const V3 eye = v3(kp.eye[0], kp.eye[1], kp.eye[2]);

    Counters c = {0, 0, 0, 0, 0, 0, 0, 0};
    Counters c0 = c;   // DBG builds only
    int mode = kNeed;
    uint32_t s = 0, s_end = 0, unit_id = 0;
    int px = 0, py = 0, depth = 0;
    uint32_t sd = 1;
    V3 part = v3(0, 0, 0), color = v3(1, 1, 1);
    RayState r;
    r.o = eye;
    r.d = v3(0, 0, -1);
    r.htri = -1;

    // start sample s of the current unit: primary ray, then its root interval
    auto start_path = [&]() {
        const uint32_t pix = (uint32_t)py * (uint32_t)kp.width + (uint32_t)px;
        primary_ray(kp, pix, px, py, s, sd, r.d);
        r.o = eye;
        color = v3(1, 1, 1);
        depth = 0;
        c.paths++;
        c.rays++;
        mode = begin_ray(r, sc) ? kTrav : kReady;
    };

#ifdef MCPT_PHASE_TIMING
    unsigned long long tm_units = 0, tm_trav = 0, tm_shade = 0, tm_iters = 0, tm_t0;
#define MCPT_STAMP(acc) do { unsigned long long t1_ = __builtin_amdgcn_s_memtime(); acc += t1_ - tm_t0; tm_t0 = t1_; } while (0)
    tm_t0 = __builtin_amdgcn_s_memtime();
#else
#define MCPT_STAMP(acc) do {} while (0)
#endif
    for (;;) {
        // ---- work units: one atomic per wave for every lane that needs one ----
        for (;;) {
            const uint64_t m = __ballot(mode == kNeed);
            if (!m) break;
            const int leader = __ffsll((unsigned long long)m) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(kp.counter, (uint32_t)__popcll(m));
            base = __shfl(base, leader);
            if (mode == kNeed) {
                const uint32_t unit = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                if (unit >= kp.total_units) {
                    mode = kDead;
                } else {
                    unit_id = unit;
                    if constexpr (DBG) c0 = c;
                    const uint32_t chunk = unit / kp.npix_local;
                    const uint32_t v = unit - chunk * kp.npix_local;
                    s = chunk * kp.chunk;
                    s_end = min(s + kp.chunk, kp.spp);
                    part = v3(0, 0, 0);
                    if (unit_pixel(kp, v, px, py)) {
                        start_path();
                    } else {
                        kp.partial[unit] = make_float4(0, 0, 0, 0);
                    }
                }
            }
        }
        if (!__ballot(mode != kDead)) break;
        MCPT_STAMP(tm_units);

        // ---- traversal burst: until half the wave is ready to shade --------
        for (;;) {
#ifdef MCPT_PHASE_TIMING
            tm_iters++;
#endif
            if (mode == kTrav) {
                if (trav_iter<S>(r, tris, nodes, leafs, st, BLOCK, spill, spill_stride, c))
                    mode = kReady;
            }
            const uint64_t trv = __ballot(mode == kTrav);
            const uint64_t rdy = __ballot(mode == kReady);
            if (!trv || __popcll(rdy) >= kp.ready_thresh) break;
        }
        MCPT_STAMP(tm_trav);

        // ---- shading round for every ready lane (CUTracer.cu:105-175) -------
        if (mode == kReady) {
            bool done = false;
            V3 L = v3(0, 0, 0);
            if (depth < kp.max_depth) {
                if (r.htri < 0) {
                    done = true;
                } else {
                    const uint32_t gi = __float_as_uint(tris[3 * r.htri + 1].w);
                    const GpuGeom& g = geoms[gi];
                    if (g.Ka[0] > 0 || g.Ka[1] > 0 || g.Ka[2] > 0) {
                        L = v3(color.x * (g.Ka[0] * kp.illum), color.y * (g.Ka[1] * kp.illum),
                               color.z * (g.Ka[2] * kp.illum));
                        done = true;
                    } else {
                        c.shades++;
                        const float4 n1 = sc.normals[3 * r.htri], n2 = sc.normals[3 * r.htri + 1],
                                     n3 = sc.normals[3 * r.htri + 2];
                        V3 nrm = vadd(vadd(vscale(v3(n1.x, n1.y, n1.z), 1.0f - r.hbeta - r.hgamma),
                                           vscale(v3(n2.x, n2.y, n2.z), r.hbeta)),
                                      vscale(v3(n3.x, n3.y, n3.z), r.hgamma));
                        normalize_cu(nrm);
                        V3 dir = r.d;
                        if (g.Tr > 0) {
                            dir = sample_fresnel(sd, nrm, dir, g.Tr, g.Ni);
                            if (kp.fresnel_kd) color = v3(color.x * g.Kd[0], color.y * g.Kd[1], color.z * g.Kd[2]);
                        } else if (g.Ns > 1) {
                            dir = sample_phong(sd, nrm, dir, g.Ns_u);
                            color = v3(color.x * g.Ks[0], color.y * g.Ks[1], color.z * g.Ks[2]);
                        } else {
                            color = v3(color.x * g.Kd[0], color.y * g.Kd[1], color.z * g.Kd[2]);
                            if (dot3(dir, nrm) > 0) {
                                const V3 hd = sample_hemi(sd, nrm);
                                dir = v3(-hd.x, -hd.y, -hd.z);
                            } else {
                                dir = sample_hemi(sd, nrm);
                            }
                        }
                        // hitPoint = pos + t*dir at the accepted t (CUTracer.cu:89-91), then
                        // pos = hitPoint + dir*0.01 (:134,143,159)
                        const V3 hp = v3(r.o.x + r.best * r.d.x, r.o.y + r.best * r.d.y, r.o.z + r.best * r.d.z);
                        r.o = vadd(hp, vscale(dir, 0.01f));
                        r.d = dir;
                        depth++;
                        c.rays++;
                        mode = begin_ray(r, sc) ? kTrav : kReady;
                                    }
                }
            } else {
                if (r.htri >= 0) {
                    const uint32_t gi = __float_as_uint(tris[3 * r.htri + 1].w);
                    const GpuGeom& g = geoms[gi];
                    L = v3(color.x * (g.Ka[0] * kp.illum), color.y * (g.Ka[1] * kp.illum),
                           color.z * (g.Ka[2] * kp.illum));
                }
                done = true;
            }
            if (done) {
                part = vadd(part, L);
                s++;
                if (s == s_end) {
                    kp.partial[unit_id] = make_float4(part.x, part.y, part.z, 0.0f);   // [chunk][v]
                    if constexpr (DBG) {
                        uint32_t* uc = kp.unit_counters + 4 * (size_t)unit_id;
                        uc[0] = c.rays - c0.rays;
                        uc[1] = c.inner - c0.inner;
                        uc[2] = c.leaf - c0.leaf;
                        uc[3] = c.tests - c0.tests;
                    }
                    mode = kNeed;
                } else {
                    start_path();
                }
            }
        }
        MCPT_STAMP(tm_shade);
    }

#ifdef MCPT_PHASE_TIMING
    if (lane == 0) {
        atomicAdd(kp.stats + 8, tm_units);
        atomicAdd(kp.stats + 9, tm_trav);
        atomicAdd(kp.stats + 10, tm_shade);
        atomicAdd(kp.stats + 11, tm_iters);
    }
#endif
    // ---- counters: wave reduction, one atomic per wave per counter --------
    uint32_t vals[8] = {c.rays, c.paths, c.inner, c.leaf, c.refs, c.tests, c.shades, c.spills};
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t x = vals[i];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
        vals[i] = x;
    }
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < 8; i++) atomicAdd(kp.stats + i, (unsigned long long)vals[i]);
    }
}

// partial sums -> mean -> running mean (CUTracer.cu:214-217), chunk order
__global__ void __launch_bounds__(256) reduce_kernel(const KernelParams kp, float4* __restrict__ fb) {
    const uint32_t v = blockIdx.x * 256u + threadIdx.x;
    if (v >= kp.npix_local) return;
    int x, y;
    if (!unit_pixel(kp, v, x, y)) return;
    V3 sum = v3(0, 0, 0);
    for (uint32_t c = 0; c < kp.nchunks; c++) {
        const float4 p = kp.partial[(size_t)c * kp.npix_local + v];
        sum = vadd(sum, v3(p.x, p.y, p.z));
    }
    const V3 mean = vdiv(sum, (float)kp.spp);
    const size_t idx = kp.packed ? (size_t)v : (size_t)y * (size_t)kp.width + (size_t)x;
    float4 out;
    if (kp.prev_count == 0) {
        out = make_float4(mean.x, mean.y, mean.z, 0.0f);
    } else {
        const float4 pv = fb[idx];
        const float pc = (float)kp.prev_count, pc1 = (float)(kp.prev_count + 1u);
        out = make_float4((pv.x * pc + mean.x) / pc1, (pv.y * pc + mean.y) / pc1, (pv.z * pc + mean.z) / pc1, 0.0f);
    }
    fb[idx] = out;
}

template <bool IN_LDS, int S, int BLOCK>
hipError_t launch_path(const KernelParams& kp, int grid, size_t lds, hipStream_t st) {
    auto kern = kp.unit_counters ? path_kernel<IN_LDS, S, BLOCK, true> : path_kernel<IN_LDS, S, BLOCK, false>;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), lds, st, kp);
    return hipGetLastError();
}

}  // namespace

// LDS need of the in-LDS variant for a scene image of `image_bytes`
size_t lds_bytes_in_lds(uint32_t image_bytes, int S) { return (size_t)image_bytes + (size_t)S * kLdsBlock * 16; }

hipError_t launch_render(const KernelParams& kp_in, int cus, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1,
                         hipEvent_t ev2, float4* fb, int* variant_out) {
    KernelParams kp = kp_in;
    const uint32_t img = kp.scene.image_bytes;
    kp.lds_stack_off = lds_bytes_in_lds(img, 4) <= kMaxLds ? img : 0u;
    kp.total_lanes = (uint32_t)total_lanes_for(img, cus);
    hipError_t e = hipMemsetAsync(kp.counter, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    if (ev0) hipEventRecord(ev0, st);
    int variant = 0;
    if (lds_bytes_in_lds(img, 8) <= kMaxLds) {
        variant = 1;
        e = launch_path<true, 8, kLdsBlock>(kp, cus, lds_bytes_in_lds(img, 8), st);
    } else if (lds_bytes_in_lds(img, 4) <= kMaxLds) {
        variant = 2;
        e = launch_path<true, 4, kLdsBlock>(kp, cus, lds_bytes_in_lds(img, 4), st);
    } else {
        variant = 3;
        e = launch_path<false, 8, kGlobalBlock>(kp, cus * kGlobalBlocksPerCu, (size_t)8 * kGlobalBlock * 16, st);
    }
    if (e != hipSuccess) return e;
    if (ev1) hipEventRecord(ev1, st);
    hipLaunchKernelGGL(reduce_kernel, dim3((kp.npix_local + 255u) / 256u), dim3(256), 0, st, kp, fb);
    e = hipGetLastError();
    if (ev2) hipEventRecord(ev2, st);
    if (variant_out) *variant_out = variant;
    return e;
}

int total_lanes_for(uint32_t image_bytes, int cus) {
    if (lds_bytes_in_lds(image_bytes, 4) <= kMaxLds) return cus * kLdsBlock;
    return cus * kGlobalBlocksPerCu * kGlobalBlock;
}

}  // namespace mcpt
