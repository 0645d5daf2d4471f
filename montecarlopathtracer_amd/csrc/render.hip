// render.hip -- MI355X (gfx950) path-tracing megakernel and its host launcher.
//
// Replaces rayTraceKernel (CVMCTracer/CUDA/CUTracer.cu:179-218, one thread per
// pixel, brute-force intersect :44-96) with:
//   * persistent workgroups (one 1024-thread workgroup per CU when the scene
//     image fits in LDS) that pull work units (pixel, sample-chunk) from a
//     device counter, one atomic per wave per 64 units (__ballot / popcount);
//   * path regeneration: a lane whose path ends immediately starts the next
//     sample of its unit; traversal bursts alternate with shading rounds
//     (raised wave priority) for the lanes whose closest hit is known;
//   * the scene image (triangles, KD nodes, leaf ids, materials) copied into
//     LDS once per workgroup; the KD traversal stack keeps up to S entries in
//     LDS (lane-strided, conflict-free, managed lazily) and older ones in
//     global memory;
//   * the RNG seed of every path from its (pixel, sample) by a PCG hash, at the
//     path's start (stateless: any scheduling draws the same streams);
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
#include "trace_device.hpp"

namespace mcpt {

using namespace dev;
using namespace trace;

namespace {

// Both layouts run 16 waves per CU and need <= 128 VGPRs; keep an eye on the
// global variant (at 130 it lost a quarter of its occupancy: C4 -20%).  An
// explicit min-waves bound (__launch_bounds__(BLOCK, 4)) made it slower (C4
// 1.81 vs 1.97 G rays/s), so the budget is kept by the code instead.  Five
// lean workgroups per CU (LDS fits 5 x 32 KB; bound 5 -> 96 VGPRs, no scratch)
// lost 3.7% on C4 against four.
// sum of a unit's samples -> partial[chunk][v], or one tail sample's radiance
__device__ __forceinline__ void store_part(const KernelParams& kp, uint32_t id, V3 part) {
    const float4 val = make_float4(part.x, part.y, part.z, 0.0f);
    if (id & 0x80000000u)
        kp.tail_buf[id & 0x7FFFFFFFu] = val;
    else
        kp.partial[id] = val;
}

template <bool IN_LDS, int S, int BLOCK, bool DBG, bool QE, bool COUNT>
// counting kernels of the global layout are held to 4 waves per SIMD (128 VGPRs)
// by the launch bound; the lean (timed) kernels fit without it
__global__ void __launch_bounds__(BLOCK, (!IN_LDS && COUNT) ? 4 : 1) path_kernel(const KernelParams kp) {
    static_assert((BLOCK & (BLOCK - 1)) == 0, "stack slot addresses (slot_of) mask by a power-of-two block");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = (int)threadIdx.x;
    const int lane = tid & 63;
    const GpuScene& sc = kp.scene;

    const float4* tris;
    const uint2* nodes;
    const uint32_t* leafs;
    const GpuGeom* geoms;
    // LDS: [traversal stack S x BLOCK x 16 B | scene image].  The stack at LDS
    // address 0 makes a slot address (sp & (S-1)) << log2(BLOCK*16) | tid * 16:
    // fewer instructions per push and pop than an offset base
    unsigned char* const lds_image = smem + (size_t)S * BLOCK * 16;
    if constexpr (IN_LDS) {
        const uint4* src = reinterpret_cast<const uint4*>(sc.image);
        uint4* dst = reinterpret_cast<uint4*>(lds_image);
        const uint32_t n16 = sc.image_bytes / 16u;
        for (uint32_t i = (uint32_t)tid; i < n16; i += BLOCK) dst[i] = src[i];
        __syncthreads();
        tris = reinterpret_cast<const float4*>(lds_image + sc.off_tris);
        nodes = reinterpret_cast<const uint2*>(lds_image + sc.off_nodes) + 1;   // node i at slot i+1
        leafs = reinterpret_cast<const uint32_t*>(lds_image + sc.off_leafs);
        geoms = reinterpret_cast<const GpuGeom*>(lds_image + sc.off_geoms);
    } else {
        tris = reinterpret_cast<const float4*>(sc.image + sc.off_tris);
        nodes = reinterpret_cast<const uint2*>(sc.image + sc.off_nodes) + 1;
        leafs = reinterpret_cast<const uint32_t*>(sc.image + sc.off_leafs);
        geoms = reinterpret_cast<const GpuGeom*>(sc.image + sc.off_geoms);
    }
    const uint4* pairs = reinterpret_cast<const uint4*>(sc.image + sc.off_nodes);   // 48-B pair records (global variant)
    uint4* st = reinterpret_cast<uint4*>(smem) + tid;   // [S][BLOCK] x 16 B
    const uint32_t gl = blockIdx.x * BLOCK + (uint32_t)tid;
    uint4* spill = kp.spill + gl;
    const uint32_t spill_stride = kp.total_lanes;
    const V3 eye = v3(kp.eye[0], kp.eye[1], kp.eye[2]);

    Counters c = {0, 0, 0, 0, 0, 0, 0, 0};
    Counters c0 = c;   // DBG builds only
#ifdef MCPT_PHASE_TIMING
    LaneUse lu = {0, 0, 0, 0, 0, 0};
#endif
    int mode = kNeed;
    SlotCursor units = {0, kChunk};
    uint32_t s = 0, s_end = 0, unit_id = 0;
    int px = 0, py = 0, depth = 0;
    uint32_t sd = 1;
    V3 part = v3(0, 0, 0), color = v3(1, 1, 1);
    RayState r;
    r.o = eye;
    r.d = v3(0, 0, -1);
    r.htri = -1;

    // sample s of the current unit: its primary ray (the caller then starts it)
    auto new_path = [&]() {
        sd = path_seed(kp, (uint32_t)py * (uint32_t)kp.width + (uint32_t)px, s);
        if constexpr (QE) {
            primary_ray_qe_sd(kp, px, py, sd, r.o, r.d);
        } else {
            primary_ray_sd(kp, px, py, sd, r.d);
            r.o = eye;
        }
        color = v3(1, 1, 1);
        depth = 0;
        if constexpr (COUNT) c.paths++;
    };
    // next query of this lane: count it, root interval (one inlined copy per phase)
    auto start_ray = [&]() {
        c.rays++;
        mode = begin_ray(r, sc, kp.best_init) ? kTrav : kReady;
    };

#ifdef MCPT_PHASE_TIMING
    unsigned long long tm_units = 0, tm_trav = 0, tm_shade = 0, tm_iters = 0, tm_scatter = 0, tm_t0;
#define MCPT_STAMP(acc) do { unsigned long long t1_ = __builtin_amdgcn_s_memtime(); acc += t1_ - tm_t0; tm_t0 = t1_; } while (0)
    tm_t0 = __builtin_amdgcn_s_memtime();
#else
#define MCPT_STAMP(acc) do {} while (0)
#endif
    // Main loop: a shading round for the ready lanes (raised issue priority:
    // a wave in its short round gets back to traversal sooner while the other
    // waves' bursts fill the gaps, +0.6%), the work-unit handout for lanes whose
    // unit is done, the next rays of all of them, then a traversal burst.  The
    // first round finds every lane needing a unit.  Lanes starting a path (a new
    // unit's first sample or a unit's next sample) and lanes scattering share
    // one instruction stream for their two uniforms, the normalize (primary
    // direction / shading normal) and the root interval, so each runs once per
    // round however the lanes split (CV mode).
    for (;;) {
        __builtin_amdgcn_s_setprio(1);
        bool scat = false, newp = false;   // this lane scatters / starts a path in this round
        uint32_t gi = 0;                   // geometry of the hit (scatter lanes)
        if (mode == kReady) {
            // ---- shading (CUTracer.cu:105-175; QE rtx.hlsl:309-370) ----
            const bool hit = r.htri >= 0;
            if (hit) gi = __float_as_uint(tris[r.htri + 1].w);
            const GpuGeom& g = geoms[gi];
            bool emit = false;
            if constexpr (QE) {
                // miss or bounce >= 3*depth ends the path; roulette from bounce `depth`
                // on; emitters return color*Ka (no ILLUM)
                const bool alive = hit && depth < 3 * kp.max_depth &&
                                   !(depth >= kp.max_depth && !qe_roulette(sd, color));
                emit = alive && is_emitter(g);
                scat = alive && !emit;
            } else {
                emit = hit && (is_emitter(g) || depth >= kp.max_depth);   // the terminal query collects Ka
                scat = hit && !emit;
            }
            MCPT_STAMP(tm_scatter);
            if (!scat) {
                const V3 L = emit ? emitted(color, g, QE ? 1.0f : kp.illum) : v3(0, 0, 0);
                part = vadd(part, L);
                s++;
                if (s == s_end) {
                    store_part(kp, unit_id, part);
                    if constexpr (DBG) {
                        uint32_t* uc = kp.unit_counters + 4 * (size_t)unit_id;
                        uc[0] = c.rays - c0.rays;
                        uc[1] = c.inner - c0.inner;
                        uc[2] = c.leaf - c0.leaf;
                        uc[3] = c.tests - c0.tests;
                    }
                    mode = kNeed;
                } else {
                    newp = true;
                }
            }
        }
        MCPT_STAMP(tm_shade);

        // ---- work units: one atomic per wave for every lane that needs one ----
        for (;;) {
            const uint64_t m = __ballot(mode == kNeed);
            if (!m) break;
            uint32_t unit;
            if constexpr (IN_LDS) {
                unit = units.take(mode == kNeed, kp.counter);   // 64 items per atomic
            } else {
                // scenes in global memory: units strictly in global order, one atomic
                // per refill (C4 1.94 vs 1.69 G rays/s with 64-unit wave chunks)
                const int leader = __ffsll((unsigned long long)m) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(kp.counter, (uint32_t)__popcll(m));
                unit = __shfl(base, leader) + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            }
            if (mode == kNeed) {
                if (unit >= kp.total_items) {
                    mode = kDead;
                } else {
                    // item -> unit u (+ one sample j of it in the tail split)
                    uint32_t u = unit, j = 0, cnt = kp.chunk;
                    const bool single = unit >= kp.tail_units;
                    if (single) {
                        const uint32_t k = unit - kp.tail_units;
                        const uint32_t q = kp.div_chunk.div(k);
                        u = kp.tail_units + q;
                        j = k - q * kp.chunk;
                        cnt = 1;
                    }
                    const uint32_t chunk = kp.div_npix.div(u);
                    const uint32_t v = u - chunk * kp.npix_local;
                    s = chunk * kp.chunk + j;
                    s_end = min(s + cnt, kp.spp);
                    // partial index, or the tail sample's slot with the top bit set
                    unit_id = single ? (0x80000000u | (unit - kp.tail_units)) : u;
                    if constexpr (DBG) c0 = c;
                    part = v3(0, 0, 0);
                    if (s >= s_end) {
                        // sample past spp in a ragged last chunk: nothing to do, take another item
                    } else if (unit_pixel(kp, v, px, py)) {
                        newp = true;
                        mode = kReady;
                    } else {
                        store_part(kp, unit_id, part);
                    }
                }
            }
        }
        if (!__ballot(mode != kDead)) break;
        if constexpr (!DBG) bound_counters<COUNT>(c, kp.stats);   // (DBG: per-unit deltas of c)
        MCPT_STAMP(tm_units);

        // ---- next rays: scattered rays and the first rays of new paths ----
        if constexpr (QE) {
            if (newp) new_path();
            if (scat) {
                if constexpr (COUNT) c.shades++;
                scatter<true>(geoms[gi], sc.normals, r.htri, r.hbeta, r.hgamma, r.best, 0, sd, color, r.o, r.d);
                depth++;
            }
        } else {
            const bool fres = scat && geoms[gi].Tr > 0;
            if (newp) sd = path_seed(kp, (uint32_t)py * (uint32_t)kp.width + (uint32_t)px, s);
            // the lane's next two uniforms (a Fresnel scatter consumes only the first):
            // the primary ray's jitter (CUTracer.cu:189-190) or the sampler's draws
            float u1 = 0.0f, u2 = 0.0f;
            if (scat | newp) {
                uint32_t s1 = sd;
                u1 = rng_next(s1);
                uint32_t s2 = s1;
                u2 = rng_next(s2);
                sd = fres ? s1 : s2;
            }
            V3 vec = v3(0, 0, 0);
            if (scat) vec = shading_normal_raw(sc.normals, r.htri, r.hbeta, r.hgamma);
            if (newp) vec = primary_dir_raw(kp, px, py, u1, u2);
            if (scat | newp) normalize_cu(vec);
            if (newp) {
                r.d = vec;
                r.o = eye;
                color = v3(1, 1, 1);
                depth = 0;
                if constexpr (COUNT) c.paths++;
            }
            if (scat) {
                if constexpr (COUNT) c.shades++;
                scatter_u(geoms[gi], vec, u1, u2, r.best, kp.fresnel_kd, color, r.o, r.d);
                depth++;
            }
        }
        if (scat | newp) start_ray();
        MCPT_STAMP(tm_shade);

        // ---- traversal burst: until ready_thresh lanes are ready to shade ----
        __builtin_amdgcn_s_setprio(0);
        for (;;) {
#ifdef MCPT_PHASE_TIMING
            tm_iters++;
            {
                const uint64_t tv = __ballot(mode == kTrav);
                if (lane == 0) { lu.burst_w += 1; lu.burst_l += (unsigned long long)__popcll(tv); }
            }
#endif
            if (mode == kTrav) {
                if (trav_iter<S, !IN_LDS, COUNT, IN_LDS>(r, tris, nodes, leafs, st, BLOCK, spill, spill_stride, c MCPT_LU_ARG, pairs))
                    mode = kReady;
            }
            const uint64_t trv = __ballot(mode == kTrav);
            const uint64_t rdy = __ballot(mode == kReady);
            if (!trv || (int)__popcll(rdy) >= kp.ready_thresh) break;
        }
        MCPT_STAMP(tm_trav);
    }

#ifdef MCPT_PHASE_TIMING
    if (lane == 0) {
        atomicAdd(kp.stats + 8, tm_units);
        atomicAdd(kp.stats + 9, tm_trav);
        atomicAdd(kp.stats + 10, tm_shade);
        atomicAdd(kp.stats + 11, tm_iters);
        atomicAdd(kp.stats + 12, tm_scatter);
    }
    {
        unsigned long long* g = reinterpret_cast<unsigned long long*>(&g_lane_use);
        const unsigned long long v[6] = {lu.desc_w, lu.desc_l, lu.tri_w, lu.tri_l, lu.burst_w, lu.burst_l};
        for (int i = 0; i < 6; i++) {
            unsigned long long x = v[i];
            for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
            if (lane == 0) atomicAdd(g + i, x);
        }
    }
#endif
    flush_counters(c, kp.stats);
}

// running mean of a pixel (CUTracer.cu:214-217; QE gamma-space, rtx.hlsl:401-402):
// the old framebuffer value pv (read only when prev_count > 0) and this call's mean
__device__ __forceinline__ float4 running_mean(float4 pv, V3 mean, uint32_t prev_count, int32_t mode) {
    if (mode == kModeQE) {
        if (!prev_count) pv = make_float4(0, 0, 0, 0);
        return make_float4(qe_blend(pv.x, mean.x, prev_count), qe_blend(pv.y, mean.y, prev_count),
                           qe_blend(pv.z, mean.z, prev_count), 0.0f);
    }
    if (prev_count == 0) return make_float4(mean.x, mean.y, mean.z, 0.0f);
    const float pc = (float)prev_count, pc1 = (float)(prev_count + 1u);
    return make_float4((pv.x * pc + mean.x) / pc1, (pv.y * pc + mean.y) / pc1, (pv.z * pc + mean.z) / pc1, 0.0f);
}

// partial sums -> mean -> running mean (CUTracer.cu:214-217), chunk order
__global__ void __launch_bounds__(256) reduce_kernel(const KernelParams kp, float4* __restrict__ fb) {
    const uint32_t v = blockIdx.x * 256u + threadIdx.x;
    if (v >= kp.npix_local) return;
    int x, y;
    if (!unit_pixel(kp, v, x, y)) return;
    V3 sum = v3(0, 0, 0);
    for (uint32_t c = 0; c < kp.nchunks; c++) {
        const uint32_t u = c * kp.npix_local + v;
        V3 pc;
        if (u >= kp.tail_units) {   // tail split: the unit's samples, in sample order
            const float4* tb = kp.tail_buf + (size_t)(u - kp.tail_units) * kp.chunk;
            const uint32_t n = min(kp.chunk, kp.spp - c * kp.chunk);
            pc = v3(0, 0, 0);
            for (uint32_t j = 0; j < n; j++) pc = vadd(pc, v3(tb[j].x, tb[j].y, tb[j].z));
        } else {
            const float4 p = kp.partial[u];
            pc = v3(p.x, p.y, p.z);
        }
        sum = vadd(sum, pc);
    }
    const V3 mean = vdiv(sum, (float)kp.spp);
    const size_t idx = kp.packed ? (size_t)v : (size_t)y * (size_t)kp.width + (size_t)x;
    if (kp.raw_mean) {
        fb[idx] = make_float4(mean.x, mean.y, mean.z, 0.0f);
        return;
    }
    const bool old = kp.prev_count != 0;
    fb[idx] = running_mean(old ? fb[idx] : make_float4(0, 0, 0, 0), mean, kp.prev_count, kp.mode);
}

// multi-device gather: shard r's packed means -> row-major running mean
__global__ void __launch_bounds__(256) gather_kernel(const GatherParams g) {
    const uint32_t v = blockIdx.x * 256u + threadIdx.x;
    const uint32_t r = blockIdx.y;
    if (v >= g.slot) return;
    const uint32_t T = (uint32_t)g.tile, T2 = T * T;
    const uint32_t k = v / T2, w = v - k * T2;
    const uint64_t t = (uint64_t)r + (uint64_t)k * (uint32_t)g.nshards;
    const uint32_t tx = (uint32_t)(t % (uint32_t)g.tiles_x), ty = (uint32_t)(t / (uint32_t)g.tiles_x);
    const uint32_t x = tx * T + w % T, y = ty * T + w / T;
    if (x >= (uint32_t)g.width || y >= (uint32_t)g.height) return;   // also t past the last tile
    const float4 m = g.src[(size_t)r * g.slot + v];
    const size_t idx = (size_t)y * (size_t)g.width + x;
    g.fb[idx] = running_mean(g.prev_count ? g.fb[idx] : make_float4(0, 0, 0, 0), v3(m.x, m.y, m.z), g.prev_count,
                             g.mode);
}

// Closest-hit batch (mcpt_intersect): the reference's intersect()
// (CUTracer.cu:44-96) for caller-given rays, through the traversal the path
// kernel runs -- trav_iter on the scene image in global memory, the stack's
// top entries in LDS -- one ray per lane.  Output per ray: the triangle's
// image slot (-1: miss) and (beta, gamma, t).  Lanes past n run a dummy ray
// so every lane reaches the wave-level counter flush.
template <bool BOXES, int S>
__global__ void __launch_bounds__(kQueryBlock) query_kernel(const QueryParams q) {
    static_assert((kQueryBlock & (kQueryBlock - 1)) == 0, "stack slot addresses (slot_of) mask by a power-of-two block");
    __shared__ uint4 stk[S * kQueryBlock];
    const GpuScene& sc = q.scene;
    const int tid = (int)threadIdx.x;
    const uint32_t i = blockIdx.x * kQueryBlock + (uint32_t)tid;
    const bool live = i < q.n;
    const float4* tris = reinterpret_cast<const float4*>(sc.image + sc.off_tris);
    const uint2* nodes = reinterpret_cast<const uint2*>(sc.image + sc.off_nodes) + 1;
    const uint32_t* leafs = reinterpret_cast<const uint32_t*>(sc.image + sc.off_leafs);
    const uint4* pairs = reinterpret_cast<const uint4*>(sc.image + sc.off_nodes);
    Counters c = {0, 0, 0, 0, 0, 0, 0, 0};
#ifdef MCPT_PHASE_TIMING
    LaneUse lu = {0, 0, 0, 0, 0, 0};
#endif
    RayState r;
    r.o = live ? v3(q.o[3 * i], q.o[3 * i + 1], q.o[3 * i + 2]) : v3(0, 0, 0);
    r.d = live ? v3(q.d[3 * i], q.d[3 * i + 1], q.d[3 * i + 2]) : v3(0, 0, 1);
    if (live) c.rays++;
    if (begin_ray(r, sc, q.best_init) && live)
        while (!trav_iter<S, BOXES, true>(r, tris, nodes, leafs, stk + tid, kQueryBlock, q.spill + i, q.n,
                                          c MCPT_LU_ARG, pairs)) {
        }
    if (live) {
        q.slot[i] = r.htri < 0 ? -1 : r.htri / 3;
        q.hit[3 * i] = r.hbeta;
        q.hit[3 * i + 1] = r.hgamma;
        q.hit[3 * i + 2] = r.htri < 0 ? 0.0f : r.best;
    }
    flush_counters(c, q.stats);
}

template <bool IN_LDS, int S, int BLOCK>
hipError_t launch_path(const KernelParams& kp, int grid, size_t lds, hipStream_t st) {
    const bool qe = kp.mode == kModeQE;
    auto kern = kp.unit_counters
                    ? (qe ? path_kernel<IN_LDS, S, BLOCK, true, true, true> : path_kernel<IN_LDS, S, BLOCK, true, false, true>)
                : kp.lean ? (qe ? path_kernel<IN_LDS, S, BLOCK, false, true, false>
                                : path_kernel<IN_LDS, S, BLOCK, false, false, false>)
                          : (qe ? path_kernel<IN_LDS, S, BLOCK, false, true, true>
                                : path_kernel<IN_LDS, S, BLOCK, false, false, true>);
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
    kp.total_lanes = (uint32_t)total_lanes_for(img, cus);
    hipError_t e = hipMemsetAsync(kp.counter, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    if (ev0 && (e = hipEventRecord(ev0, st)) != hipSuccess) return e;
    int variant = 0;
    if (kp.scene.node_boxes) {                     // image built for global memory
        variant = 3;
        e = launch_path<false, 8, kGlobalBlock>(kp, cus * kGlobalBlocksPerCu, (size_t)8 * kGlobalBlock * 16, st);
    } else if (lds_bytes_in_lds(img, 8) <= kMaxLds) {
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
    if (ev1 && (e = hipEventRecord(ev1, st)) != hipSuccess) return e;
    e = launch_reduce(kp, fb, st);
    if (e == hipSuccess && ev2) e = hipEventRecord(ev2, st);
    if (variant_out) *variant_out = variant;
    return e;
}

#ifdef MCPT_PHASE_TIMING
void read_lane_use(unsigned long long out[6]) {   // megakernel lane-use counters, then reset
    LaneUse z = {0, 0, 0, 0, 0, 0};
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lane_use), sizeof z);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_lane_use), &z, sizeof z);
}
#endif

hipError_t launch_reduce(const KernelParams& kp, float4* fb, hipStream_t st) {
    hipLaunchKernelGGL(reduce_kernel, dim3((kp.npix_local + 255u) / 256u), dim3(256), 0, st, kp, fb);
    return hipGetLastError();
}

hipError_t launch_query(const QueryParams& q, hipStream_t st) {
    if (!q.n) return hipSuccess;
    const dim3 grid((q.n + kQueryBlock - 1) / kQueryBlock);
    if (q.scene.node_boxes)
        hipLaunchKernelGGL((query_kernel<true, 8>), grid, dim3(kQueryBlock), 0, st, q);
    else
        hipLaunchKernelGGL((query_kernel<false, 4>), grid, dim3(kQueryBlock), 0, st, q);
    return hipGetLastError();
}

hipError_t launch_gather(const GatherParams& g, hipStream_t st) {
    if (!g.slot || g.nshards < 1) return hipSuccess;
    hipLaunchKernelGGL(gather_kernel, dim3((g.slot + 255u) / 256u, (uint32_t)g.nshards), dim3(256), 0, st, g);
    return hipGetLastError();
}

int total_lanes_for(uint32_t image_bytes, int cus) {
    // an image that fits in LDS is built without leaf boxes (capi.cpp build_image)
    if (lds_bytes_in_lds(image_bytes, 4) + 32 <= kMaxLds) return cus * kLdsBlock;
    return cus * (kGlobalBlocksPerCu > kWfGlobalSegsPerCu ? kGlobalBlocksPerCu : kWfGlobalSegsPerCu) * kGlobalBlock;
}

}  // namespace mcpt
