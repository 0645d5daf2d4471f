// wavefront.hip -- wavefront (split-kernel) variant of the path tracer (C5,
// SURVEY.md §8(f)1).
//
// Same paths, same arithmetic as the megakernel (render.hip), reorganised as
// queues in HBM so that every kernel does one kind of work:
//   generate    one primary ray per (pixel, sample) of the batch, appended to
//               ray queue 0 (wave ballot + prefix compaction, one atomic/wave)
//   extend b    closest hit of every ray in queue b: persistent workgroups,
//               scene image in LDS (or global), lanes refill from the queue as
//               soon as their ray is done; the slot is appended to one of four
//               per-class lists (terminate / diffuse / phong / fresnel) -- the
//               material sort of the extend -> shade hand-off
//   shade b     one class list after another, so each wave runs ONE material
//               branch: radiance of terminated paths, or the scatter event and
//               the next ray appended (compacted) to queue b+1
//   accumulate  per pixel, the batch's samples summed in sample order into the
//               same [chunk][pixel] partial sums the megakernel writes
// followed by the megakernel's reduction.  The RNG is stateless per
// (pixel, sample) and every float operation is shared (trace_device.hpp), so
// the image is bit-identical to the megakernel's and the oracle's.  Queue
// order is scheduling-dependent but nothing reads it: a path's state is keyed
// by its path id.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mcpt_device.hpp"
#include "render_launch.hpp"
#include "trace_device.hpp"

namespace mcpt {

using namespace dev;
using namespace trace;

namespace {

constexpr int kGenBlock = 256;
constexpr int kShadeBlock = 256;
constexpr int kClassTerminate = 0;

__device__ __forceinline__ float4 pack(V3 v, uint32_t w) { return make_float4(v.x, v.y, v.z, __uint_as_float(w)); }
__device__ __forceinline__ V3 xyz(float4 v) { return v3(v.x, v.y, v.z); }

// ---- generate: primary rays of the batch (CUTracer.cu:186-211) -------------
__global__ void __launch_bounds__(kGenBlock) wf_generate(const KernelParams kp, const WfParams wf) {
    const uint32_t n = wf.nb * wf.ns;
    const V3 eye = v3(kp.eye[0], kp.eye[1], kp.eye[2]);
    Counters c = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint32_t stride = gridDim.x * kGenBlock;
    // wave-uniform trip count: every lane of a wave runs each iteration
    const uint32_t wave0 = (blockIdx.x * kGenBlock + threadIdx.x) & ~63u;
    for (uint32_t base = wave0; base < n; base += stride) {
        const uint32_t pid = base + (threadIdx.x & 63u);
        bool ok = false;
        V3 d = v3(0, 0, 0);
        if (pid < n) {
            const uint32_t s_local = pid / wf.nb;
            const uint32_t v = wf.v0 + (pid - s_local * wf.nb);
            int px, py;
            if (unit_pixel(kp, v, px, py)) {
                uint32_t sd;
                const uint32_t pix = (uint32_t)py * (uint32_t)kp.width + (uint32_t)px;
                primary_ray(kp, pix, px, py, wf.s_begin + s_local, sd, d);
                wf.pstate[pid] = make_float4(1.0f, 1.0f, 1.0f, __uint_as_float(sd));
                c.paths++;
                c.rays++;
                ok = true;
            } else {
                wf.radiance[pid] = make_float4(0, 0, 0, 0);
            }
        }
        const uint32_t slot = wave_append(ok, &wf.cnt[0].queued);
        if (ok) {
            wf.q_o[0][slot] = pack(eye, pid);
            wf.q_d[0][slot] = pack(d, 0u);
        }
    }
    flush_counters(c, kp.stats);
}

// ---- extend: closest hit of every queued ray --------------------------------
template <bool IN_LDS, int S, int BLOCK>
__global__ void __launch_bounds__(BLOCK) wf_extend(const KernelParams kp, const WfParams wf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    WfCounters* cn = wf.cnt + wf.bounce;
    const uint32_t count = cn->queued;
    if (count == 0) return;
    const int tid = (int)threadIdx.x;
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
        nodes = reinterpret_cast<const uint2*>(smem + sc.off_nodes) + 1;
        leafs = reinterpret_cast<const uint32_t*>(smem + sc.off_leafs);
        geoms = reinterpret_cast<const GpuGeom*>(smem + sc.off_geoms);
    } else {
        tris = reinterpret_cast<const float4*>(sc.image + sc.off_tris);
        nodes = reinterpret_cast<const uint2*>(sc.image + sc.off_nodes) + 1;
        leafs = reinterpret_cast<const uint32_t*>(sc.image + sc.off_leafs);
        geoms = reinterpret_cast<const GpuGeom*>(sc.image + sc.off_geoms);
    }
    uint4* st = reinterpret_cast<uint4*>(smem + kp.lds_stack_off) + tid;
    uint4* spill = kp.spill + (blockIdx.x * BLOCK + (uint32_t)tid);
    const uint32_t spill_stride = kp.total_lanes;
    const float4* qo = wf.q_o[wf.bounce & 1];
    const float4* qd = wf.q_d[wf.bounce & 1];

    Counters c = {0, 0, 0, 0, 0, 0, 0, 0};
    RayState r;
    r.htri = -1;
    int mode = kNeed;
    uint32_t slot = 0, depth = 0;
    for (;;) {
        // ---- refill idle lanes from the queue (one atomic per wave) ---------
        const uint32_t got = wave_append(mode == kNeed, &cn->fetched);
        if (mode == kNeed) {
            if (got >= count) {
                mode = kDead;
            } else {
                slot = got;
                const float4 o4 = qo[slot], d4 = qd[slot];
                r.o = xyz(o4);
                r.d = xyz(d4);
                depth = __float_as_uint(d4.w);
                mode = begin_ray(r, sc) ? kTrav : kReady;
            }
        }
        if (!__ballot(mode != kDead)) break;
        // ---- traversal burst until enough lanes are done ---------------------
        for (;;) {
            if (mode == kTrav) {
                if (trav_iter<S>(r, tris, nodes, leafs, st, BLOCK, spill, spill_stride, c)) mode = kReady;
            }
            const uint64_t trv = __ballot(mode == kTrav);
            const uint64_t rdy = __ballot(mode == kReady);
            if (!trv || __popcll(rdy) >= wf.refill_thresh) break;
        }
        // ---- hand-off: hit record + per-material class list -----------------
        uint32_t cls = 4u;
        if (mode == kReady) {
            wf.hit[slot] = make_float4(r.best, r.hbeta, r.hgamma, __int_as_float(r.htri));
            cls = kClassTerminate;
            if (r.htri >= 0 && (int32_t)depth < kp.max_depth) {
                const GpuGeom& g = geoms[__float_as_uint(tris[3 * r.htri + 1].w)];
                if (!is_emitter(g)) cls = material_class(g);
            }
            mode = kNeed;
        }
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t at = wave_append(cls == k, &cn->cls[k]);
            if (cls == k) wf.cls_list[(size_t)k * wf.capacity + at] = slot;
        }
    }
    flush_counters(c, kp.stats);
}

// ---- shade: one material class after another (CUTracer.cu:105-175) ----------
__global__ void __launch_bounds__(kShadeBlock) wf_shade(const KernelParams kp, const WfParams wf) {
    WfCounters* cn = wf.cnt + wf.bounce;
    WfCounters* nx = cn + 1;
    const GpuScene& sc = kp.scene;
    const float4* tris = reinterpret_cast<const float4*>(sc.image + sc.off_tris);
    const GpuGeom* geoms = reinterpret_cast<const GpuGeom*>(sc.image + sc.off_geoms);
    const float4* qo = wf.q_o[wf.bounce & 1];
    const float4* qd = wf.q_d[wf.bounce & 1];
    float4* qo2 = wf.q_o[(wf.bounce + 1) & 1];
    float4* qd2 = wf.q_d[(wf.bounce + 1) & 1];
    const int lane = (int)(threadIdx.x & 63u);
    Counters c = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t k = 0; k < 4; k++) {
        const uint32_t n = cn->cls[k];
        const uint32_t* list = wf.cls_list + (size_t)k * wf.capacity;
        for (;;) {
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&cn->taken[k], 64u);
            base = __shfl(base, 0);
            if (base >= n) break;
            const uint32_t i = base + (uint32_t)lane;
            bool cont = false;
            float4 o_next = make_float4(0, 0, 0, 0), d_next = make_float4(0, 0, 0, 0);
            if (i < n) {
                const uint32_t slot = list[i];
                const float4 o4 = qo[slot], d4 = qd[slot], h = wf.hit[slot];
                const uint32_t pid = __float_as_uint(o4.w);
                const uint32_t depth = __float_as_uint(d4.w);
                const int32_t htri = __float_as_int(h.w);
                const float4 ps = wf.pstate[pid];
                V3 color = xyz(ps);
                if (k == kClassTerminate) {
                    // miss -> 0; emitter -> color*Ka*ILLUM (:111-113); terminal query (:162-175)
                    V3 L = v3(0, 0, 0);
                    if (htri >= 0) {
                        const GpuGeom& g = geoms[__float_as_uint(tris[3 * htri + 1].w)];
                        if ((int32_t)depth >= kp.max_depth || is_emitter(g)) L = emitted(color, g, kp.illum);
                    }
                    wf.radiance[pid] = make_float4(L.x, L.y, L.z, 0.0f);
                } else {
                    c.shades++;
                    const GpuGeom& g = geoms[__float_as_uint(tris[3 * htri + 1].w)];
                    uint32_t sd = __float_as_uint(ps.w);
                    V3 o = xyz(o4), d = xyz(d4);
                    scatter(g, sc.normals, htri, h.y, h.z, h.x, kp.fresnel_kd, sd, color, o, d);
                    wf.pstate[pid] = pack(color, sd);
                    o_next = pack(o, pid);
                    d_next = pack(d, depth + 1u);
                    c.rays++;
                    cont = true;
                }
            }
            const uint32_t at = wave_append(cont, &nx->queued);
            if (cont) {
                qo2[at] = o_next;
                qd2[at] = d_next;
            }
        }
    }
    flush_counters(c, kp.stats);
}

// ---- accumulate: samples of the batch in sample order -> partial sums -------
__global__ void __launch_bounds__(256) wf_accumulate(const KernelParams kp, const WfParams wf) {
    const uint32_t u = blockIdx.x * 256u + threadIdx.x;
    if (u >= wf.nb) return;
    V3 part = v3(0, 0, 0);
    for (uint32_t s = 0; s < wf.ns; s++) part = vadd(part, xyz(wf.radiance[(size_t)s * wf.nb + u]));
    kp.partial[(size_t)wf.chunk_index * kp.npix_local + wf.v0 + u] = make_float4(part.x, part.y, part.z, 0.0f);
}

template <bool IN_LDS, int S, int BLOCK>
hipError_t launch_extend(const KernelParams& kp, const WfParams& wf, int grid, size_t lds, hipStream_t st) {
    auto kern = wf_extend<IN_LDS, S, BLOCK>;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), lds, st, kp, wf);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_wavefront(const KernelParams& kp_in, const WfParams& wf_in, int cus, int max_bounces,
                            hipStream_t st, hipEvent_t ev0, hipEvent_t ev1, hipEvent_t ev2, float4* fb,
                            int* variant_out) {
    KernelParams kp = kp_in;
    const uint32_t img = kp.scene.image_bytes;
    const bool in_lds = lds_bytes_in_lds(img, 4) <= kMaxLds;
    kp.lds_stack_off = in_lds ? img : 0u;
    kp.total_lanes = (uint32_t)total_lanes_for(img, cus);
    hipError_t e = hipSuccess;
    if (ev0) hipEventRecord(ev0, st);
    for (uint32_t chunk = 0; chunk < kp.nchunks; chunk++) {
        WfParams wf = wf_in;
        wf.chunk_index = chunk;
        wf.s_begin = chunk * kp.chunk;
        wf.ns = (kp.spp - wf.s_begin) < kp.chunk ? (kp.spp - wf.s_begin) : kp.chunk;
        const uint32_t nb_max = wf.capacity / wf.ns;
        for (uint32_t v0 = 0; v0 < kp.npix_local; v0 += nb_max) {
            wf.v0 = v0;
            wf.nb = (kp.npix_local - v0) < nb_max ? (kp.npix_local - v0) : nb_max;
            e = hipMemsetAsync(wf.cnt, 0, sizeof(WfCounters) * (size_t)(max_bounces + 1), st);
            if (e != hipSuccess) return e;
            const uint32_t n = wf.nb * wf.ns;
            const uint32_t gen_grid = (n + kGenBlock - 1) / kGenBlock;
            hipLaunchKernelGGL(wf_generate, dim3(gen_grid < 8u * (uint32_t)cus ? gen_grid : 8u * (uint32_t)cus),
                               dim3(kGenBlock), 0, st, kp, wf);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            for (int b = 0; b < max_bounces; b++) {
                wf.bounce = b;
                if (in_lds)
                    e = launch_extend<true, 4, kLdsBlock>(kp, wf, cus, lds_bytes_in_lds(img, 4), st);
                else
                    e = launch_extend<false, 8, kGlobalBlock>(kp, wf, cus * kGlobalBlocksPerCu,
                                                              (size_t)8 * kGlobalBlock * 16, st);
                if (e != hipSuccess) return e;
                hipLaunchKernelGGL(wf_shade, dim3(cus * 8), dim3(kShadeBlock), 0, st, kp, wf);
                if ((e = hipGetLastError()) != hipSuccess) return e;
            }
            hipLaunchKernelGGL(wf_accumulate, dim3((wf.nb + 255u) / 256u), dim3(256), 0, st, kp, wf);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
    }
    if (ev1) hipEventRecord(ev1, st);
    e = launch_reduce(kp, fb, st);
    if (ev2) hipEventRecord(ev2, st);
    if (variant_out) *variant_out = in_lds ? 4 : 5;
    return e;
}

}  // namespace mcpt
