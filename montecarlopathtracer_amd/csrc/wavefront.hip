// wavefront.hip -- wavefront (split-kernel) variant of the path tracer (C5,
// SURVEY.md §8(f)1).
//
// Same paths, same arithmetic as the megakernel (render.hip), reorganised as
// queues in HBM so that every kernel does one kind of work:
//   generate    one primary ray per (pixel, sample) of the batch into ray
//               queue 0, path groups (an 8x8 tile; 256 tiles for scenes in
//               global memory) dealt to the segments round-robin; in CV mode
//               with queue-order shading only the direction stream is
//               written (MCPT_WF_IMPLICIT0: the origin is the eye, and bounce
//               0's shade recomputes the path state from the slot)
//   extend b    closest hit of every ray in queue b: one persistent workgroup
//               per queue segment, scene image in LDS (or global); waves
//               reserve slots 64 at a time from an LDS counter, each lane
//               prefetches its next ray while tracing the current one and
//               refills as soon as it is done; it writes the slot's hit id
//   shade b     each segment's queue b in blocks of slots: radiance of
//               terminated paths, or the scatter event whose next ray goes to
//               the next free slot of the segment's queue b+1 (per-bounce
//               compaction by one LDS atomic per wave); with the material sort
//               (wf_sort = 1) each block is first sorted by material in LDS, so
//               a wave runs one material branch
//   accumulate  per pixel, the batch's samples summed in sample order into the
//               same [chunk][pixel] partial sums the megakernel writes
// followed by the megakernel's reduction.  A path never leaves its segment,
// so no kernel touches a device-wide atomic (one shared counter serialised
// ~0.5 M returning atomics per launch in the first version: 85% of wave
// cycles parked).  The RNG is stateless per (pixel, sample) and every float
// operation is shared (trace_device.hpp), so the image is bit-identical to the
// megakernel's and the oracle's; queue order is scheduling-dependent but
// nothing reads it: a path's state is keyed by its path id.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "mcpt_device.hpp"
#include "render_launch.hpp"
#include "trace_device.hpp"


// MCPT_WF_PRIMARY_TU = 1 (wavefront_primary.hip): this file compiled for the
// bounce-0 packet extend alone, in a translation unit of its own so that it
// can take its own code-generation flags (_build.py: its wave-uniform control
// flow left unstructurized); every other kernel and the host launch code are
// compiled here with MCPT_WF_PRIMARY_TU = 0.
#ifndef MCPT_WF_PRIMARY_TU
#define MCPT_WF_PRIMARY_TU 0
#endif

namespace mcpt {

using namespace dev;
using namespace trace;

namespace {

constexpr int kGenBlock = 256;
constexpr int kClassTerminate = 0;
// Rays are carried as (o.xyz, pid) and (d.xyz, depth); depth kNoRay marks a
// queue slot without a ray (pixel outside the image): it ends as a miss with
// zero radiance and is counted nowhere, like the megakernel's empty units.
constexpr uint32_t kNoRay = 0xFFFFFFFFu;

__device__ __forceinline__ float opaque(float x) {
    float y;
    asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
    return y;
}
__device__ __forceinline__ float4 pack(V3 v, uint32_t w) { return make_float4(v.x, v.y, v.z, __uint_as_float(w)); }

// Queue layout: field k of slot j (kQO {o, pid}, kQD {d, depth}, kQPS
// {throughput, rng}: SoA float4 streams of slot_stride entries each, then
// kQHIT, the 4-B hit ids) -- extend's ray reads and hit writes are dense lane
// streams (64-B AoS records: generate 9 -> 33 ms per C2 frame, round 2).
// WfParams::sort (mcpt_render_params::wf_sort): 0 (default) -- shade takes its
// segment's queue in slot order, dense streams, the merged samplers absorbing
// the material mix; 1 -- shade sorts each block of slots by material first
// (wf_shade_slots SORTB).  Either way continuing rays go to the next queue
// with one LDS atomic per wave.  (Until round 6 the sort went through
// per-class slot lists that extend appended to and shade gathered from: 9.5
// against 13.6 G rays/s for the block sort on C2, PERFLOG row 156.)
__device__ __forceinline__ size_t qf(uint32_t slot, uint32_t k, uint32_t stride) {
    return (size_t)k * stride + slot;
}
// queue streams: origin + path id, direction + depth, throughput + RNG state,
// hit (last: it holds only 4-B triangle ids, so the queue is 3 x 16 + 4 B per
// slot)
constexpr uint32_t kQO = 0, kQD = 1, kQPS = 2, kQHIT = 3;
__device__ __forceinline__ V3 xyz(float4 v) { return v3(v.x, v.y, v.z); }

// Queue streams are touched once per bounce: MCPT_WF_NT marks the streaming
// reads (bit 0) and writes (bit 1) of generate, shade and extend's ray reads
// non-temporal, so that they do not push extend's partially written hit lines
// out of the L2.  Default 3 (C2 wavefront +3.5%, C4 +2%; the 4-B hit ids
// themselves are plain stores, PERFLOG row 79).
#ifndef MCPT_WF_NT
#define MCPT_WF_NT 3
#endif
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldq(const float4* p) {
#if MCPT_WF_NT & 1
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
__device__ __forceinline__ void stq(float4* p, float4 v) {
#if MCPT_WF_NT & 2
    const f32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f32x4*>(p));
#else
    *p = v;
#endif
}

// Group k of block b (b-th run of nseg consecutive groups) -> its segment:
// every block deals one group to each segment, rotated by a hash of b.  With
// a plain k -> k (an image of 2^14 8x8 tiles, 256 segments) each segment got
// the same 64 tiles for every sample -- a fixed stripe of the image, whose
// cost differs from the others' and left CUs idle at the end of every extend.
// WfParams::xcd_deal (global-memory scenes, MCPT_WF_XCD): the rotation is a
// multiple of 8, so group k of every block goes to a segment g = k (mod 8).
// Extend and shade workgroup g (one per segment) is dispatched to XCD g mod 8,
// and a group's image region (a 1024x16 strip of 2^14 paths) is k mod (regions
// per sample): every sample of a region then runs on the same XCD, whose L2
// and the caches behind it serve the part of the scene image that region's
// paths walk.  C4 +1.6% (9.31 / 9.34 -> 9.48 / 9.48 G rays/s; serialized
// extends 880 -> 771 ms per two frames at the same L2 hit rate, 0.776 /
// 0.778); LDS scenes keep the finer rotation (C2 -2.3% with it: the coarser
// rotation balances the segments' work less well).
#ifndef MCPT_WF_XCD
#define MCPT_WF_XCD 1
#endif
__device__ __forceinline__ uint32_t seg_of(uint32_t k, uint32_t b, uint32_t nseg, bool xcd) {
    const uint32_t rot = (MCPT_WF_XCD && xcd && (nseg & 7u) == 0u)
                             ? (uint32_t)(((uint64_t)(b * 2654435761u) * (nseg >> 3)) >> 32) << 3
                             : (uint32_t)(((uint64_t)(b * 2654435761u) * nseg) >> 32);
    const uint32_t g = k + rot;
    return g >= nseg ? g - nseg : g;
}

// Inverse of generate's dealing: path id of local slot j of segment g's queue 0.
__device__ __forceinline__ uint32_t slot_pid(const WfParams& wf, uint32_t g, uint32_t j) {
    const uint32_t gs = wf.group_shift, blk = j >> gs;
    const uint32_t rot = seg_of(0, blk, wf.nseg, wf.xcd_deal);
    const uint32_t k = g >= rot ? g - rot : g + wf.nseg - rot;
    return ((blk * wf.nseg + k) << gs) | (j & ((1u << gs) - 1u));
}

// Length of segment g's queue 0 for the batch: its whole groups (the last
// group of the batch may be partial).  Written by generate, or by the
// generate-free bounce-0 extend (MCPT_WF_GEN0).
__device__ __forceinline__ uint32_t seg_queue0_len(const WfParams& wf, uint32_t g) {
    const uint32_t n = wf.nb * wf.ns;
    const uint32_t gs = wf.group_shift, gm = (1u << gs) - 1u;
    const uint32_t ngroups = (n + gm) >> gs;
    const uint32_t full = ngroups / wf.nseg, rem = ngroups - full * wf.nseg;
    // block `full` (partial, rem groups) covers segments rot, rot+1, ... (mod nseg)
    const uint32_t k = (g + wf.nseg - seg_of(0, full, wf.nseg, wf.xcd_deal)) % wf.nseg;
    uint32_t len = (full + (k < rem ? 1u : 0u)) << gs;
    const uint32_t lb = (ngroups - 1u) / wf.nseg;            // block of the last group
    if (seg_of(ngroups - 1u - lb * wf.nseg, lb, wf.nseg, wf.xcd_deal) == g) len -= (ngroups << gs) - n;
    return len;
}

// MCPT_WF_IMPLICIT0 = 1: bounce 0's shade (queue order, CV mode) recomputes a
// primary ray's origin, direction and RNG state from its slot instead of
// reading them, and generate skips the {throughput, rng} stream (64 B of
// queue traffic less per path); 2 (default): also the {o, pid} stream
// (extend's bounce-0 origins are the eye; 32 B more).  With MCPT_WF_NT = 3:
// level 1 C2 wavefront +0.3%, level 2 +0.9% (C4 +1.4%).
#ifndef MCPT_WF_IMPLICIT0
#define MCPT_WF_IMPLICIT0 2
#endif
__host__ __device__ __forceinline__ bool implicit0(const KernelParams& kp, const WfParams& wf) {
    return MCPT_WF_IMPLICIT0 && kp.mode != kModeQE;
}
// Hit ids: extend writes only the hit triangle's id (4 B, the
// first quarter of the hit stream as i32) and shade recomputes t, beta, gamma
// of a scattering ray from it (tri_hit_params: the traversal's own
// operations, bit-identical).  The 16-B hit records cost the extend 2.4x their
// bytes in partly written L2 lines; C2 wavefront +3.7% (12.70 -> 13.18, three
// rounds), C4 +2.8%.  (capi.cpp wf_layout sizes the queues for this.)

#if !MCPT_WF_PRIMARY_TU
// ---- generate: primary rays of the batch (CUTracer.cu:186-211) -------------
// Paths go to segments in groups of 2^group_shift (64 = one 8x8 tile of one
// sample: a coherent wave of primary rays), group j -> segment j % nseg, so
// every segment holds tiles from all over the image and the workgroups
// finish together.
__global__ void __launch_bounds__(kGenBlock) wf_generate(const KernelParams kp, const WfParams wf) {
    const uint32_t n = wf.nb * wf.ns;
    const uint32_t gs = wf.group_shift, gm = (1u << gs) - 1u;
    const V3 eye = v3(kp.eye[0], kp.eye[1], kp.eye[2]);
    Counters c = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t pid = blockIdx.x * kGenBlock + threadIdx.x; pid < n; pid += gridDim.x * kGenBlock) {
        const uint32_t s_local = pid / wf.nb;
        const uint32_t v = wf.v0 + (pid - s_local * wf.nb);
        const uint32_t grp = pid >> gs, blk = grp / wf.nseg;
        const uint32_t g = seg_of(grp - blk * wf.nseg, blk, wf.nseg, wf.xcd_deal);
        const uint32_t slot = g * wf.seg + (blk << gs) + (pid & gm);
        if (grp < wf.nseg && (pid & gm) == 0u) wf.cnt[g].queued = seg_queue0_len(wf, g);   // segment g's queue length
        int px, py;
        V3 d = v3(0, 0, 0);
        uint32_t depth = kNoRay;
        V3 o = eye;
        if (unit_pixel(kp, v, px, py)) {
            uint32_t sd;
            const uint32_t pix = (uint32_t)py * (uint32_t)kp.width + (uint32_t)px;
            if (kp.mode == kModeQE)
                primary_ray_qe(kp, pix, px, py, wf.s_begin + s_local, sd, o, d);
            else
                primary_ray(kp, pix, px, py, wf.s_begin + s_local, sd, d);
            if (!implicit0(kp, wf))
                stq(&wf.q[0][qf(slot, kQPS, wf.slot_stride)], make_float4(1.0f, 1.0f, 1.0f, __uint_as_float(sd)));
            c.paths++;
            c.rays++;
            depth = 0;
        }
        if (!(MCPT_WF_IMPLICIT0 >= 2 && implicit0(kp, wf))) stq(&wf.q[0][qf(slot, kQO, wf.slot_stride)], pack(o, pid));
        stq(&wf.q[0][qf(slot, kQD, wf.slot_stride)], pack(d, depth));
    }
    flush_counters(c, kp.stats);
}

#endif  // !MCPT_WF_PRIMARY_TU

// Issue priority of the extend's traversal bursts (its hand-off runs one
// higher); the co-resident shade runs at 0.
#ifndef MCPT_WF_EXT_PRIO
#define MCPT_WF_EXT_PRIO 0
#endif

// Descent steps per traversal call in the wavefront extend (the megakernel's
// MCPT_DESCENT_CAP is 4): with shading out of the loop a longer descent burst
// pays (C2 wf cap 3 / 4 / 5 / 6: 13.57 / 13.64 / 13.84 / 13.57 G rays/s)
#ifndef MCPT_WF_DESCENT_CAP
#define MCPT_WF_DESCENT_CAP 5
#endif
// Global-memory scenes: 6 since round 6's cheaper descent step (C4 cap
// 4 / 5 / 6 / 7: 10.84 / 11.19 / 11.40 / 11.06 and 10.86 / 11.14 / 11.30 /
// 11.05 G rays/s, PERFLOG row 164); the megakernel keeps MCPT_DESCENT_CAP_GLOBAL
#ifndef MCPT_WF_DESCENT_CAP_GLOBAL
#define MCPT_WF_DESCENT_CAP_GLOBAL 6
#endif
constexpr int kWfLdsCap = MCPT_WF_DESCENT_CAP;

// Residency of the global-memory extend (C4: a walk bound by the latency of
// node and triangle reads from L2 / MALL, so every resident wave counts).
// Workgroups of 256 threads, kGlobalBlocksPerCu per CU per launch; other
// streams' extends fill further slots as far as LDS and VGPRs allow.
// MCPT_WF_GLOBAL_S: LDS stack entries per lane; MCPT_WF_GLOBAL_WAVES: waves per
// SIMD the compiler must allow (its VGPR budget; the lean kernel only -- the
// untimed counting kernels keep their registers) -- with 256-thread
// workgroups (one wave per SIMD each) that is the resident workgroups per CU.
// 6 x 6: 80 VGPRs (no scratch) and 6 x 24 KB of LDS, six extend waves per
// SIMD.  C4 G rays/s:
// S = 8, no hint (round 3: 32 KB, four workgroups, 88 VGPRs) 9.46 / 9.47;
// S = 6 9.61 / 9.63; S = 7 (five workgroups) 9.85 / 9.87; S = 5 9.20; S = 4
// 8.78 (spills); S = 6 with six workgroups (80 VGPRs) 10.36 / 10.31.
#ifndef MCPT_WF_GLOBAL_S
#define MCPT_WF_GLOBAL_S 6
#endif
#ifndef MCPT_WF_GLOBAL_WAVES
#define MCPT_WF_GLOBAL_WAVES 6
#endif
static_assert(kGlobalBlock == 256, "MCPT_WF_GLOBAL_WAVES = workgroups per CU only for one wave per SIMD each");
#ifndef MCPT_WF_GLOBAL_PREFETCH
#define MCPT_WF_GLOBAL_PREFETCH 1
#endif
// register budgets (waves per SIMD the compiler plans for; 0 = none) of the
// LDS scenes' lean extend and of the queue-order shade, and the shade's
// workgroup beside an LDS extend workgroup (512: two waves per SIMD)
#ifndef MCPT_WF_LDS_WPE
#define MCPT_WF_LDS_WPE 0
#endif
#ifndef MCPT_WF_SHADE_WPE
#define MCPT_WF_SHADE_WPE 0
#endif
#ifndef MCPT_WF_SHADE_LDS_BLOCK
#define MCPT_WF_SHADE_LDS_BLOCK 512
#endif
#ifndef MCPT_WF_GEO_LDS
#define MCPT_WF_GEO_LDS 1
#endif
constexpr size_t kLdsPerCu = 160 * 1024;
constexpr int kLayGlobal = 0, kLayLds = 1;


#if !MCPT_WF_PRIMARY_TU
// ---- extend: closest hit of every ray of this workgroup's segment -----------
// COUNT = false (lean renders): the traversal counters are compiled out.
// LAY: kLayGlobal (scene image with child-box records in global memory) or
// kLayLds (the whole 8-B-node image copied into LDS; a hybrid with only the
// triangle records in L1/L2 and two 768-thread workgroups per CU measured
// -24%, round 4)
template <int LAY, int S, int BLOCK, bool COUNT>
__global__ void __launch_bounds__(BLOCK, (LAY == kLayGlobal && !COUNT && MCPT_WF_GLOBAL_WAVES)
                                             ? MCPT_WF_GLOBAL_WAVES
                                             : (LAY == kLayLds && !COUNT && MCPT_WF_LDS_WPE
                                                    ? MCPT_WF_LDS_WPE : 1))   // (waves per SIMD)
wf_extend(const KernelParams kp, const WfParams wf) {
    constexpr bool IN_LDS = LAY != kLayGlobal;            // node words in LDS
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t g = blockIdx.x;
    WfCounters* cn = wf.cnt + (size_t)wf.bounce * wf.nseg + g;
    const uint32_t count = g < wf.nseg ? cn->queued : 0u;
    if (count == 0) {
        if (g < wf.nseg && threadIdx.x == 0) cn->hits = 0;
        return;
    }
    const int tid = (int)threadIdx.x;
    const GpuScene& sc = kp.scene;
    // LDS: [stack S x BLOCK x 16 B | scene image (kLayLds) | slot counter]
    unsigned char* const lds_image = smem + (size_t)S * BLOCK * 16;
    uint32_t* const lslot = reinterpret_cast<uint32_t*>(lds_image + (IN_LDS ? sc.image_bytes : 0u));
    if (tid == 0) *lslot = 0;
    const float4* tris;
    const uint2* nodes;
    const uint32_t* leafs;
    if constexpr (IN_LDS) {
        const uint4* src = reinterpret_cast<const uint4*>(sc.image);
        uint4* dst = reinterpret_cast<uint4*>(lds_image);
        const uint32_t n16 = sc.image_bytes / 16u;
        for (uint32_t i = (uint32_t)tid; i < n16; i += BLOCK) dst[i] = src[i];
        tris = reinterpret_cast<const float4*>(lds_image + sc.off_tris);
        nodes = reinterpret_cast<const uint2*>(lds_image + sc.off_nodes) + 1;
        leafs = reinterpret_cast<const uint32_t*>(lds_image + sc.off_leafs);
    } else {
        tris = reinterpret_cast<const float4*>(sc.image + sc.off_tris);
        nodes = reinterpret_cast<const uint2*>(sc.image + sc.off_nodes) + 1;
        leafs = reinterpret_cast<const uint32_t*>(sc.image + sc.off_leafs);
    }
    const uint4* pairs = reinterpret_cast<const uint4*>(sc.image + sc.off_nodes);   // 48-B pair records (global variant)
    __syncthreads();
    uint4* st = reinterpret_cast<uint4*>(smem) + tid;
    uint4* spill = kp.spill + (blockIdx.x * BLOCK + (uint32_t)tid);
    const uint32_t spill_stride = kp.total_lanes;
    const size_t seg0 = (size_t)g * wf.seg;
    float4* qb = wf.q[wf.bounce & 1];                      // this bounce's queue
    const uint32_t qs = wf.slot_stride;

    Counters c = {0, 0, 0, 0, 0, 0, 0, 0};
#ifdef MCPT_PHASE_TIMING
    LaneUse lu = {0, 0, 0, 0, 0, 0};
#endif
    SlotCursor cur_chunk = {0, kChunk};
    RayState r;
    r.htri = -1;
    int mode = kDead;
    // PF: the next ray of every lane is loaded a whole burst ahead (no4/nd4);
    // without it (MCPT_WF_GLOBAL_PREFETCH = 0, global-memory scenes only) a
    // finished lane loads its next ray in the hand-off, 8 VGPRs fewer
    constexpr bool PF = LAY != kLayGlobal || MCPT_WF_GLOBAL_PREFETCH;
    uint32_t slot = cur_chunk.take(true, lslot), depth = 0;
    uint32_t nslot = PF ? cur_chunk.take(true, lslot) : 0u;
    float4 no4 = make_float4(0, 0, 0, 0), nd4 = make_float4(0, 0, 0, 0);
    auto start = [&](float4 o4, float4 d4) {
        // opaque copies: the loop below must not see its ray registers as
        // memory-loaded, or LLVM flushes vmcnt in the descent loop's preheader
        // (the loop holds the spill store) and waits for the next-ray prefetch
        r.o = v3(opaque(o4.x), opaque(o4.y), opaque(o4.z));
        r.d = v3(opaque(d4.x), opaque(d4.y), opaque(d4.z));
        depth = __float_as_uint(d4.w);
        // (no branch: an empty slot's walk is set up and dropped; begin_ray
        // leaves htri = -1, its miss)
        const bool live = begin_ray(r, sc, kp.best_init);
        mode = (depth != kNoRay && live) ? kTrav : kReady;
    };
#ifdef MCPT_PHASE_TIMING
    // stats[8] setup, [9] traversal bursts, [10] hand-offs, [11] burst iterations
    unsigned long long tm_setup = 0, tm_trav = 0, tm_hand = 0, tm_iters = 0, tm_hands = 0,
                       tm_t0 = __builtin_amdgcn_s_memtime();
#define WF_STAMP(acc) do { unsigned long long t1_ = __builtin_amdgcn_s_memtime(); acc += t1_ - tm_t0; tm_t0 = t1_; } while (0)
#else
#define WF_STAMP(acc) do {} while (0)
#endif
    // the refill threshold as an asm result: a kernel argument read in the
    // loop was a scalar load still counted at the loop's exit test, whose
    // lgkmcnt(0) then also waited for every LDS access in flight, each iteration
    int refill;
    asm volatile("s_mov_b32 %0, %1" : "=s"(refill) : "s"(wf.refill_thresh));
    // MCPT_WF_IMPLICIT0 >= 2: bounce 0's origins are the eye (CV mode), not read
    const bool eye0 = MCPT_WF_IMPLICIT0 >= 2 && wf.bounce == 0 && implicit0(kp, wf);
    const float4 eye4 = make_float4(kp.eye[0], kp.eye[1], kp.eye[2], 0.0f);
    auto ld_o = [&](uint32_t sl) { return eye0 ? eye4 : ldq(&qb[qf(seg0 + sl, kQO, qs)]); };
    if (slot < count) start(ld_o(slot), ldq(&qb[qf(seg0 + slot, kQD, qs)]));
    if (PF && nslot < count) { no4 = ld_o(nslot); nd4 = ldq(&qb[qf(seg0 + nslot, kQD, qs)]); }
    WF_STAMP(tm_setup);
    for (;;) {
        // ---- traversal burst until enough lanes are done ---------------------
        __builtin_amdgcn_s_setprio(MCPT_WF_EXT_PRIO);
        for (;;) {
#ifdef MCPT_PHASE_TIMING
            tm_iters++;
            {
                const uint64_t tv = __ballot(mode == kTrav);
                if ((threadIdx.x & 63u) == 0) { lu.burst_w += 1; lu.burst_l += (unsigned long long)__popcll(tv); }
            }
#endif
            MCPT_MARK(5);
            if (mode == kTrav) {
                if (trav_iter<S, !IN_LDS, COUNT, LAY == kLayLds, IN_LDS ? kWfLdsCap : MCPT_WF_DESCENT_CAP_GLOBAL>(r, tris, nodes, leafs, st, BLOCK, spill, spill_stride, c MCPT_LU_ARG,
                                                 pairs))
                    mode = kReady;
            }
            MCPT_MARK(6);
            const uint64_t trv = __ballot(mode == kTrav);
            const uint64_t rdy = __ballot(mode == kReady);
            if (!trv || (int)__popcll(rdy) >= refill) break;
        }
        WF_STAMP(tm_trav);
#ifdef MCPT_PHASE_TIMING
        tm_hands++;
#endif
        // ---- hand-off: hit id, next ray -----------------------------------
        MCPT_MARK(7);
        __builtin_amdgcn_s_setprio(MCPT_WF_EXT_PRIO + 1);   // as the megakernel's shading rounds: short phase, raised priority
        // Settle the prefetch (issued a whole burst ago) before any store of
        // this hand-off: gfx9's vmcnt also counts stores, so any later wait on
        // the prefetch registers would wait for the stores' acknowledgements.
        // The origin's .w (unused here) is settled too: it keeps its register
        // live across the burst -- a dead load destination is reused by the
        // loop, which must then wait for the load first (a vmcnt wait in every
        // burst's first iteration: C2 +0.9%, C4 +2.8% without it).
        if constexpr (PF) {
            no4 = make_float4(opaque(no4.x), opaque(no4.y), opaque(no4.z), opaque(no4.w));
            nd4 = make_float4(opaque(nd4.x), opaque(nd4.y), opaque(nd4.z), opaque(nd4.w));
        }
        const bool fin = mode == kReady;
        const uint32_t ns0 = PF ? 0u : cur_chunk.take(fin, lslot);   // (collective: every lane)
        const uint32_t fslot = slot;
        if (fin) {
            const int32_t hid = r.htri;
            // (the next ray set up unconditionally: no branch in the hand-off; a
            // lane past the segment's end runs on its stale prefetch, then dies)
            if constexpr (PF) {
                slot = nslot;
                start(no4, nd4);
            } else {
                slot = ns0;
                float4 o4 = make_float4(0, 0, 0, 0), d4 = make_float4(0, 0, 0, __uint_as_float(kNoRay));
                if (slot < count) { o4 = ld_o(slot); d4 = ldq(&qb[qf(seg0 + slot, kQD, qs)]); }
                start(o4, d4);
            }
            if (slot >= count) mode = kDead;
            // (r holds the next ray by now: the id saved before)
            reinterpret_cast<int32_t*>(qb + qf(0, kQHIT, qs))[seg0 + fslot] = hid;
        }
        // ---- prefetch the next ray of every lane that just started one -------
        if constexpr (PF) {
            const bool want = fin && mode != kDead;
            const uint32_t ns = cur_chunk.take(want, lslot);
            if (want) {
                nslot = ns;
                if (nslot < count) { no4 = ld_o(nslot); nd4 = ldq(&qb[qf(seg0 + nslot, kQD, qs)]); }
            }
        }
        WF_STAMP(tm_hand);
        MCPT_MARK(8);
        if (!__ballot(mode != kDead)) break;
    }
#ifdef MCPT_PHASE_TIMING
    if ((threadIdx.x & 63u) == 0) {
        atomicAdd(kp.stats + 8, tm_setup);
        atomicAdd(kp.stats + 9, tm_trav);
        atomicAdd(kp.stats + 10, tm_hand);
        atomicAdd(kp.stats + 11, tm_iters);
        atomicAdd(kp.stats + 12, tm_hands);
    }
    {
        unsigned long long* gl = reinterpret_cast<unsigned long long*>(&g_lane_use);
        const unsigned long long v[6] = {lu.desc_w, lu.desc_l, lu.tri_w, lu.tri_l, lu.burst_w, lu.burst_l};
        for (int i = 0; i < 6; i++) {
            unsigned long long x = v[i];
            for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
            if ((threadIdx.x & 63u) == 0) atomicAdd(gl + i, x);
        }
    }
#endif
    flush_counters(c, kp.stats);
    if (tid == 0) cn->hits = count;                        // every slot's hit id is written
}

#endif  // !MCPT_WF_PRIMARY_TU

// ---- extend of bounce 0, wave-coherent (CV mode, queue-order shade) ---------
// Primary rays share the eye as their origin, and generate deals them in
// 64-path groups -- one 8x8 tile of one sample -- so a wave takes one group
// and walks the KD tree ONCE for its 64 rays: the node is wave-uniform (read
// by one LDS broadcast), each lane keeps its own interval, hit and an active
// flag, and the wave enters a child if any lane's interval reaches it.  With
// a common origin every lane has the same near side at every split plane (an
// origin exactly on the plane leaves only lanes inside the plane needing both
// children, and their near child is the left one), so the wave's front-to-back
// order is each lane's own: a lane is active at exactly the nodes its own
// ordered walk (trav_iter) visits, with the same interval and best hit there,
// and it stops at the same pop.  Hits, visit and test counts are therefore
// those of the per-ray walk, bit for bit; only the schedule differs (one
// wave-uniform descent per node instead of 64 divergent ones).
// Stack: the per-ray walk's lazy LDS stack (S entries in LDS, older ones in
// the spill area) with a wave-uniform position; a lane's copy of an entry
// carries its interval, or tmax = NaN if the lane is not in that subtree.
#ifndef MCPT_WF_PACKET0
#define MCPT_WF_PACKET0 1
#endif
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

// MCPT_WF_GEN0 (default 1): no generate kernel before this extend -- each
// lane computes its slot's primary ray itself (the inverse dealing slot_pid
// and primary_ray, as bounce 0's shade already does), writes the segment's
// queue length and counts the paths; queue 0 holds no direction stream.
// Generate was the only kernel of a frame's start (0.9 ms of one rank's 33 ms
// share at N = 8) and moved 16 B per path through HBM twice.
#ifndef MCPT_WF_GEN0
#define MCPT_WF_GEN0 1
#endif
template <int S, int BLOCK, bool COUNT>
__global__ void __launch_bounds__(BLOCK, 1) wf_extend_primary(const KernelParams kp, const WfParams wf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t g = blockIdx.x;
    WfCounters* cn = wf.cnt + (size_t)wf.bounce * wf.nseg + g;
    uint32_t count = 0;
    if (g < wf.nseg) {
        if constexpr (MCPT_WF_GEN0) {
            count = seg_queue0_len(wf, g);
            if (threadIdx.x == 0) cn->queued = count;          // (read by bounce 0's shade)
        } else {
            count = cn->queued;
        }
    }
    if (count == 0) {
        if (g < wf.nseg && threadIdx.x == 0) cn->hits = 0;
        return;
    }
    const int tid = (int)threadIdx.x;
    const int lane = tid & 63;
    const GpuScene& sc = kp.scene;
    // LDS: [stack S x BLOCK x 16 B | scene image | group counter]
    unsigned char* const lds_image = smem + (size_t)S * BLOCK * 16;
    uint32_t* lgrp = reinterpret_cast<uint32_t*>(lds_image + sc.image_bytes);
    if (tid == 0) *lgrp = 0;
    {
        const uint4* src = reinterpret_cast<const uint4*>(sc.image);
        uint4* dst = reinterpret_cast<uint4*>(lds_image);
        const uint32_t n16 = sc.image_bytes / 16u;
        for (uint32_t i = (uint32_t)tid; i < n16; i += BLOCK) dst[i] = src[i];
    }
    const float4* tris = reinterpret_cast<const float4*>(lds_image + sc.off_tris);
    const uint2* nodes = reinterpret_cast<const uint2*>(lds_image + sc.off_nodes) + 1;
    const uint32_t* leafs = reinterpret_cast<const uint32_t*>(lds_image + sc.off_leafs);
    __syncthreads();
    uint4* st = reinterpret_cast<uint4*>(smem) + tid;
    uint4* spill = kp.spill + (blockIdx.x * BLOCK + (uint32_t)tid);
    const uint32_t spill_stride = kp.total_lanes;
    const size_t seg0 = (size_t)g * wf.seg;
    float4* qb = wf.q[0];
    const uint32_t qs = wf.slot_stride;
    const int32_t U = BLOCK * 16;                      // one stack position (see slot_of)
    const V3 eye = v3(kp.eye[0], kp.eye[1], kp.eye[2]);
    Counters c = {0, 0, 0, 0, 0, 0, 0, 0};
    __builtin_amdgcn_s_setprio(MCPT_WF_EXT_PRIO);
    // a wave's 64-slot groups: the next group is taken, and its directions
    // loaded, before this one's walk, so the load's latency hides behind it
    auto take_group = [&]() {
        uint32_t grp = 0;
        if (lane == 0) grp = atomicAdd(lgrp, 1u);
        return lane_bcast(grp, 0) << 6;
    };
    // The hits of a group are stored one group later, after the wait for the
    // next directions: a store issued at the end of the walk would make that
    // wait (vmcnt counts stores too) wait for its acknowledgement.
    int32_t* const hq = reinterpret_cast<int32_t*>(qb + qf(0, kQHIT, qs)) + seg0;
    // the primary ray of local slot j: direction and depth (kNoRay: a pixel
    // outside the image, an empty slot)
    auto dir_of = [&](uint32_t j) {
        if constexpr (MCPT_WF_GEN0) {
            const uint32_t pid = slot_pid(wf, g, j);
            const uint32_t s_local = pid / wf.nb;
            int px, py;
            float4 d4 = make_float4(0, 0, 0, __uint_as_float(kNoRay));
            if (unit_pixel(kp, wf.v0 + (pid - s_local * wf.nb), px, py)) {
                uint32_t sd;
                V3 d;
                primary_ray(kp, (uint32_t)py * (uint32_t)kp.width + (uint32_t)px, px, py, wf.s_begin + s_local, sd, d);
                d4 = pack(d, 0u);
                c.paths++;                                      // (generate's counts)
                c.rays++;
            }
            return d4;
        } else {
            return ldq(&qb[qf(seg0 + j, kQD, qs)]);
        }
    };
    uint32_t base = take_group();
    float4 nd4 = make_float4(0, 0, 0, 0);
    if (base + (uint32_t)lane < count) nd4 = dir_of(base + (uint32_t)lane);
    uint32_t pslot = count;                             // the previous group's slot (count: none)
    int32_t phit = -1;
    for (;;) {
        if (base >= count) break;
        const uint32_t slot = base + (uint32_t)lane;
        const float4 d4 = make_float4(opaque(nd4.x), opaque(nd4.y), opaque(nd4.z), opaque(nd4.w));
        if (pslot < count) hq[pslot] = phit;
        const uint32_t nbase = take_group();
        if (nbase + (uint32_t)lane < count) nd4 = dir_of(nbase + (uint32_t)lane);
        RayState r;
        r.o = eye;
        r.d = v3(0, 0, 1);
        r.htri = -1;
        bool active = false, done = false;
        if (slot < count && __float_as_uint(d4.w) != kNoRay) {
            r.d = xyz(d4);
            active = begin_ray(r, sc, kp.best_init);
        }
        uint32_t w0 = sc.root_w[0], w1 = sc.root_w[1];  // the wave's node
        int32_t sp = 0, lo = 0;                         // wave-uniform stack positions
        if (__ballot(active)) {
            for (;;) {
                if ((w0 >> 30) != 3u) {
                    // ---- inner node: each lane's step of isect_kd_ordered ----
                    if constexpr (COUNT) c.inner += active ? 1u : 0u;
                    const uint32_t left = w0 & kLeftMask;
                    const uint4 pr = *reinterpret_cast<const uint4*>(nodes + left);
                    const int a = (int)(w0 >> 30);
                    const float sv = __uint_as_float(w1);
                    const float oa = sel3(a, eye.x, eye.y, eye.z);   // wave-uniform (common origin)
                    const float ia = sel3(a, r.ix, r.iy, r.iz);
                    const float t = (sv - oa) * ia;
                    const float te = t * kEpsHi;
                    const bool no = !(t > 0.0f) | (t > r.tmax);
                    const bool fo = te < r.tmin;
                    bool first_left, need1, need2;
                    float lo1, hi1, lo2, hi2;
                    if (__builtin_expect(oa != sv, 1)) {
                        // (a uniform branch) the origin is off the plane: every lane's
                        // near side is the wave's first child, below == first_left,
                        // and no lane lies in the plane (pp false)
                        first_left = oa < sv;
                        const bool go_far = !no & fo, both = !no & !fo;
                        need1 = active & !go_far;
                        need2 = active & (go_far | both);
                        // (both interval ends computed unconditionally: a select of the
                        // asm min/max, not a branch around it)
                        const float mn = min_qnan(te, r.tmax), mx = max_qnan(t, r.tmin);
                        lo1 = r.tmin;
                        hi1 = both ? mn : r.tmax;
                        lo2 = go_far ? r.tmin : mx;
                        hi2 = r.tmax;
                    } else {
                        // the origin on the plane: the near side by each lane's direction
                        const float da = sel3(a, r.d.x, r.d.y, r.d.z);
                        const bool below = da <= 0.0f, pp = da == 0.0f;
                        const bool go_far = !pp & !no & fo;
                        const bool push_it = pp | (!pp & !no & !fo);
                        const bool need_near = active & !go_far, need_far = active & (go_far | push_it);
                        const float near_max = push_it ? min_qnan(te, r.tmax) : r.tmax;   // near: [tmin, near_max]
                        const float far_min = go_far ? r.tmin : max_qnan(t, r.tmin);      // far: [far_min, tmax]
                        // the wave's order: left first (the near side of every lane not in the plane)
                        first_left = true;
                        need1 = below ? need_near : need_far;
                        need2 = below ? need_far : need_near;
                        lo1 = below ? r.tmin : far_min;
                        hi1 = below ? near_max : r.tmax;
                        lo2 = below ? far_min : r.tmin;
                        hi2 = below ? r.tmax : near_max;
                    }
                    const uint32_t f0 = first_left ? pr.x : pr.z, f1 = first_left ? pr.y : pr.w;
                    const uint32_t s0 = first_left ? pr.z : pr.x, s1 = first_left ? pr.w : pr.y;
                    if (__ballot(need1)) {
                        if (__ballot(need2)) {                   // push the second child
                            lds_uint4* sl = slot_of<S>(st, BLOCK, sp);
                            if (sp - lo == S * U) {              // LDS part full: its oldest entry to memory
                                spill[((uint32_t)lo / (uint32_t)U) * spill_stride] = ld4(sl);
                                lo += U;
                                if constexpr (COUNT) c.spills++;
                            }
                            st4(sl, make_uint4(s0, s1, __float_as_uint(lo2),
                                               need2 ? __float_as_uint(hi2) : 0x7FC00001u));
                            sp += U;
                        }
                        w0 = f0;
                        w1 = f1;
                        active = need1;
                        r.tmin = lo1;
                        r.tmax = hi1;
                    } else {
                        w0 = s0;
                        w1 = s1;
                        active = need2;
                        r.tmin = lo2;
                        r.tmax = hi2;
                    }
                    continue;
                }
                // ---- leaf: the active lanes test its triangles, two per round ----
                {
                    const uint32_t lpos = w0 & 0x3FFFFFFFu, lend = lpos + w1;
                    if constexpr (COUNT) c.leaf += active ? 1u : 0u;
                    for (uint32_t i = lpos; i < lend; i += 2u) {
                        const bool two = lend - i >= 2u;
                        const uint32_t k0 = leafs[i], k1n = leafs[i + 1u];
                        const uint32_t k1 = two ? k1n : k0;
                        const float4 a0 = ld_tri<true>(tris + k0), a1 = ld_tri<true>(tris + k0 + 1);
                        const float4 a2 = ld_tri<true>(tris + k0 + 2), b0 = ld_tri<true>(tris + k1);
                        const float4 b1 = ld_tri<true>(tris + k1 + 1), b2 = ld_tri<true>(tris + k1 + 2);
                        if (active) {
                            test_tri_pair(r, a0, a1, a2, k0, b0, b1, b2, k1, two);
                            if constexpr (COUNT) {
                                c.refs += two ? 2u : 1u;
                                c.tests += two ? 2u : 1u;
                            }
                        }
                    }
                }
                // ---- pop until an entry with an active lane (or the stack is empty) ----
                bool more = false;
                while (sp > 0) {
                    sp -= U;
                    uint4 e;
                    if (sp < lo) {                               // LDS part empty: the entry is in memory
                        e = settle4(spill[((uint32_t)sp / (uint32_t)U) * spill_stride]);   // (wait here)
                        lo = sp;
                    } else {
                        e = ld4(slot_of<S>(st, BLOCK, sp));
                    }
                    w0 = uni(e.x);
                    w1 = uni(e.y);
                    const float emin = __uint_as_float(e.z), emax = __uint_as_float(e.w);
                    active = false;
                    if ((emax == emax) & !done) {                // this lane's own entry (pop_entry)
                        if (r.best <= emin * kEpsLo) {
                            done = true;                         // its walk ends here
                        } else {
                            active = true;
                            r.tmin = emin;
                            r.tmax = emax;
                        }
                    }
                    if (__ballot(active)) {
                        more = true;
                        break;
                    }
                }
                if (!more) break;
            }
        }
        pslot = slot;
        phit = r.htri;
        base = nbase;
    }
    if (pslot < count) hq[pslot] = phit;
    flush_counters(c, kp.stats);
    if (tid == 0) cn->hits = count;
}

#if !MCPT_WF_PRIMARY_TU
// ---- shade: one workgroup per segment, its queue in blocks of slots ---------
// Reads the segment's queue b as dense streams (o, d, hit, throughput/rng),
// finishes terminated paths (radiance by path id) and scatters the others; a
// continuing ray goes to the next free slot of the segment's queue b+1 (one
// LDS atomic per wave, 64 consecutive slots), so queue b+1 is dense.  Queue
// order is scheduling-dependent, but nothing reads it (state keyed by pid).
// SORTB (wf_sort = 1): the material sort, inside the workgroup --
// each block of BLOCK queue slots is first classified (terminate / diffuse /
// phong / fresnel: the slot's hit id, depth and material), then counting-sorted
// by class in LDS (ranks by ballot, one LDS atomic per class and wave), and
// lane j shades the block's j-th slot in class order, so a wave runs one
// material branch except at the (at most three) class boundaries of a block.
// The class is a scheduling key only: every slot runs the same code.
// (SORTB held at <= 80 VGPRs, the queue-order shade's count: two of its waves
// per SIMD beside the LDS extend's four)
template <int BLOCK, bool GEO_LDS, bool SORTB>
__global__ void __launch_bounds__(BLOCK, SORTB ? 6 : (MCPT_WF_SHADE_WPE ? MCPT_WF_SHADE_WPE : 1))
wf_shade_slots(const KernelParams kp, const WfParams wf) {
    const uint32_t g = blockIdx.x;
    if (g >= wf.nseg) return;
    __shared__ uint32_t lnext;
    __shared__ uint32_t lcls[SORTB ? 8 : 1];               // class counts, two sets (alternate blocks)
    __shared__ uint16_t lperm[SORTB ? BLOCK : 1];          // block position -> slot offset, in class order
    if (SORTB && threadIdx.x < 8) lcls[threadIdx.x] = 0;
    // the material table in LDS when it fits beside the co-resident extend
    // (GEO_LDS): its fields are read in the branches of the shading chain,
    // each a dependent round trip that LDS serves in a fraction of L2's time
    // (16-B aligned: it is filled through uint4 stores and read as whole records)
    extern __shared__ __attribute__((aligned(16))) GpuGeom lgeo[];
    const WfCounters* cn = wf.cnt + (size_t)wf.bounce * wf.nseg + g;
    WfCounters* nx = wf.cnt + (size_t)(wf.bounce + 1) * wf.nseg + g;
    const uint32_t total = cn->hits;                       // the slots extend b wrote a hit id for
    const GpuScene& sc = kp.scene;
    if (threadIdx.x == 0) lnext = 0;
    if constexpr (GEO_LDS) {
        const uint4* src = reinterpret_cast<const uint4*>(sc.image + sc.off_geoms);
        uint4* dst = reinterpret_cast<uint4*>(lgeo);
        for (uint32_t i = threadIdx.x; i < sc.n_geoms * 4u; i += BLOCK) dst[i] = src[i];
    }
    __syncthreads();
    const float4* tris = reinterpret_cast<const float4*>(sc.image + sc.off_tris);
    const GpuGeom* geoms = GEO_LDS ? lgeo : reinterpret_cast<const GpuGeom*>(sc.image + sc.off_geoms);
    const size_t seg0 = (size_t)g * wf.seg;
    const float4* qb = wf.q[wf.bounce & 1];
    float4* qb2 = wf.q[(wf.bounce + 1) & 1];
    const uint32_t qs = wf.slot_stride;
    const bool qe = kp.mode == kModeQE;
    const bool imp = wf.bounce == 0 && implicit0(kp, wf);
    const int lane = (int)(threadIdx.x & 63u);
    Counters c = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t par = 0;
    for (uint32_t base = 0; base < total; base += BLOCK) {      // block-uniform trip count
        uint32_t i = base + threadIdx.x;
        if constexpr (SORTB) {
            uint32_t k = 4u;                                    // past the queue's end: no entry
            if (i < total) {
                const size_t js = seg0 + i;
                const int32_t htri = reinterpret_cast<const int32_t*>(qb + qf(0, kQHIT, qs))[js];
                // (every ray of queue b is at depth b; an empty slot is a miss)
                const int32_t lim = qe ? 3 * kp.max_depth : kp.max_depth;
                k = kClassTerminate;
                if (htri >= 0 && wf.bounce < lim) {
                    const GpuGeom& gm = geoms[__float_as_uint(tris[htri + 1].w)];
                    if (!is_emitter(gm)) k = material_class(gm);
                }
            }
            uint32_t* const lc = lcls + 4u * par;
            const uint64_t m0 = __ballot(k == 0u), m1 = __ballot(k == 1u), m2 = __ballot(k == 2u),
                           m3 = __ballot(k == 3u);
            const uint64_t mk = k == 0u ? m0 : k == 1u ? m1 : k == 2u ? m2 : m3;
            const uint64_t ml = lane == 0 ? m0 : lane == 1 ? m1 : lane == 2 ? m2 : m3;
            uint32_t off = 0;
            if (lane < 4) off = atomicAdd(&lc[lane], (uint32_t)__popcll(ml));   // the wave's offset in class `lane`
            off = (uint32_t)__shfl((int)off, (int)(k & 3u));
            __syncthreads();
            // class order in the block: diffuse, phong, fresnel, terminate
            const uint32_t n1 = lc[1], n2 = lc[2], n3 = lc[3];
            const uint32_t cb = k == 1u ? 0u : k == 2u ? n1 : k == 3u ? n1 + n2 : n1 + n2 + n3;
            if (k < 4u) lperm[cb + off + (uint32_t)__popcll(mk & ((1ull << lane) - 1ull))] = (uint16_t)threadIdx.x;
            if (threadIdx.x < 4) lcls[4u * (par ^ 1u) + threadIdx.x] = 0;
            __syncthreads();
            const uint32_t nv = total - base < (uint32_t)BLOCK ? total - base : (uint32_t)BLOCK;
            if (threadIdx.x < nv) i = base + lperm[threadIdx.x];   // (others: i >= total, no slot)
            par ^= 1u;
        }
        bool cont = false;
        uint32_t pid = 0, depth = kNoRay, sd = 0;
        V3 o = v3(0, 0, 0), d = v3(0, 0, 0), color = v3(0, 0, 0);
        if (i < total) {
            const size_t js = seg0 + i;
            const int32_t htri = reinterpret_cast<const int32_t*>(qb + qf(0, kQHIT, qs))[js];
            float4 h = make_float4(0, 0, 0, 0);
            float4 o4, d4, ps;
            if (imp) {   // generate's primary ray, recomputed (a miss or an empty slot needs only pid)
                pid = slot_pid(wf, g, i);
                o4 = make_float4(kp.eye[0], kp.eye[1], kp.eye[2], __uint_as_float(pid));
                d4 = make_float4(0, 0, 0, 0);
                ps = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
                if (htri >= 0) {
                    const uint32_t s_local = pid / wf.nb;
                    int px, py;
                    (void)unit_pixel(kp, wf.v0 + (pid - s_local * wf.nb), px, py);
                    uint32_t sd0;
                    V3 d0;
                    primary_ray(kp, (uint32_t)py * (uint32_t)kp.width + (uint32_t)px, px, py, wf.s_begin + s_local,
                                sd0, d0);
                    d4 = pack(d0, 0u);
                    ps.w = __uint_as_float(sd0);
                }
            } else {
                o4 = ldq(&qb[qf(js, kQO, qs)]);
                d4 = ldq(&qb[qf(js, kQD, qs)]);
                ps = ldq(&qb[qf(js, kQPS, qs)]);
            }
            pid = __float_as_uint(o4.w);
            depth = __float_as_uint(d4.w);
            color = xyz(ps);
            sd = __float_as_uint(ps.w);
            // CV: miss -> 0; emitter -> color*Ka*ILLUM (:111-113); terminal query
            // (:162-175); else scatter.  QE: miss / bounce >= 3*depth -> 0; roulette
            // from bounce `depth` on; emitter -> color*Ka (rtx.hlsl:312-331)
            V3 L = v3(0, 0, 0);
            bool term = true;
            if (htri >= 0 && depth != kNoRay) {
                const GpuGeom& gm = geoms[__float_as_uint(tris[htri + 1].w)];
                if (qe) {
                    if ((int32_t)depth < 3 * kp.max_depth &&
                        ((int32_t)depth < kp.max_depth || qe_roulette(sd, color))) {
                        if (is_emitter(gm)) L = emitted(color, gm, 1.0f);
                        else term = false;
                    }
                } else if ((int32_t)depth >= kp.max_depth || is_emitter(gm)) {
                    L = emitted(color, gm, kp.illum);
                } else {
                    term = false;
                }
                if (!term) {
                    c.shades++;
                    o = xyz(o4);
                    d = xyz(d4);
                    tri_hit_params(o, d, tris[htri], tris[htri + 1], tris[htri + 2], h.x, h.y, h.z);
                    if (qe) scatter<true>(gm, sc.normals, htri, h.y, h.z, h.x, 0, sd, color, o, d);
                    else scatter<false>(gm, sc.normals, htri, h.y, h.z, h.x, kp.fresnel_kd, sd, color, o, d);
                    cont = true;
                    c.rays++;
                }
            }
            if (term) stq(&wf.radiance[pid], make_float4(L.x, L.y, L.z, 0.0f));   // (kNoRay slots: 0)
        }
        // next ray: the wave's continuing lanes take consecutive slots of queue b+1
        const uint64_t m = __ballot(cont);
        if (m) {
            const int leader = __ffsll((unsigned long long)m) - 1;
            uint32_t b0 = 0;
            if (lane == leader) b0 = atomicAdd(&lnext, (uint32_t)__popcll(m));
            b0 = lane_bcast(b0, leader);
            if (cont) {
                const size_t ji = seg0 + b0 + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                stq(&qb2[qf(ji, kQO, qs)], pack(o, pid));
                stq(&qb2[qf(ji, kQD, qs)], pack(d, depth + 1u));
                stq(&qb2[qf(ji, kQPS, qs)], pack(color, sd));
            }
        }
    }
    flush_counters(c, kp.stats);
    __syncthreads();
    if (threadIdx.x == 0) nx->queued = lnext;
}

// ---- accumulate: samples of the batch in sample order -> partial sums -------
// A batch holds wf.ns / wf.nsc whole chunks of nsc samples each (blockIdx.y).
__global__ void __launch_bounds__(256) wf_accumulate(const KernelParams kp, const WfParams wf) {
    const uint32_t u = blockIdx.x * 256u + threadIdx.x;
    if (u >= wf.nb) return;
    const uint32_t j = blockIdx.y;
    V3 part = v3(0, 0, 0);
    for (uint32_t s = j * wf.nsc; s < (j + 1u) * wf.nsc; s++)
        part = vadd(part, xyz(wf.radiance[(size_t)s * wf.nb + u]));
    kp.partial[(size_t)(wf.chunk_index + j) * kp.npix_local + wf.v0 + u] = make_float4(part.x, part.y, part.z, 0.0f);
}

#endif  // !MCPT_WF_PRIMARY_TU

template <int S, int BLOCK>
hipError_t launch_extend_primary(const KernelParams& kp, const WfParams& wf, int grid, size_t lds, hipStream_t st) {
    auto kern = kp.lean ? wf_extend_primary<S, BLOCK, false> : wf_extend_primary<S, BLOCK, true>;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), lds, st, kp, wf);
    return hipGetLastError();
}

#if !MCPT_WF_PRIMARY_TU
template <int BLOCK>
auto shade_kernel(bool geo_lds, bool sortb) {
    return sortb ? (geo_lds ? wf_shade_slots<BLOCK, true, true> : wf_shade_slots<BLOCK, false, true>)
                 : (geo_lds ? wf_shade_slots<BLOCK, true, false> : wf_shade_slots<BLOCK, false, false>);
}

template <int LAY, int S, int BLOCK>
hipError_t launch_extend(const KernelParams& kp, const WfParams& wf, int grid, size_t lds, hipStream_t st) {
    auto kern = kp.lean ? wf_extend<LAY, S, BLOCK, false> : wf_extend<LAY, S, BLOCK, true>;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), lds, st, kp, wf);
    return hipGetLastError();
}

// the scene image (8-B node records) is copied into LDS; an image built with
// child-box pair records (node_boxes) is always read from global memory
bool wf_in_lds(const GpuScene& sc) { return !sc.node_boxes && lds_bytes_in_lds(sc.image_bytes, 4) + 32 <= kMaxLds; }

#endif  // !MCPT_WF_PRIMARY_TU
}  // namespace

#if MCPT_WF_PRIMARY_TU
// the bounce-0 packet extend's launch, called by launch_wavefront (the other
// translation unit)
hipError_t launch_wavefront_primary(const KernelParams& kp, const WfParams& wf, int grid, size_t lds,
                                    hipStream_t st) {
    return launch_extend_primary<4, kLdsBlock>(kp, wf, grid, lds, st);
}
#else
hipError_t launch_wavefront_primary(const KernelParams& kp, const WfParams& wf, int grid, size_t lds,
                                    hipStream_t st);   // wavefront_primary.hip

#ifdef MCPT_PHASE_TIMING
void read_lane_use_wf(unsigned long long out[6]) {   // wavefront extend lane-use counters, then reset
    LaneUse z = {0, 0, 0, 0, 0, 0};
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lane_use), sizeof z);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_lane_use), &z, sizeof z);
}
#endif

int wavefront_segments(const GpuScene& sc, int cus) {
    return wf_in_lds(sc) ? cus : cus * kWfGlobalSegsPerCu;
}
// LDS bytes of an LDS-scene extend workgroup: stack + image (or its part from the nodes on) + counters
size_t wf_lds_extend_bytes(const GpuScene& sc) {
    return lds_bytes_in_lds(sc.image_bytes, 4) + 32;
}

hipError_t launch_wavefront(const KernelParams& kp_in, const WfParams* wf_in, const WfStreams& ws, int cus,
                            int max_bounces, hipEvent_t ev0, hipEvent_t ev1, hipEvent_t ev2, float4* fb,
                            int* variant_out) {
    KernelParams kp = kp_in;
    const uint32_t img = kp.scene.image_bytes;
    const bool in_lds = wf_in_lds(kp.scene);
    kp.total_lanes = (uint32_t)total_lanes_for(img, cus);
    const uint32_t nseg = (uint32_t)wavefront_segments(kp.scene, cus);
    // Several streams (ws.n > 1): batch i runs on stream i mod n, each stream
    // with its own queues/counters (wf_in[i]) and stack spill area, so one
    // batch's shade and the tail of its extend overlap another batch's extend.
    // The shade then runs in workgroups that fit on a CU beside the extend's 16
    // waves (extend <= 88 VGPRs per lane, so 160 of the SIMD's 512 are left:
    // two <= 80-VGPR shade waves; 4 B of LDS): 512 threads for LDS scenes (one
    // 1024-thread extend workgroup with 157 KB of LDS per CU), 256 for global
    // scenes (four 256-thread extend workgroups), so shading fills the
    // extend's idle issue slots instead of waiting for it (C2 wavefront 10.10
    // -> 13.20, C4 at 1024 spp 6.14 -> 8.34 G rays/s).
    const int ns = ws.n < 1 ? 1 : (ws.n > kMaxWfStreams ? kMaxWfStreams : ws.n);
    const hipStream_t st = ws.st[0];
    hipError_t e = hipSuccess;
    if (ev0 && (e = hipEventRecord(ev0, st)) != hipSuccess) return e;
    if (ns > 1) {
        if ((e = hipEventRecord(ws.fork, st)) != hipSuccess) return e;
        for (int i = 1; i < ns; i++)
            if ((e = hipStreamWaitEvent(ws.st[i], ws.fork, 0)) != hipSuccess) return e;
    }
    // Every launch error leaves the batch loops and still joins every forked
    // stream back into the caller's stream below, so no side stream keeps
    // writing the shared partial sums or spill areas behind a failed call.
    uint32_t batch = 0;
    for (uint32_t chunk = 0; chunk < kp.nchunks && e == hipSuccess;) {
        // whole-image batches may span several full chunks (fewer, longer launches)
        const uint32_t nsc = (kp.spp - chunk * kp.chunk) < kp.chunk ? (kp.spp - chunk * kp.chunk) : kp.chunk;
        uint32_t ncb = 1;
        if (nsc == kp.chunk && (uint64_t)kp.npix_local * kp.chunk <= wf_in[0].capacity) {
            const uint32_t full = (kp.spp / kp.chunk) - chunk;             // full chunks left
            const uint32_t fit = (uint32_t)(wf_in[0].capacity / ((uint64_t)kp.npix_local * kp.chunk));
            ncb = fit < full ? fit : full;
        }
        const uint32_t chunk0 = chunk;
        chunk += ncb;
        const uint32_t nb_max = wf_in[0].capacity / (ncb * nsc);
        for (uint32_t v0 = 0; v0 < kp.npix_local && e == hipSuccess; v0 += nb_max, ++batch) {
            const int h = (int)(batch % (uint32_t)ns);
            const hipStream_t bs = ws.st[h];
            KernelParams kb = kp;
            kb.spill = kp.spill + (size_t)h * 32 * kp.total_lanes;       // this stream's spill area
            WfParams wf = wf_in[h];
            wf.nseg = nseg;
            wf.chunk_index = chunk0;
            wf.s_begin = chunk0 * kp.chunk;
            wf.nsc = nsc;
            wf.ns = ncb * nsc;
            wf.v0 = v0;
            wf.nb = (kp.npix_local - v0) < nb_max ? (kp.npix_local - v0) : nb_max;
            const uint32_t n = wf.nb * wf.ns;
            // the shade's material table in LDS if it fits beside the extend's
            // workgroups on a CU (MCPT_WF_GEO_LDS)
            const size_t ext_lds = in_lds ? wf_lds_extend_bytes(kp.scene)
                                          : (size_t)kWfGlobalSegsPerCu * (MCPT_WF_GLOBAL_S * kGlobalBlock * 16 + 32);
            const size_t geo_bytes = (MCPT_WF_GEO_LDS && ext_lds + 64 * (size_t)kp.scene.n_geoms + 64 <= kLdsPerCu)
                                         ? 64 * (size_t)kp.scene.n_geoms : 0;
            // LDS scenes: one 8x8 tile of one sample per group; global-memory
            // scenes: the planned group size (whole image regions per segment)
            wf.group_shift = in_lds ? 6u : wf_in[h].group_shift;
            wf.xcd_deal = in_lds ? 0u : 1u;                                // (seg_of)
            // whole groups per segment
            wf.seg = ((((n + (1u << wf.group_shift) - 1u) >> wf.group_shift) + nseg - 1) / nseg) << wf.group_shift;
            e = hipMemsetAsync(wf.cnt, 0, sizeof(WfCounters) * (size_t)nseg * (size_t)(max_bounces + 1), bs);
            if (e != hipSuccess) break;
            // bounce 0 of CV mode (implicit queue 0: every origin is the eye): the
            // wave-coherent extend, one tree walk per 64-ray tile (MCPT_WF_PACKET0),
            // which also generates the primary rays (MCPT_WF_GEN0)
            // (the packet extend stores hit ids only: it needs the queue-order shade)
            const bool packet = MCPT_WF_PACKET0 && in_lds && MCPT_WF_IMPLICIT0 >= 2 &&
                                implicit0(kb, wf) && wf.group_shift == 6u;
            if (!(packet && MCPT_WF_GEN0)) {
                const uint32_t gen_grid = (n + kGenBlock - 1) / kGenBlock;
                hipLaunchKernelGGL(wf_generate, dim3(gen_grid < 16u * (uint32_t)cus ? gen_grid : 16u * (uint32_t)cus),
                                   dim3(kGenBlock), 0, bs, kb, wf);
                if ((e = hipGetLastError()) != hipSuccess) break;
            }
            for (int b = 0; b < max_bounces && e == hipSuccess; b++) {
                wf.bounce = b;
                const size_t llds = in_lds ? wf_lds_extend_bytes(kb.scene) : 0;
                if (packet && b == 0) {
                    e = launch_wavefront_primary(kb, wf, (int)nseg, llds, bs);
                } else if (in_lds) {
                    e = launch_extend<kLayLds, 4, kLdsBlock>(kb, wf, (int)nseg, llds, bs);
                } else
                    e = launch_extend<kLayGlobal, MCPT_WF_GLOBAL_S, kGlobalBlock>(kb, wf, (int)nseg,
                                                                            (size_t)MCPT_WF_GLOBAL_S * kGlobalBlock * 16 + 32,
                                                              bs);
                if (e != hipSuccess) break;
                const bool sortb = wf.sort != 0;
                if (in_lds && ns == 1)   // alone on the GPU: 16 waves per segment keep HBM busy
                    hipLaunchKernelGGL(shade_kernel<1024>(geo_bytes != 0, sortb), dim3(nseg), dim3(1024), geo_bytes, bs, kb, wf);
                else if (in_lds)              // beside an extend workgroup: 8 waves (2 x 80 VGPRs per SIMD)
                    hipLaunchKernelGGL(shade_kernel<MCPT_WF_SHADE_LDS_BLOCK>(geo_bytes != 0, sortb), dim3(nseg),
                                       dim3(MCPT_WF_SHADE_LDS_BLOCK), geo_bytes, bs, kb, wf);
                else
                    hipLaunchKernelGGL(shade_kernel<256>(geo_bytes != 0, sortb), dim3(nseg), dim3(256), geo_bytes, bs, kb, wf);
                e = hipGetLastError();
            }
            if (e != hipSuccess) break;
            hipLaunchKernelGGL(wf_accumulate, dim3((wf.nb + 255u) / 256u, ncb), dim3(256), 0, bs, kb, wf);
            e = hipGetLastError();
        }
    }
    for (int i = 1; i < ns; i++) {   // join (also after an error)
        hipError_t j = hipEventRecord(ws.join[i], ws.st[i]);
        if (j == hipSuccess) j = hipStreamWaitEvent(st, ws.join[i], 0);
        if (e == hipSuccess) e = j;
    }
    if (e != hipSuccess) return e;
    if (ev1 && (e = hipEventRecord(ev1, st)) != hipSuccess) return e;
    e = launch_reduce(kp, fb, st);
    if (e == hipSuccess && ev2) e = hipEventRecord(ev2, st);
    if (variant_out) *variant_out = in_lds ? 4 : 5;
    return e;
}
#endif  // MCPT_WF_PRIMARY_TU

}  // namespace mcpt
