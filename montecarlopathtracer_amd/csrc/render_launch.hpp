// render_launch.hpp -- device scene image layout and kernel parameters.
//
// Scene image (one contiguous device buffer, 16-byte aligned sections; the
// same bytes are copied verbatim into LDS by the in-LDS kernel variant):
//   tris   3 x float4 per KD triangle: (a.xyz, brute-force rank bits),
//          (a-b .xyz, geometry index bits), (a-c .xyz, the ray-independent
//          minor (a-b).y (a-c).z - (a-c).y (a-b).z of det A and det tM)   48 B
//   nodes  uint2 per KD node (BFS), stored one slot late so that every
//          sibling pair (left, left+1; left is odd in BFS order) is one aligned
//          16-B record: inner x = axis<<30 | left child, y = split value bits;
//          leaf x = 3<<30 | first leaf ref, y = count                       8 B
//   leafs  uint32 per leaf reference: the float4 index (3 x slot) of its
//          triangle's record -- also the index of its normals, and the ray's
//          hit id (no multiply on the hot path)                           4 B
//   (scenes too large for LDS: nodes are 48-B sibling-pair records instead,
//          the two node words + both children's KD boxes as 6 x fp16
//          rounded outward; the root's record is GpuScene::root_w)        48 B
//   geoms  GpuGeom per geometry (material of CUTracer.cu:300-308)      64 B
// Shading normals live outside the image (read once per shaded hit):
//   normals 3 x float4 per KD triangle (n0, n1, n2)                    48 B
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mcpt {

constexpr int kLdsBlock = 1024;          // in-LDS variant: one 16-wave workgroup per CU
constexpr int kGlobalBlock = 256;        // global variant
constexpr int kGlobalBlocksPerCu = 4;
// the wavefront extend's segments (workgroups) per CU for global-memory scenes
#ifndef MCPT_WF_GLOBAL_SEGS
#define MCPT_WF_GLOBAL_SEGS 4
#endif
constexpr int kWfGlobalSegsPerCu = MCPT_WF_GLOBAL_SEGS;
constexpr size_t kMaxLds = 160 * 1024;   // gfx950 LDS per CU

struct GpuGeom {
    float Ka[3], Kd[3], Ks[3];
    float Ns, Tr, Ni;
    uint32_t Ns_u;                       // (PWuint)Ns, Utils.hpp:72 parameter type
    uint32_t pad[3];
};
static_assert(sizeof(GpuGeom) == 64, "GpuGeom layout");

struct GpuScene {
    const unsigned char* image;
    const float4* normals;
    uint32_t image_bytes;
    uint32_t off_tris, off_nodes, off_leafs, off_geoms;
    uint32_t node_boxes;                 // 1: 48-B pair records with child boxes (global-memory scenes)
    uint32_t n_tris, n_nodes, n_leafs, n_geoms;
    float root_min[3], root_max[3];
    uint32_t root_w[2];                  // root node record (nodes[0])
};

// Unsigned division by a launch-invariant divisor d >= 1 as multiply-high and
// shifts (Granlund & Montgomery 1994, fig. 4.1): exact for every 32-bit n.
// The work-unit decode divides four times per unit; hardware has no integer
// divide, and the generic sequence cost ~5% of C2 at 8-sample chunks.
struct FastDiv {
    uint32_t m, s1, s2, d;
    static FastDiv make(uint32_t d) {
        uint32_t l = 0;
        while (l < 32 && (uint64_t(1) << l) < d) l++;          // ceil(log2 d)
        FastDiv f;
        f.m = static_cast<uint32_t>(((uint64_t(1) << 32) * ((uint64_t(1) << l) - d)) / d + 1);
        f.s1 = l < 1 ? l : 1;
        f.s2 = l > 0 ? l - 1 : 0;
        f.d = d;
        return f;
    }
    __host__ __device__ __forceinline__ uint32_t div(uint32_t n) const {
        const uint32_t t = static_cast<uint32_t>((uint64_t(m) * n) >> 32);   // v_mul_hi_u32
        return (t + ((n - t) >> s1)) >> s2;
    }
};

struct KernelParams {
    GpuScene scene;
    int32_t width, height;
    int32_t tile, tiles_x, shard_count, shard_index, packed;
    uint32_t npix_local;                 // owned tiles * tile^2
    uint32_t spp, spp_offset, chunk, nchunks, total_units;
    int32_t max_depth;
    float illum, tan_half_fov;
    int32_t fresnel_kd;
    uint32_t prev_count;
    int32_t mode;                        // 0 CVMCTracer, 1 QuinEngine (rtx.hlsl:304-405)
    float proj11, proj22;                // QE projection scales (PerspectiveFovRH)
    float best_init;                     // closest-hit start: FLT_MAX, QE 10000 (rtx.hlsl:88)
    float eye[3], fwd[3], up[3], right[3];
    uint32_t key;                        // TEA-16 key of the 64-bit seed
    float4* partial;                     // [nchunks][npix_local]
    uint32_t* counter;                   // work-unit counter
    unsigned long long* stats;           // 8 counters
    uint4* spill;                        // traversal-stack spill [32][total_lanes]
    uint32_t total_lanes;
    uint32_t* unit_counters;             // optional [total_units][4]: rays, inner, leaf, tests
    int32_t ready_thresh;                // lanes ready before a shading round (1..64)
    int32_t lean;                        // 1: no per-step traversal counters (mcpt_render_params::lean)
    FastDiv div_npix, div_tt, div_tiles_x, div_tile;   // npix_local, tile^2, tiles_x, tile
    // Tail split (megakernel): units [tail_units, total_units) -- the last
    // ~6 per lane -- are handed out one sample at a time (work items
    // tail_units + (u - tail_units) * chunk + j), each sample's radiance going
    // to tail_buf[(u - tail_units) * chunk + j]; the reduction sums them in
    // sample order, so the image is the one of whole units, bit for bit.
    uint32_t tail_units, total_items;
    FastDiv div_chunk;                   // chunk
    float4* tail_buf;
    // primary rays (CUTracer.cu:202-203, double): H / W, and 2^-k when W = 2^k (else 0)
    double h_over_w, inv_w_pow2;
    // 1: the reduction writes the plain mean of this call's samples (a device's
    // shard of a multi-device render; gather_kernel applies the running mean)
    int32_t raw_mean;
};

// Multi-device gather (capi.cpp render_multi): shard r of `nshards` wrote the
// plain means of its owned tiles, packed tile-major, to src[r * slot ...]
// (peer-copied to the primary device); gather_kernel unpermutes them into the
// row-major framebuffer with the running mean of reduce_kernel, bit for bit.
struct GatherParams {
    const float4* src;                   // [nshards][slot]
    float4* fb;                          // row-major W x H
    uint32_t slot;                       // packed pixels per shard slot (>= every shard's count)
    int32_t width, height, tile, tiles_x, nshards;
    uint32_t prev_count;
    int32_t mode;
};

// Closest-hit batch (mcpt_intersect, render.hip query_kernel): rays i < n,
// origins / directions as 3 floats each; out slot[i] = the hit triangle's image
// slot (-1 miss), hit[3i..] = beta, gamma, t; spill = [32][n] stack entries
constexpr int kQueryBlock = 256;
struct QueryParams {
    GpuScene scene;
    const float* o;
    const float* d;
    int32_t* slot;
    float* hit;
    uint4* spill;
    unsigned long long* stats;           // 8 counters (Counters order)
    uint32_t n;
    float best_init;
};

// Wavefront pipeline workspace (wavefront.hip).  One batch = samples
// [s_begin, s_begin + ns) of chunk `chunk` for owned pixels [v0, v0 + nb);
// path id pid = s_local * nb + (v - v0).  The batch is cut into `nseg`
// segments of `seg` paths, one per extend workgroup; a path stays in its
// segment for all bounces, so each segment's queues and counters are private
// to one workgroup (LDS atomics only).  Queue slot j of
// segment g is entry g*seg + j; path state and radiance are indexed by pid.
struct WfCounters {                      // per (bounce, segment), 8 words
    uint32_t queued;                     // rays in this segment's queue (written by its producer)
    uint32_t hits;                       // slots whose hit id extend wrote (= queued; shade's count)
    uint32_t pad[6];
};
struct WfParams {
    // ray queue b: three float4 streams of slot_stride entries (SoA),
    // {o.xyz pid} {d.xyz depth} {throughput.xyz rng}, then the 4-B hit ids;
    // extend reads streams 0-1 and writes the ids, shade reads all four
    float4* q[2];
    float4* radiance;                    // path radiance per pid                   [capacity]
    WfCounters* cnt;                     // [max_depth + 2][nseg]
    uint32_t capacity;                   // paths per batch
    uint32_t slot_stride;                // queue entries per stream (>= nseg * seg)
    uint32_t v0, nb, s_begin, ns, chunk_index;   // pixels [v0, v0+nb) x samples [s_begin, s_begin+ns)
    uint32_t nsc;                        // samples per chunk (ns = whole chunks of nsc)
    uint32_t nseg, seg;                  // segments (= extend workgroups) and slots per segment
    uint32_t group_shift;                // paths are dealt to segments in groups of 2^group_shift
                                         // (the plan's for global-memory scenes; 6 in LDS)
    int32_t bounce;
    int32_t refill_thresh;               // idle lanes before an extend wave refills
    int32_t sort;                        // 1: shade sorts each block of slots by material first
    uint32_t xcd_deal;                   // 1: groups dealt to segments by XCD (global-memory scenes, seg_of)
};

size_t lds_bytes_in_lds(uint32_t image_bytes, int S);
int total_lanes_for(uint32_t image_bytes, int cus);
// memset counter, path kernel (events ev0/ev1 around it), reduce kernel (ev2)
hipError_t launch_render(const KernelParams& kp, int cus, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1,
                         hipEvent_t ev2, float4* fb, int* variant_out);
hipError_t launch_reduce(const KernelParams& kp, float4* fb, hipStream_t st);
hipError_t launch_gather(const GatherParams& g, hipStream_t st);
hipError_t launch_query(const QueryParams& q, hipStream_t st);
#ifdef MCPT_PHASE_TIMING
void read_lane_use(unsigned long long out[6]);      // diagnostic build only: megakernel
void read_lane_use_wf(unsigned long long out[6]);   // wavefront extend
#endif
// wavefront queue segments (= extend workgroups) for a scene image
int wavefront_segments(const GpuScene& sc, int cus);
// wavefront pipeline: generate / extend / shade per bounce / accumulate per
// batch, then the same reduction (events: ev0 before, ev1 after the batches)
// wavefront streams: batch i runs on stream i mod n (st[0] = the caller's),
// forked from and joined back into st[0] with the events of each extra stream
constexpr int kMaxWfStreams = 4;
struct WfStreams {
    int n;
    hipStream_t st[kMaxWfStreams];
    hipEvent_t fork, join[kMaxWfStreams];
};
hipError_t launch_wavefront(const KernelParams& kp, const WfParams* wf, const WfStreams& ws, int cus,
                            int max_bounces, hipEvent_t ev0, hipEvent_t ev1, hipEvent_t ev2, float4* fb,
                            int* variant_out);

}  // namespace mcpt
