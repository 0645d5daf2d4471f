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

struct Hit {
    int32_t tri;
    float beta, gamma;
    V3 hp;
};

struct Counters {
    uint32_t rays, paths, inner, leaf, refs, tests, shades, spills;
};

__device__ __forceinline__ float sel3(int a, float x, float y, float z) {
    return a == 0 ? x : (a == 1 ? y : z);
}

// Ordered KD traversal; mirrors oracle/render_ref.c isect_kd_ordered().
template <int S>
__device__ __forceinline__ Hit trace(V3 o, V3 d, const GpuScene& sc, const float4* __restrict__ tris,
                                     const uint2* __restrict__ nodes, const uint32_t* __restrict__ leafs,
                                     uint32_t* st_node, float* st_lo, float* st_hi, int stride,
                                     uint4* __restrict__ spill, uint32_t spill_stride, Counters& c) {
    Hit h;
    h.tri = -1;
    h.beta = h.gamma = 0.0f;
    h.hp = v3(0.0f, 0.0f, 0.0f);
    const float ix = 1.0f / d.x, iy = 1.0f / d.y, iz = 1.0f / d.z;
    float tmin = 0.0f, tmax = kFltMax;
    {
        const float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z}, inv[3] = {ix, iy, iz};
#pragma unroll
        for (int a = 0; a < 3; a++) {
            if (dd[a] == 0.0f) {
                if (oo[a] < sc.root_min[a] || oo[a] > sc.root_max[a]) return h;
            } else {
                float t0 = (sc.root_min[a] - oo[a]) * inv[a];
                float t1 = (sc.root_max[a] - oo[a]) * inv[a];
                float lo = dd[a] < 0.0f ? t1 : t0;
                float hi = dd[a] < 0.0f ? t0 : t1;
                tmin = lo > tmin ? lo : tmin;
                tmax = hi < tmax ? hi : tmax;
            }
        }
    }
    if (tmin > tmax * kEpsHi) return h;

    float best = kFltMax;
    uint32_t bprio = 0xFFFFFFFFu;
    uint32_t node = 0;
    int sp = 0;

    auto push = [&](uint32_t n, float lo, float hi) {
        const int slot = (sp & (S - 1)) * stride;
        if (sp >= S) {
            spill[(uint32_t)(sp - S) * spill_stride] = make_uint4(st_node[slot], __float_as_uint(st_lo[slot]),
                                                                  __float_as_uint(st_hi[slot]), 0u);
            c.spills++;
        }
        st_node[slot] = n;
        st_lo[slot] = lo;
        st_hi[slot] = hi;
        sp++;
    };

    for (;;) {
        uint2 nd = nodes[node];
        while ((nd.x >> 30) != 3u) {
            c.inner++;
            const int a = (int)(nd.x >> 30);
            const float sv = __uint_as_float(nd.y);
            const uint32_t left = nd.x & 0x3FFFFFFFu;
            const float oa = sel3(a, o.x, o.y, o.z);
            const float da = sel3(a, d.x, d.y, d.z);
            const float ia = sel3(a, ix, iy, iz);
            const float t = (sv - oa) * ia;
            const bool below = (oa < sv) || (oa == sv && da <= 0.0f);
            const uint32_t nearc = below ? left : left + 1;
            const uint32_t farc = below ? left + 1 : left;
            if (da == 0.0f && oa == sv) {
                push(farc, tmin, tmax);
                node = nearc;
            } else if (!(t > 0.0f) || t > tmax * kEpsHi) {
                node = nearc;
            } else if (t * kEpsHi < tmin) {
                node = farc;
            } else {
                push(farc, t > tmin ? t : tmin, tmax);
                node = nearc;
                tmax = t < tmax ? t : tmax;
            }
            nd = nodes[node];
        }
        c.leaf++;
        const uint32_t begin = nd.x & 0x3FFFFFFFu;
        const uint32_t cnt = nd.y;
        for (uint32_t i = 0; i < cnt; i++) {
            const uint32_t k = leafs[begin + i];
            c.refs++;
            c.tests++;
            const float4 A0 = tris[3 * k], A1 = tris[3 * k + 1], A2 = tris[3 * k + 2];
            // a, e1 = a-b, e2 = a-c (exact precomputed differences)
            const float aox = A0.x - o.x, aoy = A0.y - o.y, aoz = A0.z - o.z;
            const float detA = det3(A1.x, A2.x, d.x, A1.y, A2.y, d.y, A1.z, A2.z, d.z);
            const float beta = det3(aox, A2.x, d.x, aoy, A2.y, d.y, aoz, A2.z, d.z) / detA;
            const float gamma = det3(A1.x, aox, d.x, A1.y, aoy, d.y, A1.z, aoz, d.z) / detA;
            const float t = det3(A1.x, A2.x, aox, A1.y, A2.y, aoy, A1.z, A2.z, aoz) / detA;
            const uint32_t prio = __float_as_uint(A0.w);
            if (beta + gamma < 1.0f && beta > 0.0f && gamma > 0.0f && t > 0.0f &&
                (t < best || (t == best && prio < bprio))) {
                best = t;
                bprio = prio;
                h.tri = (int32_t)k;
                h.beta = beta;
                h.gamma = gamma;
                h.hp = v3(o.x + t * d.x, o.y + t * d.y, o.z + t * d.z);
            }
        }
        if (sp == 0) break;
        sp--;
        {
            const int slot = (sp & (S - 1)) * stride;
            node = st_node[slot];
            tmin = st_lo[slot];
            tmax = st_hi[slot];
            if (sp >= S) {
                const uint4 e = spill[(uint32_t)(sp - S) * spill_stride];
                st_node[slot] = e.x;
                st_lo[slot] = __uint_as_float(e.y);
                st_hi[slot] = __uint_as_float(e.z);
            }
        }
        if (best <= tmin * kEpsLo) break;
    }
    return h;
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

template <bool IN_LDS, int S, int BLOCK>
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
        nodes = reinterpret_cast<const uint2*>(smem + sc.off_nodes);
        leafs = reinterpret_cast<const uint32_t*>(smem + sc.off_leafs);
        geoms = reinterpret_cast<const GpuGeom*>(smem + sc.off_geoms);
    } else {
        tris = reinterpret_cast<const float4*>(sc.image + sc.off_tris);
        nodes = reinterpret_cast<const uint2*>(sc.image + sc.off_nodes);
        leafs = reinterpret_cast<const uint32_t*>(sc.image + sc.off_leafs);
        geoms = reinterpret_cast<const GpuGeom*>(sc.image + sc.off_geoms);
    }
    unsigned char* stk = smem + kp.lds_stack_off;
    uint32_t* st_node = reinterpret_cast<uint32_t*>(stk) + tid;
    float* st_lo = reinterpret_cast<float*>(stk + (size_t)S * BLOCK * 4) + tid;
    float* st_hi = reinterpret_cast<float*>(stk + (size_t)2 * S * BLOCK * 4) + tid;
    const uint32_t gl = blockIdx.x * BLOCK + (uint32_t)tid;
    uint4* spill = kp.spill + gl;
    const uint32_t spill_stride = kp.total_lanes;

    const V3 eye = v3(kp.eye[0], kp.eye[1], kp.eye[2]);
    const V3 fwd = v3(kp.fwd[0], kp.fwd[1], kp.fwd[2]);
    const V3 up = v3(kp.up[0], kp.up[1], kp.up[2]);
    const V3 right = v3(kp.right[0], kp.right[1], kp.right[2]);

    Counters c = {0, 0, 0, 0, 0, 0, 0, 0};
    bool alive = true, has_unit = false, need_path = false;
    uint32_t s = 0, s_end = 0, pix = 0, v = 0, chunk = 0, unit_id = 0;
    Counters c0 = c;
    int px = 0, py = 0, depth = 0;
    uint32_t sd = 1;
    V3 part = v3(0, 0, 0), color = v3(1, 1, 1), o = eye, dir = v3(0, 0, -1);

    for (;;) {
        // ---- 1. refill work units: one atomic per wave ----------------------
        const bool need_unit = alive && !has_unit;
        const uint64_t m = __ballot(need_unit);
        if (m) {
            const int leader = __ffsll((unsigned long long)m) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(kp.counter, (uint32_t)__popcll(m));
            base = __shfl(base, leader);
            if (need_unit) {
                const uint32_t unit = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                if (unit >= kp.total_units) {
                    alive = false;
                } else {
                    unit_id = unit;
                    c0 = c;
                    chunk = unit / kp.npix_local;
                    v = unit - chunk * kp.npix_local;
                    s = chunk * kp.chunk;
                    s_end = min(s + kp.chunk, kp.spp);
                    part = v3(0, 0, 0);
                    if (unit_pixel(kp, v, px, py)) {
                        pix = (uint32_t)py * (uint32_t)kp.width + (uint32_t)px;
                        has_unit = true;
                        need_path = true;
                    } else {
                        kp.partial[(size_t)chunk * kp.npix_local + v] = make_float4(0, 0, 0, 0);
                    }
                }
            }
        }
        if (!__any(alive)) break;

        // ---- 2. new path: primary ray (CUTracer.cu:193-211) ---------------------
        if (alive && has_unit && need_path) {
            sd = rng_init(pix, kp.key, kp.spp_offset + s);
            const float biasx = (float)(uint32_t)px + (rng_next(sd) * 2.0f - 1.0f);
            const float biasy = (float)(uint32_t)py + (rng_next(sd) * 2.0f - 1.0f);
            const double th = (double)kp.tan_half_fov;
            const double W = (double)(uint32_t)kp.width, H = (double)(uint32_t)kp.height;
            const float idx = (float)((2.0 * (double)biasx / W - 1) * th);
            const float idy = (float)((1.0 * H / W - 2.0 * (double)biasy / W) * th);
            const float idz = -1.0f;
            V3 wr;
            wr.x = right.x * idx + up.x * idy - fwd.x * idz;
            wr.y = right.y * idx + up.y * idy - fwd.y * idz;
            wr.z = right.z * idx + up.z * idy - fwd.z * idz;
            normalize_cu(wr);
            o = eye;
            dir = wr;
            color = v3(1, 1, 1);
            depth = 0;
            need_path = false;
            c.paths++;
        }
        const bool tracing = alive && has_unit;

        // ---- 3. closest hit -------------------------------------------------
        Hit h;
        h.tri = -1;
        if (tracing) {
            c.rays++;
            h = trace<S>(o, dir, sc, tris, nodes, leafs, st_node, st_lo, st_hi, BLOCK, spill, spill_stride, c);
        }

        // ---- 4. shade (CUTracer.cu:105-175) ---------------------------------
        if (tracing) {
            bool done = false;
            V3 L = v3(0, 0, 0);
            if (depth < kp.max_depth) {
                if (h.tri < 0) {
                    done = true;
                } else {
                    const uint32_t gi = __float_as_uint(tris[3 * h.tri + 1].w);
                    const GpuGeom& g = geoms[gi];
                    if (g.Ka[0] > 0 || g.Ka[1] > 0 || g.Ka[2] > 0) {
                        L = v3(color.x * (g.Ka[0] * kp.illum), color.y * (g.Ka[1] * kp.illum),
                               color.z * (g.Ka[2] * kp.illum));
                        done = true;
                    } else {
                        c.shades++;
                        const float4 n1 = sc.normals[3 * h.tri], n2 = sc.normals[3 * h.tri + 1],
                                     n3 = sc.normals[3 * h.tri + 2];
                        V3 nrm = vadd(vadd(vscale(v3(n1.x, n1.y, n1.z), 1.0f - h.beta - h.gamma),
                                           vscale(v3(n2.x, n2.y, n2.z), h.beta)),
                                      vscale(v3(n3.x, n3.y, n3.z), h.gamma));
                        normalize_cu(nrm);
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
                        o = vadd(h.hp, vscale(dir, 0.01f));
                        depth++;
                    }
                }
            } else {
                if (h.tri >= 0) {
                    const uint32_t gi = __float_as_uint(tris[3 * h.tri + 1].w);
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
                    kp.partial[(size_t)chunk * kp.npix_local + v] = make_float4(part.x, part.y, part.z, 0.0f);
                    has_unit = false;
                    if (kp.unit_counters) {
                        uint32_t* uc = kp.unit_counters + 4 * (size_t)unit_id;
                        uc[0] = c.rays - c0.rays;
                        uc[1] = c.inner - c0.inner;
                        uc[2] = c.leaf - c0.leaf;
                        uc[3] = c.tests - c0.tests;
                    }
                } else {
                    need_path = true;
                }
            }
        }
    }

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
    auto kern = path_kernel<IN_LDS, S, BLOCK>;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), lds, st, kp);
    return hipGetLastError();
}

}  // namespace

// LDS need of the in-LDS variant for a scene image of `image_bytes`
size_t lds_bytes_in_lds(uint32_t image_bytes, int S) { return (size_t)image_bytes + (size_t)S * kLdsBlock * 12; }

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
        e = launch_path<false, 8, kGlobalBlock>(kp, cus * kGlobalBlocksPerCu, (size_t)8 * kGlobalBlock * 12, st);
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
