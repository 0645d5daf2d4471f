// trace_device.hpp -- per-ray device code shared by the megakernel
// (render.hip) and the wavefront pipeline (wavefront.hip): ray state, root
// interval, the exact Cramer test with its prefilter, the resumable ordered
// KD traversal step, pixel mapping and primary-ray generation.  Both
// pipelines run exactly these operations, so their images are bit-identical.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mcpt_device.hpp"
#include "render_launch.hpp"

namespace mcpt {
namespace trace {

using namespace dev;

struct Counters {
    uint32_t rays, paths, inner, leaf, refs, tests, shades, spills;
};

#ifdef MCPT_PHASE_TIMING
// diagnostic build: executions of a loop body by the wave (w) and by its lanes (l)
struct LaneUse {
    unsigned long long desc_w, desc_l, tri_w, tri_l, burst_w, burst_l;
};
static __device__ LaneUse g_lane_use;   // summed over waves (diagnostic only)
__device__ __forceinline__ void lane_use(unsigned long long& w, unsigned long long& l) {
    const uint64_t ex = __builtin_amdgcn_read_exec();
    if ((threadIdx.x & 63u) == (uint32_t)(__ffsll((unsigned long long)ex) - 1)) {
        w += 1;
        l += (unsigned long long)__popcll(ex);
    }
}
#define MCPT_LANE_USE(wf, lf, acc) lane_use(acc.wf, acc.lf)
#else
#define MCPT_LANE_USE(wf, lf, acc) do {} while (0)
#endif

// IEEE maxNum / minNum as one instruction: a quiet-NaN operand yields the
// other one.  (fmaxf/fminf compile to the same instruction plus a canonicalizing
// v_max of each input, which only matters for signalling NaNs -- the operands
// here are products and stored interval ends, never sNaN.)
__device__ __forceinline__ float max_qnan(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float min_qnan(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// the same over three operands in one instruction (v_max3 / v_min3: the
// nested maxNum / minNum, so the same quiet-NaN rule)
__device__ __forceinline__ float max3_qnan(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float min3_qnan(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float sel3(int a, float x, float y, float z) {
    return a == 0 ? x : (a == 1 ? y : z);
}

// Stack slot (i mod S) of this lane.  RayState::sp and ::lo count stack
// entries in units of one slot row (stride x 16 B), so the slot address is the
// masked position OR the lane's base -- one instruction on every push and pop.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_uint4;
__device__ __forceinline__ uint4 ld4(const lds_uint4* p) {
    const u32x4 v = *p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st4(lds_uint4* p, uint4 v) { *p = u32x4{v.x, v.y, v.z, v.w}; }
template <int S>
__device__ __forceinline__ lds_uint4* slot_of(uint4* st, int stride, int32_t pos) {
    // pos = stack index x (stride x 16 B), so the slot's byte offset is pos's
    // bits under the mask, OR'd with this lane's base (the stack starts at LDS
    // address 0 and a lane's base is below one slot row): one v_and_or_b32
    const uint32_t base = (uint32_t)(size_t)(lds_uint4*)st;
    const uint32_t row = (uint32_t)stride * 16u;
    // (stride is a compile-time block size after inlining, so the test folds)
    if (((S & (S - 1)) == 0) && ((stride & (stride - 1)) == 0)) {
        return (lds_uint4*)(size_t)(((uint32_t)pos & ((uint32_t)(S - 1) * row)) | base);
    } else {                                  // (S or the block not 2^k: the row index mod S)
        return (lds_uint4*)(size_t)(((uint32_t)pos / row % (uint32_t)S) * row + base);
    }
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
    float tmin;
    float tmax;                          // the interval's far end times kEpsHi (rounded), see begin_ray
    float best;
    uint32_t nw0, nw1, bprio;            // current node record
    int32_t sp, htri;                    // sp, lo: stack positions x (slot row bytes), see slot_of
    int32_t lo;                          // stack entries [0, lo) live in the spill memory
    uint32_t lpos, lend;                 // leaf refs still to test (capped leaf loop)
    float hbeta, hgamma;
};

// root interval (oracle: isect_kd_ordered prologue); returns false on a miss
__device__ __forceinline__ bool begin_ray(RayState& r, const GpuScene& sc, float best_init) {
    r.ix = 1.0f / r.d.x;
    r.iy = 1.0f / r.d.y;
    r.iz = 1.0f / r.d.z;
    r.htri = -1;
    r.hbeta = r.hgamma = 0.0f;
    r.best = best_init;
    r.bprio = 0xFFFFFFFFu;
    r.nw0 = sc.root_w[0];
    r.nw1 = sc.root_w[1];
    r.sp = 0;
    r.lo = 0;
    r.lpos = r.lend = 0;
    float tmin = 0.0f, tmax = kFltMax;
    const float oo[3] = {r.o.x, r.o.y, r.o.z}, dd[3] = {r.d.x, r.d.y, r.d.z}, inv[3] = {r.ix, r.iy, r.iz};
    bool miss = false;
    // branch-free: a zero direction component only tests the origin against
    // that slab and leaves the interval alone (no exec-mask branches in the
    // extend's hand-off, where every new ray passes through here)
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const bool z = dd[a] == 0.0f;
        miss = miss | (z & ((oo[a] < sc.root_min[a]) | (oo[a] > sc.root_max[a])));
        const float t0 = (sc.root_min[a] - oo[a]) * inv[a];
        const float t1 = (sc.root_max[a] - oo[a]) * inv[a];
        const float lo = dd[a] < 0.0f ? t1 : t0;
        const float hi = dd[a] < 0.0f ? t0 : t1;
        tmin = (!z & (lo > tmin)) ? lo : tmin;
        tmax = (!z & (hi < tmax)) ? hi : tmax;
    }
    r.tmin = tmin;
    // the walk compares against tmax only as tmax * kEpsHi, so the state keeps
    // that product: RN(x * kEpsHi) is monotone in x, hence RN(min(t, tmax) * kEpsHi)
    // = min(RN(t * kEpsHi), RN(tmax * kEpsHi)) and the interval updates keep it
    // exactly (one multiply per descent step less; stack entries carry it too)
    r.tmax = tmax * kEpsHi;
    return !miss && !(tmin > r.tmax);
}

// Cramer test (CUTracer.cu:54-92) with an exact-result-preserving prefilter:
// the three IEEE divisions run only when the signs of the determinants allow
// beta, gamma, t > 0 and the magnitudes do not already rule out beta+gamma < 1
// or t < best (2^-20 margins cover every rounding of the exact path).
struct TriDets {
    float detA, qb, qg, qt;
};
__device__ __forceinline__ bool tri_prefilter(const RayState& r, const float4 A0, const float4 A1, const float4 A2,
                                              TriDets& q) {
    const float aox = A0.x - r.o.x, aoy = A0.y - r.o.y, aoz = A0.z - r.o.z;
    // A2.w = A1.y * A2.z - A2.y * A1.z, precomputed (the last minor of det A and det tM)
    q.detA = det3_m(A1.x, A2.x, r.d.x, A1.y, A2.y, r.d.y, A1.z, A2.z, r.d.z, A2.w);
    q.qb = det3(aox, A2.x, r.d.x, aoy, A2.y, r.d.y, aoz, A2.z, r.d.z);
    q.qg = det3(A1.x, aox, r.d.x, A1.y, aoy, r.d.y, A1.z, aoz, r.d.z);
    q.qt = det3_m(A1.x, A2.x, aox, A1.y, A2.y, aoy, A1.z, A2.z, aoz, A2.w);
    // sign-normalised numerators: beta, gamma, t > 0 needs all three > 0 (a NaN
    // anywhere means no hit, so min3 may drop it); detA == 0 fails the magnitude test
    const uint32_t sA = __float_as_uint(q.detA) & 0x80000000u;
    const float xb = __uint_as_float(__float_as_uint(q.qb) ^ sA);
    const float xg = __uint_as_float(__float_as_uint(q.qg) ^ sA);
    const float xt = __uint_as_float(__float_as_uint(q.qt) ^ sA);
    const bool signs_ok = __builtin_fminf(__builtin_fminf(xb, xg), xt) > 0.0f;
    const float adet = fabsf(q.detA) * 1.00000095367431640625f;   // 1 + 2^-20
    const bool mags_ok = !(xb + xg > adet) & !(xt > r.best * adet);
    return signs_ok & mags_ok;
}
// the IEEE quotients of the Cramer test (CUTracer.cu:84-92)
__device__ __forceinline__ void tri_quotients(const TriDets& q, float& beta, float& gamma, float& t) {
    const double rA = recip_shared(q.detA);   // (= IEEE f32 division, mcpt_device.hpp)
    beta = div_shared(q.qb, rA);
    gamma = div_shared(q.qg, rA);
    t = div_shared(q.qt, rA);
}
// the exact tail of a triangle whose prefilter passed
__device__ __forceinline__ void tri_accept(RayState& r, const TriDets& q, uint32_t prio, uint32_t k) {
    float beta, gamma, t;
    tri_quotients(q, beta, gamma, t);
    if (beta + gamma < 1.0f && beta > 0.0f && gamma > 0.0f && t > 0.0f &&
        (t < r.best || (t == r.best && prio < r.bprio))) {
        r.best = t;
        r.bprio = prio;
        r.htri = (int32_t)k;
        r.hbeta = beta;
        r.hgamma = gamma;
    }
}
// (t, beta, gamma) of ray (o, d) against the triangle record A0..A2: the same
// operations as the traversal's accepted hit, so a hit recomputed from the
// triangle id is bit-identical to the one the traversal found
__device__ __forceinline__ void tri_hit_params(V3 o, V3 d, const float4 A0, const float4 A1, const float4 A2,
                                               float& t, float& beta, float& gamma) {
    RayState r;
    r.o = o;
    r.d = d;
    r.best = 0.0f;
    TriDets q;
    (void)tri_prefilter(r, A0, A1, A2, q);
    tri_quotients(q, beta, gamma, t);
}
__device__ __forceinline__ void test_tri_v(RayState& r, const float4 A0, const float4 A1, const float4 A2, uint32_t k) {
    TriDets q;
    if (tri_prefilter(r, A0, A1, A2, q)) tri_accept(r, q, __float_as_uint(A0.w), k);
}
// Two triangles a, b of a leaf (b only if `two`): both prefilters first (b's
// with the best before a's tail -- a larger best only widens the prefilter, the
// exact tail still decides), then ONE exact tail for a lane's first candidate
// (a, else b) and a second one only for lanes where both passed: a wave with
// some lanes passing on a and others on b runs the tail once, not twice.  The
// closest hit is the lexicographic minimum of (t, rank), so the tail order is
// immaterial.
// EARLY_PRIO (records in global memory): the tail's rank select is made before
// the tail's branch, so the records' .w words come with their first loads
// (one 16-B load each) instead of a dependent 4-B load inside the tail
template <bool EARLY_PRIO = false>
__device__ __forceinline__ void test_tri_pair(RayState& r, const float4 A0, const float4 A1, const float4 A2,
                                              uint32_t ka, const float4 B0, const float4 B1, const float4 B2,
                                              uint32_t kb, bool two) {
    TriDets qa, qb;
    const bool oka = tri_prefilter(r, A0, A1, A2, qa);
    const bool okb = tri_prefilter(r, B0, B1, B2, qb) & two;
    uint32_t prio = 0;
    if constexpr (EARLY_PRIO) prio = oka ? __float_as_uint(A0.w) : __float_as_uint(B0.w);
    if (oka | okb) {
        TriDets q;
        q.detA = oka ? qa.detA : qb.detA;
        q.qb = oka ? qa.qb : qb.qb;
        q.qg = oka ? qa.qg : qb.qg;
        q.qt = oka ? qa.qt : qb.qt;
        if constexpr (!EARLY_PRIO) prio = oka ? __float_as_uint(A0.w) : __float_as_uint(B0.w);
        tri_accept(r, q, prio, oka ? ka : kb);
    }
    if (oka & okb) tri_accept(r, qb, __float_as_uint(B0.w), kb);
}
__device__ __forceinline__ void test_tri(RayState& r, const float4* __restrict__ tris, uint32_t k) {
    test_tri_v(r, tris[k], tris[k + 1], tris[k + 2], k);
}

// A triangle record read whole (16 B): the compiler would narrow reads whose .w
// is unused to 12 B, and the LDS array serves a ds_read_b96 in 8 cycles, a
// ds_read_b128 in 4 (MI355X_MICROARCH.md, LDS table).
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) f32x4 lds_f32x4;
template <bool IN_LDS>
__device__ __forceinline__ float4 ld_tri(const float4* __restrict__ p) {
    if constexpr (IN_LDS) {     // (volatile: not narrowed)
        const f32x4 v = *(const volatile lds_f32x4*)p;
        return make_float4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}

// One resumable traversal iteration: descend to a leaf, test it (two
// triangles at most, both records read up front), pop (the stack top read
// during the tests).  Returns true when the ray's closest hit is final.  The
// children of the current node are read as one 16-B sibling-pair record whose
// address is known before the split-plane decision, so the LDS latency overlaps
// the decision; stack entries carry the far child's record (16 B: w0, w1, lo,
// hi), so a pop needs no node re-read.
// Diagnostic builds only (-DMCPT_PHASE_MARKERS, scripts/phase_isa.py): a
// marker pair `s_nop 15; s_nop n` at each phase boundary of the walk, so the
// static instruction count of each phase can be read from the code object.
#ifdef MCPT_PHASE_MARKERS
#define MCPT_MARK(n) asm volatile("s_nop 15\n\ts_nop " #n ::: "memory")
#else
#define MCPT_MARK(n) do {} while (0)
#endif
#ifdef MCPT_PHASE_TIMING
#define MCPT_LU_PARAM , LaneUse& lu
#define MCPT_LU_ARG , lu
#else
#define MCPT_LU_PARAM
#define MCPT_LU_ARG
#endif
// Descent steps per call are capped (MCPT_DESCENT_CAP): a lane that has not
// reached a leaf keeps its node record and interval in RayState and resumes on
// the next call, so the wave's descent loop is not as long as its deepest
// lane's (lane use of the uncapped loop: 22%; cap sweep at the current kernel:
// 3 / 4 / 5 / 6 -> 10.60 / 10.71 / 10.61 / 10.37 G rays/s).  Likewise two
// triangle tests per call (a pair), the leaf's remaining refs [lpos, lend)
// kept in RayState (uncapped leaf loop: 35%).  Same visit order and counts.
#ifndef MCPT_DESCENT_CAP
#define MCPT_DESCENT_CAP 4
#endif
#ifndef MCPT_DESCENT_CAP_GLOBAL
#define MCPT_DESCENT_CAP_GLOBAL 5                // global-memory scenes (C4: 5 > 4)
#endif
// Child-box cull (scenes in global memory): each sibling-pair record also
// carries both children's KD boxes (the node region clipped to its
// triangles' bounds, KDTree.hpp:154-155) as fp16 rounded outward
// (half_box.hpp).  A child whose box the ray segment (0, best] misses is not
// entered: a hit that could improve `best` lies inside the exact box, hence
// inside the stored one, and its slab intervals contain t up to rounding,
// which the 2^-12 margins cover.
__device__ __forceinline__ float h2f(uint32_t bits16) {
    return (float)__builtin_bit_cast(_Float16, (unsigned short)bits16);
}
// box = lo.x lo.y | lo.z hi.x | hi.y hi.z as three packed fp16 pairs.
// Slab ends ordered by the sign of the direction, not by value, and the
// interval updated by NaN-passing max / min: a zero component has
// inv = +-inf, so (b - o) * inv is -inf / +inf on the inside / outside of each
// bound and NaN (no constraint) with the origin on it -- exactly the
// containment test, with no mask and no branch.  (Round 5's form ordered the
// ends by value, masked zero components and put the containment test in a
// rare branch: 14 VALU more per descent step; C4 +4.0% with this one,
// PERFLOG round 6.)  Equal decisions for every box with lo <= hi; an
// inverted (empty-node) box is always culled.
__device__ __forceinline__ bool box_hit(const RayState& r, uint32_t b0, uint32_t b1, uint32_t b2) {
    const float lx = h2f(b0 & 0xFFFFu), hx = h2f(b1 >> 16);
    const float ly = h2f(b0 >> 16), hy = h2f(b2 & 0xFFFFu);
    const float lz = h2f(b1 & 0xFFFFu), hz = h2f(b2 >> 16);
    const bool nx = __float_as_uint(r.d.x) >> 31, ny = __float_as_uint(r.d.y) >> 31, nz = __float_as_uint(r.d.z) >> 31;
    const float tx0 = ((nx ? hx : lx) - r.o.x) * r.ix, tx1 = ((nx ? lx : hx) - r.o.x) * r.ix;
    const float ty0 = ((ny ? hy : ly) - r.o.y) * r.iy, ty1 = ((ny ? ly : hy) - r.o.y) * r.iy;
    const float tz0 = ((nz ? hz : lz) - r.o.z) * r.iz, tz1 = ((nz ? lz : hz) - r.o.z) * r.iz;
    const float lo = max_qnan(max3_qnan(0.0f, tx0, ty0), tz0);
    const float hi = min_qnan(min3_qnan(r.best, tx1, ty1), tz1);
    return !(lo * kEpsLo > hi * kEpsHi);
}

// a loaded value made an asm output: its wait sits here, not at a later join
__device__ __forceinline__ uint4 settle4(uint4 v) {
    asm volatile("v_mov_b32 %0, %0\n\tv_mov_b32 %1, %1\n\tv_mov_b32 %2, %2\n\tv_mov_b32 %3, %3"
                 : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
    return v;
}
// Pop the next interval: false = traversal finished (empty stack, or the best
// hit lies before the popped interval)
// LAZY (scenes in LDS, 4-entry LDS part): the LDS part holds entries
// [lo, sp), older ones are in memory; a push spills only when the LDS part is
// full and a pop reads memory only when it is empty, so a push after a pop
// neither re-stores nor (as the eager refill did) reloads an entry, and no pop
// waits for a refill it may never use (C2 +0.9%, spills/ray 0.32 -> see bench).
// Eager (global-memory scenes, 8-entry LDS part, spills rare): the freed slot
// is refilled at once.
// `top`, if given, is the LDS slot of the top entry read ahead by the caller.
template <int S, bool LAZY>
__device__ __forceinline__ bool pop_entry(RayState& r, uint4* st, int stride, uint4* __restrict__ spill,
                                          uint32_t spill_stride, const uint4* top = nullptr) {
    const int32_t U = stride * 16;          // one stack position
    if (r.sp == 0) return false;
    r.sp -= U;
    uint4 e;
    if constexpr (LAZY) {
        if (r.sp < r.lo) {                    // LDS part empty: the entry is in memory
            // (settled inside this branch: at the join a wait for it would be
            // a vmcnt(0) on every pop, i.e. a wait for the extend's next-ray
            // prefetch and hit stores)
            e = settle4(spill[((uint32_t)r.sp / (uint32_t)U) * spill_stride]);
            r.lo = r.sp;
        } else {
            if (top) e = *top;
            else e = ld4(slot_of<S>(st, stride, r.sp));
        }
    } else {                                  // refill the freed slot with the next older entry
        lds_uint4* slot = slot_of<S>(st, stride, r.sp);
        if (top) e = *top;
        else e = ld4(slot);
        if (r.sp >= S * U) st4(slot, spill[((uint32_t)r.sp / (uint32_t)U - S) * spill_stride]);
    }
    r.nw0 = e.x;
    r.nw1 = e.y;
    r.tmin = __uint_as_float(e.z);
    r.tmax = __uint_as_float(e.w);
    return !(r.best <= r.tmin * kEpsLo);
}

constexpr uint32_t kLeftMask = 0x3FFFFFFFu;   // inner node word: child pair index

// Descent of a ray between leaves: at most `cap` inner-node steps (the node
// record and interval stay in the ray state); 0 = cap reached mid-descent,
// 1 = a leaf reached (its refs in [lpos, lend)), 2 = the walk ended (a
// global-memory scene's box cull popped past the last interval).
// COUNT = false (lean renders): the counters are compiled out.
template <int S, bool BOXES = false, bool COUNT = true>
__device__ __forceinline__ int descend_steps(RayState& r, const uint2* __restrict__ nodes1, uint4* st, int stride,
                                             uint4* __restrict__ spill, uint32_t spill_stride, Counters& c,
                                             const uint4* __restrict__ pairs, int cap MCPT_LU_PARAM) {
    const int32_t U = stride * 16;            // one stack position (see slot_of)
    // the walk advances r.nw0/r.nw1 in place (local copies written back at
    // the cap cost register moves on every path through the loop)
    uint32_t& w0 = r.nw0;
    uint32_t& w1 = r.nw1;
    int steps = 0;
    while ((w0 >> 30) != 3u) {
        if (steps == cap) return 0;           // resume next call
        steps++;
        MCPT_MARK(1);
        if constexpr (COUNT) c.inner++;
        MCPT_LANE_USE(desc_w, desc_l, lu);
        const uint32_t left = w0 & kLeftMask;
        uint4 pr, bx0, bx1;
        if constexpr (BOXES) {            // 48-B pair record: words, box(left), box(right)
            const uint4* rec = pairs + left;   // (global layout: left = the record's 16-B offset)
            pr = rec[0];
            bx0 = rec[1];
            bx1 = rec[2];
        } else {
            pr = *reinterpret_cast<const uint4*>(nodes1 + left);   // children left, left+1
        }
        const int a = (int)(w0 >> 30);
        const float sv = __uint_as_float(w1);
        const float oa = sel3(a, r.o.x, r.o.y, r.o.z);
        const float ia = sel3(a, r.ix, r.iy, r.iz);
        const float t = (sv - oa) * ia;
        // near side: below the plane, or on it and heading down; pp = ray inside
        // the plane (both children).  Only an origin exactly on the plane needs
        // the direction, so its select and tests sit in a rarely taken branch.
        bool below = oa < sv, pp = false;
        if (__builtin_expect(oa == sv, 0)) {
            const float da = sel3(a, r.d.x, r.d.y, r.d.z);
            below = da <= 0.0f;
            pp = da == 0.0f;
        }
        // if/else chain of the oracle, evaluated branch-free
        const float te = t * kEpsHi;
        const bool no = !(t > 0.0f) | (t > r.tmax);                 // near child only
        const bool fo = te < r.tmin;                                // far child only
        const bool go_far = !pp & !no & fo;
        const bool both = !pp & !no & !fo;                          // push far, go near
        bool push_it = pp | both;
        bool near_ok = true, far_ok = true;
        if constexpr (BOXES) {
            const bool hl = box_hit(r, bx0.x, bx0.y, bx0.z);
            const bool hr = box_hit(r, bx0.w, bx1.x, bx1.y);
            near_ok = below ? hl : hr;
            far_ok = below ? hr : hl;
            push_it = push_it & far_ok;
        }
        const uint32_t f0 = below ? pr.z : pr.x, f1 = below ? pr.w : pr.y;     // far child record
        if (push_it) {
            // pp ? tmin : max(t, tmin) without the select: a pp lane's t is
            // (+0) * (+-inf) = NaN (da = +-0, oa == sv), and max returns tmin
            const float plo = max_qnan(t, r.tmin);
            lds_uint4* slot = slot_of<S>(st, stride, r.sp);
            if constexpr (!BOXES) {
                if (r.sp - r.lo == S * U) {       // LDS part full: its oldest entry (same slot) to memory
                    spill[((uint32_t)r.lo / (uint32_t)U) * spill_stride] = ld4(slot);
                    r.lo += U;
                    if constexpr (COUNT) c.spills++;
                }
            } else if (r.sp >= S * U) {
                spill[((uint32_t)r.sp / (uint32_t)U - S) * spill_stride] = ld4(slot);
                if constexpr (COUNT) c.spills++;
            }
            st4(slot, make_uint4(f0, f1, __float_as_uint(plo), __float_as_uint(r.tmax)));
            r.sp += U;
            if constexpr (!BOXES)                // here push_it & !pp == both; te = NaN for pp
                r.tmax = min_qnan(te, r.tmax);
        }
        if constexpr (BOXES)                                        // the near child's interval,
            if (both) r.tmax = te < r.tmax ? te : r.tmax;           // pushed far or not
        // the child entered: the near one, or the far one when go_far (the
        // left record when below != go_far) -- two selects, not four
        const bool enter_left = below != go_far;
        w0 = enter_left ? pr.x : pr.z;
        w1 = enter_left ? pr.y : pr.w;
        if constexpr (BOXES) {
            if (!(go_far ? far_ok : near_ok)) {   // the chosen child's box is missed: next interval
                if (!pop_entry<S, !BOXES>(r, st, stride, spill, spill_stride)) return 2;
            }
        }
    }
    MCPT_MARK(2);
    if constexpr (COUNT) c.leaf++;
    r.lpos = w0 & 0x3FFFFFFFu;
    r.lend = r.lpos + w1;
    return 1;
}

// COUNT = false (lean renders): the counters below are compiled out (rays stay)
// TRIS_LDS: `tris` points into LDS (the scene image copied there), so its
// records can be read by full-width LDS loads (ld_tri).  CAP: descent steps per
// call (0: MCPT_DESCENT_CAP / MCPT_DESCENT_CAP_GLOBAL).
template <int S, bool BOXES = false, bool COUNT = true, bool TRIS_LDS = false, int CAP = 0>
__device__ __forceinline__ bool trav_iter(RayState& r, const float4* __restrict__ tris,
                                          const uint2* __restrict__ nodes1, const uint32_t* __restrict__ leafs,
                                          uint4* st, int stride, uint4* __restrict__ spill, uint32_t spill_stride,
                                          Counters& c MCPT_LU_PARAM, const uint4* __restrict__ pairs = nullptr) {
    const int32_t U = stride * 16;            // one stack position (see slot_of)
    if (r.lpos == r.lend) {                   // between leaves: descend
        const int k = descend_steps<S, BOXES, COUNT>(r, nodes1, st, stride, spill, spill_stride, c, pairs,
                                                      CAP > 0 ? CAP : BOXES ? MCPT_DESCENT_CAP_GLOBAL : MCPT_DESCENT_CAP
                                                      MCPT_LU_ARG);
        if (k == 0) return false;
        if (k == 2) return true;
    }
    // the stack's top slot, read ahead: the pop after this leaf's last tests
    // then needs no LDS round trip of its own (unused if the leaf goes on or
    // the stack is empty -- the slot index is in range either way)
    MCPT_MARK(3);
    const uint4 top = ld4(slot_of<S>(st, stride, r.sp - U));
    if (r.lpos < r.lend) {
        // both triangles' records are read before either test runs, so the two
        // LDS round trips (leaf ref -> triangle) overlap instead of chaining; a
        // leaf's last single triangle re-reads its own record as the second one
        // (in bounds: the ref after a leaf section's end is image padding/geoms).
        // (Leaf records carrying their first two triangle slots inline, with the
        // next pair prefetched a call ahead, removed the ref round trip but
        // measured 10.52 vs 10.72 G rays/s: the kernel is issue-bound there.)
        const bool two = r.lend - r.lpos >= 2u;
        const uint32_t k0 = leafs[r.lpos], k1n = leafs[r.lpos + 1u];
        const uint32_t k1 = two ? k1n : k0;
        const float4 a0 = ld_tri<TRIS_LDS>(tris + k0), a1 = ld_tri<TRIS_LDS>(tris + k0 + 1);
        const float4 a2 = ld_tri<TRIS_LDS>(tris + k0 + 2), b0 = ld_tri<TRIS_LDS>(tris + k1);
        const float4 b1 = ld_tri<TRIS_LDS>(tris + k1 + 1), b2 = ld_tri<TRIS_LDS>(tris + k1 + 2);
        MCPT_LANE_USE(tri_w, tri_l, lu);
        if constexpr (COUNT) c.refs += two ? 2u : 1u;
        if constexpr (COUNT) c.tests += two ? 2u : 1u;
        test_tri_pair<!TRIS_LDS>(r, a0, a1, a2, k0, b0, b1, b2, k1, two);
        r.lpos += two ? 2u : 1u;
    }
    MCPT_MARK(4);
    if (r.lpos < r.lend) return false;        // more triangles in this leaf
    return !pop_entry<S, !BOXES>(r, st, stride, spill, spill_stride, &top);
}

// work unit v (packed owned-pixel index) -> image pixel; false outside the image
__device__ __forceinline__ bool unit_pixel(const KernelParams& kp, uint32_t v, int& x, int& y) {
    const uint32_t k = kp.div_tt.div(v), w = v - k * kp.div_tt.d;
    const uint32_t t = (uint32_t)kp.shard_index + k * (uint32_t)kp.shard_count;
    const uint32_t ty = kp.div_tiles_x.div(t), tx = t - ty * (uint32_t)kp.tiles_x;
    const uint32_t wy = kp.div_tile.div(w), wx = w - wy * (uint32_t)kp.tile;
    x = (int)(tx * (uint32_t)kp.tile + wx);
    y = (int)(ty * (uint32_t)kp.tile + wy);
    return x < kp.width && y < kp.height;
}

// primary ray of pixel (px, py) from its sample's RNG seed sd (CUTracer.cu:186-211)
__device__ __forceinline__ void primary_ray_sd(const KernelParams& kp, int px, int py, uint32_t& sd, V3& dir) {
    const float biasx = (float)(uint32_t)px + (rng_next(sd) * 2.0f - 1.0f);
    const float biasy = (float)(uint32_t)py + (rng_next(sd) * 2.0f - 1.0f);
    const double th = (double)kp.tan_half_fov;
    const double W = (double)(uint32_t)kp.width;
    // (2 b) / W == (2 b) * 2^-k exactly when W = 2^k; 1.0 * H / W is the host's
    // identical IEEE double division
    const double qx = kp.inv_w_pow2 != 0.0 ? 2.0 * (double)biasx * kp.inv_w_pow2 : 2.0 * (double)biasx / W;
    const double qy = kp.inv_w_pow2 != 0.0 ? 2.0 * (double)biasy * kp.inv_w_pow2 : 2.0 * (double)biasy / W;
    const float idx = (float)((qx - 1) * th);
    const float idy = (float)((kp.h_over_w - qy) * th);
    const float idz = -1.0f;
    V3 wr;
    wr.x = kp.right[0] * idx + kp.up[0] * idy - kp.fwd[0] * idz;
    wr.y = kp.right[1] * idx + kp.up[1] * idy - kp.fwd[1] * idz;
    wr.z = kp.right[2] * idx + kp.up[2] * idy - kp.fwd[2] * idz;
    normalize_cu(wr);
    dir = wr;
}
// primary_ray_sd's direction before its normalize, from its two jitter
// uniforms u1, u2 (the main loop normalizes it together with the shading
// normals of the scattering lanes)
__device__ __forceinline__ V3 primary_dir_raw(const KernelParams& kp, int px, int py, float u1, float u2) {
    const float biasx = (float)(uint32_t)px + (u1 * 2.0f - 1.0f);
    const float biasy = (float)(uint32_t)py + (u2 * 2.0f - 1.0f);
    const double th = (double)kp.tan_half_fov;
    const double W = (double)(uint32_t)kp.width;
    const double qx = kp.inv_w_pow2 != 0.0 ? 2.0 * (double)biasx * kp.inv_w_pow2 : 2.0 * (double)biasx / W;
    const double qy = kp.inv_w_pow2 != 0.0 ? 2.0 * (double)biasy * kp.inv_w_pow2 : 2.0 * (double)biasy / W;
    const float idx = (float)((qx - 1) * th);
    const float idy = (float)((kp.h_over_w - qy) * th);
    const float idz = -1.0f;
    V3 wr;
    wr.x = kp.right[0] * idx + kp.up[0] * idy - kp.fwd[0] * idz;
    wr.y = kp.right[1] * idx + kp.up[1] * idy - kp.fwd[1] * idz;
    wr.z = kp.right[2] * idx + kp.up[2] * idy - kp.fwd[2] * idz;
    return wr;
}
// primary ray of sample s of pixel (px, py)
__device__ __forceinline__ void primary_ray(const KernelParams& kp, uint32_t pix, int px, int py, uint32_t s,
                                            uint32_t& sd, V3& dir) {
    sd = rng_init(pix, kp.key, kp.spp_offset + s);
    primary_ray_sd(kp, px, py, sd, dir);
}


// ---- shading (CUTracer.cu:105-175) ------------------------------------------
__device__ __forceinline__ bool is_emitter(const GpuGeom& g) {   // CUTracer.cu:111
    return g.Ka[0] > 0 || g.Ka[1] > 0 || g.Ka[2] > 0;
}
__device__ __forceinline__ V3 emitted(V3 color, const GpuGeom& g, float illum) {   // :112-113, :166-170
    return v3(color.x * (g.Ka[0] * illum), color.y * (g.Ka[1] * illum), color.z * (g.Ka[2] * illum));
}
// One scatter event at a non-emitting hit (CUTracer.cu:120-160): interpolated
// normal, BSDF sample by material, throughput update, next origin/direction.
// n1..n3 are the hit triangle's vertex normals (fetched by the caller).  QE:
// rtx.hlsl:336-358 -- HLSL normalize of the normal, QE Fresnel (always
// normalized), Phong with the float Ns; fresnel_kd is 0 for QE (rtx.hlsl:345).
template <bool QE = false>
__device__ __forceinline__ void scatter_n(const GpuGeom& g, float4 n1, float4 n2, float4 n3, float hbeta,
                                          float hgamma, float best, int32_t fresnel_kd, uint32_t& sd, V3& color,
                                          V3& o, V3& d) {
    V3 nrm = vadd(vadd(vscale(v3(n1.x, n1.y, n1.z), 1.0f - hbeta - hgamma), vscale(v3(n2.x, n2.y, n2.z), hbeta)),
                  vscale(v3(n3.x, n3.y, n3.z), hgamma));
    if constexpr (QE) normalize_hlsl(nrm);
    else normalize_cu(nrm);
    V3 dir = d;
    if (g.Tr > 0) {
        dir = sample_fresnel<QE>(sd, nrm, dir, g.Tr, g.Ni);
        if (fresnel_kd) color = v3(color.x * g.Kd[0], color.y * g.Kd[1], color.z * g.Kd[2]);
    } else {
        // Phong (Utils.hpp:72-95) and diffuse (:46-70) share one sampler body
        const bool ph = g.Ns > 1;
        const bool flip = dot3(dir, nrm) > 0;
        const V3 h = sample_lobe(sd, nrm, ph, QE ? g.Ns + 1.0f : (float)(g.Ns_u + 1u));
        if (ph) {
            dir = vsub(dir, vscale(vscale(h, dot3(dir, h)), 2.0f));
            color = v3(color.x * g.Ks[0], color.y * g.Ks[1], color.z * g.Ks[2]);
        } else {
            color = v3(color.x * g.Kd[0], color.y * g.Kd[1], color.z * g.Kd[2]);
            dir = flip ? v3(-h.x, -h.y, -h.z) : h;
        }
    }
    // hitPoint = pos + t*dir at the accepted t (CUTracer.cu:89-91), then
    // pos = hitPoint + dir*0.01 (:134,143,159)
    const V3 hp = v3(o.x + best * d.x, o.y + best * d.y, o.z + best * d.z);
    o = vadd(hp, vscale(dir, 0.01f));
    d = dir;
}
// The shading normal before its normalize (CUTracer.cu:120-126)
__device__ __forceinline__ V3 shading_normal_raw(const float4* __restrict__ normals, int32_t htri, float hbeta,
                                                 float hgamma) {
    const float4 n1 = normals[htri], n2 = normals[htri + 1], n3 = normals[htri + 2];
    return vadd(vadd(vscale(v3(n1.x, n1.y, n1.z), 1.0f - hbeta - hgamma), vscale(v3(n2.x, n2.y, n2.z), hbeta)),
                vscale(v3(n3.x, n3.y, n3.z), hgamma));
}
// scatter_n (CVMCTracer mode) from the normalized shading normal and the
// lane's next two uniforms, already drawn (u2 unused by a Fresnel material)
__device__ __forceinline__ void scatter_u(const GpuGeom& g, V3 nrm, float u1, float u2, float best,
                                          int32_t fresnel_kd, V3& color, V3& o, V3& d) {
    V3 dir = d;
    if (g.Tr > 0) {
        dir = sample_fresnel_u<false>(u1, nrm, dir, g.Tr, g.Ni);
        if (fresnel_kd) color = v3(color.x * g.Kd[0], color.y * g.Kd[1], color.z * g.Kd[2]);
    } else {
        const bool ph = g.Ns > 1;
        const bool flip = dot3(dir, nrm) > 0;
        const V3 h = sample_lobe_u(u1, u2, nrm, ph, (float)(g.Ns_u + 1u));
        if (ph) {
            dir = vsub(dir, vscale(vscale(h, dot3(dir, h)), 2.0f));
            color = v3(color.x * g.Ks[0], color.y * g.Ks[1], color.z * g.Ks[2]);
        } else {
            color = v3(color.x * g.Kd[0], color.y * g.Kd[1], color.z * g.Kd[2]);
            dir = flip ? v3(-h.x, -h.y, -h.z) : h;
        }
    }
    const V3 hp = v3(o.x + best * d.x, o.y + best * d.y, o.z + best * d.z);
    o = vadd(hp, vscale(dir, 0.01f));
    d = dir;
}
template <bool QE = false>
__device__ __forceinline__ void scatter(const GpuGeom& g, const float4* __restrict__ normals, int32_t htri,
                                        float hbeta, float hgamma, float best, int32_t fresnel_kd, uint32_t& sd,
                                        V3& color, V3& o, V3& d) {
    const float4 n1 = normals[htri], n2 = normals[htri + 1], n3 = normals[htri + 2];
    scatter_n<QE>(g, n1, n2, n3, hbeta, hgamma, best, fresnel_kd, sd, color, o, d);
}
// material class of a geometry for the wavefront's per-material queues
__device__ __forceinline__ uint32_t material_class(const GpuGeom& g) {
    return g.Tr > 0 ? 3u : (g.Ns > 1 ? 2u : 1u);
}


// ---- wave-level helpers -----------------------------------------------------
// Reserve one slot per lane with `want` in a device-wide append buffer: one
// atomic per wave (ballot + popcount), lanes ranked by their position.
// x of lane `src` (wave-uniform) for every lane: v_readlane into a scalar
// register -- what __shfl(x, src) computes, without its ds_bpermute round trip
__device__ __forceinline__ uint32_t lane_bcast(uint32_t x, int src) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, src);
}
__device__ __forceinline__ uint32_t wave_append(bool want, uint32_t* counter) {
    const uint64_t m = __ballot(want);
    const int lane = (int)(threadIdx.x & 63u);
    uint32_t base = 0;
    if (m) {
        const int leader = __ffsll((unsigned long long)m) - 1;
        if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
        base = lane_bcast(base, leader);
    }
    return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}
constexpr uint32_t kChunk = 64;           // indices a wave reserves at once
// Wave-level reservation: lanes with `want` get consecutive indices from the
// wave's current 64-index chunk of a shared counter (LDS or global), one
// atomic per 64 indices instead of one per refill.
struct SlotCursor {
    uint32_t base, used;
    __device__ __forceinline__ uint32_t take(bool want, uint32_t* counter) {
        const uint64_t m = __ballot(want);
        const uint32_t n = (uint32_t)__popcll(m);
        const int lane = (int)(threadIdx.x & 63u);
        const uint32_t rank = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        uint32_t res = base + used + rank;
        if (used + n > kChunk) {                       // wave-uniform
            const uint32_t first = kChunk - used;
            uint32_t nb = 0;
            if (lane == 0) nb = atomicAdd(counter, kChunk);
            nb = lane_bcast(nb, 0);
            if (rank >= first) res = nb + (rank - first);
            base = nb;
            used = n - first;
        } else {
            used += n;
        }
        return res;
    }
};

// counters: wave reduction in 64 bits (64 lanes of 32-bit counts may exceed
// 2^32), one atomic per wave per counter
__device__ __forceinline__ void flush_counters(const Counters& c, unsigned long long* stats) {
    const uint32_t vals[8] = {c.rays, c.paths, c.inner, c.leaf, c.refs, c.tests, c.shades, c.spills};
    unsigned long long sums[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        unsigned long long x = vals[i];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
        sums[i] = x;
    }
    if ((threadIdx.x & 63u) == 0) {
#pragma unroll
        for (int i = 0; i < 8; i++)
            if (sums[i]) atomicAdd(stats + i, sums[i]);
    }
}
// Per-lane counts are 32-bit: a wave flushes them (and restarts from 0) once
// any lane's largest count passes 2^30, so no count can wrap however long a
// persistent wave runs (a C4-mesh frame at 4096 spp reaches ~2^21 per lane).
// Wave-uniform; the check is one compare and a ballot per main-loop round.
template <bool COUNT>
__device__ __forceinline__ void bound_counters(Counters& c, unsigned long long* stats) {
    const uint32_t big = COUNT ? c.inner : c.rays;   // the fastest-growing count of the kernel
    if (__ballot(big > (1u << 30))) {
        flush_counters(c, stats);
        c = Counters{0, 0, 0, 0, 0, 0, 0, 0};
    }
}


// ---- QuinEngine semantics (rtx.hlsl:304-405) ----------------------------------
constexpr int32_t kModeQE = 1;
constexpr float kQeGamma = 2.2f;
constexpr float kQeInvGamma = 0.454545454545f;   // 1 / 2.2 as float
// primary ray: TEA-16(pixel, frame seed) + two warm-up draws, +-0.5 px jitter,
// origin on the near plane z = -1 of the view, view -> world by the basis
__device__ __forceinline__ void primary_ray_qe_sd(const KernelParams& kp, int px, int py, uint32_t& sd, V3& o,
                                                  V3& dir) {
    (void)rng_next(sd);
    (void)rng_next(sd);
    const float bx = (float)(uint32_t)px + (rng_next(sd) - 0.5f);
    const float by = (float)(uint32_t)py + (rng_next(sd) - 0.5f);
    const float vx = (2.0f * bx / (float)(uint32_t)kp.width - 1.0f) / kp.proj11;
    const float vy = (1.0f - 2.0f * by / (float)(uint32_t)kp.height) / kp.proj22;
    const float vz = -1.0f;
    V3 w;
    w.x = kp.right[0] * vx + kp.up[0] * vy - kp.fwd[0] * vz;
    w.y = kp.right[1] * vx + kp.up[1] * vy - kp.fwd[1] * vz;
    w.z = kp.right[2] * vx + kp.up[2] * vy - kp.fwd[2] * vz;
    o = v3(w.x + kp.eye[0], w.y + kp.eye[1], w.z + kp.eye[2]);
    normalize_hlsl(w);   // rtx.hlsl:395 (|w| >= 1 here, so the same as the guarded form)
    dir = w;
}
__device__ __forceinline__ void primary_ray_qe(const KernelParams& kp, uint32_t pix, int px, int py, uint32_t s,
                                               uint32_t& sd, V3& o, V3& dir) {
    sd = tea16(pix, kp.key + kp.spp_offset + s);
    primary_ray_qe_sd(kp, px, py, sd, o, dir);
}
// RNG seed of sample s of pixel pix: rng_init (CV) or the TEA-16 state (QE)
__device__ __forceinline__ uint32_t path_seed(const KernelParams& kp, uint32_t pix, uint32_t s) {
    return kp.mode == kModeQE ? tea16(pix, kp.key + kp.spp_offset + s) : rng_init(pix, kp.key, kp.spp_offset + s);
}
// Russian roulette from bounce `depth` on (rtx.hlsl:314-325); false = path dies
__device__ __forceinline__ bool qe_roulette(uint32_t& sd, V3& color) {
    const float illum = fmaxf(fmaxf(color.x, color.y), color.z);
    if (illum > rng_next(sd)) {
        color = vdiv(color, illum);
        return true;
    }
    return false;
}
// gamma-space running mean (rtx.hlsl:401-402)
__device__ __forceinline__ float qe_blend(float old, float c, uint32_t prev) {
    if (prev == 0) return pow_f(c, kQeInvGamma);
    const float pc = (float)prev, pc1 = (float)(prev + 1u);
    return pow_f((pow_f(old, kQeGamma) * pc + c) / pc1, kQeInvGamma);
}

}  // namespace trace
}  // namespace mcpt
