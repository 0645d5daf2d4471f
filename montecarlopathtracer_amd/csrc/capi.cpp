// capi.cpp -- implementation of the C ABI declared in include/mcpt.h.
//
// Host side of the reference's PW::Tracer module (CVMCTracer/CUDA/CUTracer.cu:
// 220-404): device selection, scene upload (CreateGeometry), teardown
// (DestroyGeometry, here freeing exactly what was allocated) and the render
// entry (RenderScene).  Unlike the reference, no module globals hold the scene:
// every call takes the opaque handle it works on.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>   // types and prototypes only: librccl is loaded on first use (rccl())

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/mcpt.h"
#include "half_box.hpp"
#include "host_model.hpp"
#include "render_launch.hpp"

struct mcpt_model {
    mcpt::ObjModel m;
};

namespace {

thread_local std::string g_err;
// mcpt_init's device list for scenes created later on this thread (empty: the
// current device only)
thread_local std::vector<int> g_devices;
// peer access enabled between every pair of distinct devices of g_devices
thread_local bool g_peer_ok = true;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            throw mcpt::Error{e_ == hipErrorOutOfMemory ? MCPT_E_NOMEM : MCPT_E_DEVICE,   \
                              std::string(#expr) + ": " + hipGetErrorString(e_)};       \
    } while (0)

template <typename F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const mcpt::Error& e) {
        return fail(e.code, e.msg);
    } catch (const std::bad_alloc&) {
        return fail(MCPT_E_NOMEM, "out of host memory");
    } catch (const std::exception& e) {
        return fail(MCPT_E_INVALID, e.what());
    }
}

uint32_t tea16(uint32_t v0, uint32_t v1) {   // MCRT/QuinEngine/Shader/rtx.hlsl:61-72
    uint32_t sum = 0;
    for (int n = 0; n < 16; n++) {
        sum += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + sum) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    return v0;
}

struct Vf {
    float x, y, z;
};
// Math::Vector3f::normal()/cross() (CVMCTracer/Framework/Math.hpp:112-123)
Vf normal_of(Vf v) {
    float len = std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
    float d = std::fmax(len, FLT_MIN);
    return Vf{v.x / d, v.y / d, v.z / d};
}
Vf cross_of(Vf a, Vf b) { return Vf{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }

struct Workspace {
    void* partial = nullptr;
    size_t partial_bytes = 0;
    void* small = nullptr;       // counter (16 B) + stats (64 B)
    void* spill = nullptr;
    size_t spill_bytes = 0;
    void* fb = nullptr;          // mcpt_render staging framebuffer
    size_t fb_bytes = 0;
    void* wf = nullptr;          // wavefront queues / path state (one allocation)
    size_t wf_bytes = 0;
    void* tail = nullptr;        // megakernel tail split: one float4 per tail sample
    size_t tail_bytes = 0;
};

struct Timing {
    hipEvent_t e[3];
};

// Restores the calling thread's current HIP device on every exit path
struct DeviceGuard {
    int prev = -1;
    DeviceGuard() { (void)hipGetDevice(&prev); }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// RCCL, resolved from librccl at the first render that asks for its gather
// (mcpt_render_params::gather): libmcpt itself does not depend on it, so it
// loads where RCCL is absent and a one-process renderer that never asks pays
// nothing for it.
struct Rccl {
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGather) gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string load_error;
};
const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            x.load_error = std::string("cannot load librccl: ") + (e ? e : "?");
            return x;
        }
        x.comm_init_all = reinterpret_cast<decltype(&ncclCommInitAll)>(dlsym(h, "ncclCommInitAll"));
        x.comm_destroy = reinterpret_cast<decltype(&ncclCommDestroy)>(dlsym(h, "ncclCommDestroy"));
        x.gather = reinterpret_cast<decltype(&ncclGather)>(dlsym(h, "ncclGather"));
        x.group_start = reinterpret_cast<decltype(&ncclGroupStart)>(dlsym(h, "ncclGroupStart"));
        x.group_end = reinterpret_cast<decltype(&ncclGroupEnd)>(dlsym(h, "ncclGroupEnd"));
        x.error_string = reinterpret_cast<decltype(&ncclGetErrorString)>(dlsym(h, "ncclGetErrorString"));
        if (!x.comm_init_all || !x.comm_destroy || !x.gather || !x.group_start || !x.group_end || !x.error_string)
            x.load_error = "librccl lacks ncclCommInitAll / ncclGather / ncclGroupStart / ncclGroupEnd";
        return x;
    }();
    return r;
}

#define NCCL_TRY(expr)                                                                                  \
    do {                                                                                                \
        ncclResult_t r_ = (expr);                                                                       \
        if (r_ != ncclSuccess)                                                                          \
            throw mcpt::Error{MCPT_E_DEVICE, std::string(#expr) + ": " + rccl().error_string(r_)};   \
    } while (0)

}  // namespace

struct mcpt_scene {
    mcpt::HostScene hs;
    bool on_device = false;
    int device = -1;
    int cus = 0;
    std::vector<unsigned char> image;   // host copy of the device image
    std::vector<uint32_t> tri_order;    // image triangle slot -> kd id
    mcpt::GpuScene gpu{};
    void* d_image = nullptr;
    void* d_normals = nullptr;
    Workspace ws;
    std::vector<Timing> pending, free_timing;
    // events of renders captured into a graph: recorded by the graph's replays,
    // never read (a captured render has no time of its own) nor recycled
    // (created once, mcpt_scene_reserve)
    Timing capture_timing{};
    bool has_capture_timing = false;
    int last_variant = 0;
    uint64_t renders = 0;
    // wavefront queue bytes set aside by mcpt_scene_reserve: later renders with a
    // default batch never grow past them (no hipMalloc inside a stream capture)
    size_t wf_reserved = 0;
    // set by mcpt_scene_reserve: from then on a workspace buffer that has to grow
    // is retired (kept until the scene is destroyed), never freed, so a HIP graph
    // captured against the reservation keeps valid pointers (grow_ws)
    bool reserved = false;
    std::vector<void*> retired;
    // multi-device scene (mcpt_init with n > 1): the primary (this object, on
    // devices[0]) owns one replica per further device -- the same image and
    // normals, its own workspace, a non-blocking stream and a completion event --
    // and the gather buffer its shards are peer-copied into
    std::vector<std::unique_ptr<mcpt_scene>> replicas;
    hipStream_t stream = nullptr;       // replicas: the shard's stream
    hipEvent_t done = nullptr;          // replicas: shard rendered and copied
    hipEvent_t start = nullptr;         // primary: inputs ready on the caller's stream
    void* gather = nullptr;
    size_t gather_bytes = 0;
    // wavefront: a second stream for every other batch, forked from and joined
    // back into the caller's stream (created on first use)
    hipStream_t wf_stream[mcpt::kMaxWfStreams] = {};   // [0] unused (the caller's)
    hipEvent_t wf_fork = nullptr, wf_join[mcpt::kMaxWfStreams] = {};
    bool peer_access = true;            // multi-device: peer access enabled between every device pair
    // multi-device, gather = RCCL: one communicator per device of the list
    // (ncclCommInitAll, rank r = device r of the list) and rank 0's send buffer
    std::vector<ncclComm_t> comms;
    void* gather_send = nullptr;
    size_t gather_send_bytes = 0;

    ~mcpt_scene() {
        if (!on_device) return;
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(device);
        (void)hipDeviceSynchronize();
        if (!comms.empty()) {               // no collective in flight on any device, then the comms
            for (auto& R : replicas) {
                (void)hipSetDevice(R->device);
                (void)hipDeviceSynchronize();
            }
            for (ncclComm_t c : comms) (void)rccl().comm_destroy(c);
            (void)hipSetDevice(device);
        }
        for (void* p : {d_image, d_normals, ws.partial, ws.small, ws.spill, ws.fb, ws.wf, ws.tail, gather, gather_send})
            if (p) (void)hipFree(p);
        for (void* p : retired) (void)hipFree(p);
        for (auto& t : pending) for (auto ev : t.e) (void)hipEventDestroy(ev);
        for (auto& t : free_timing) for (auto ev : t.e) (void)hipEventDestroy(ev);
        if (has_capture_timing) for (auto ev : capture_timing.e) (void)hipEventDestroy(ev);
        for (hipEvent_t ev : {done, start, wf_fork})
            if (ev) (void)hipEventDestroy(ev);
        for (int i = 0; i < mcpt::kMaxWfStreams; i++) {
            if (wf_join[i]) (void)hipEventDestroy(wf_join[i]);
            if (wf_stream[i]) (void)hipStreamDestroy(wf_stream[i]);
        }
        if (stream) (void)hipStreamDestroy(stream);
        replicas.clear();                 // each replica frees on its own device
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

namespace {

// Device node order: treelet clusters.  A cluster holds the sibling pairs of
// the 3 levels below its root (<= 7 pairs) contiguously, so a descent through
// those levels stays within 112 B (16-B pairs, LDS scenes) or 336 B (48-B
// pair records with child boxes, global-memory scenes); clusters are emitted
// breadth-first (the top of the tree comes first).  Slot 0 is padding and
// slot 1 the root.  Triangles and leaf references are renumbered in the order
// the leaves appear, so a leaf's triangles sit near its neighbours'.  Only
// addresses change: traversal order, results and counters are those of the
// BFS tree.
struct DeviceOrder {
    std::vector<uint32_t> node_new;     // host node -> device node index
    uint32_t n_slots = 0;               // device node indices in use (incl. padding)
    std::vector<uint32_t> leaf_order;   // host leaf nodes in device order
    std::vector<uint32_t> tri_order;    // device triangle slot -> kd id
    std::vector<uint32_t> tri_new;      // kd id -> device triangle slot
};

// leaves in device node order, triangles by first appearance
void order_leaves(const mcpt::HostScene& hs, DeviceOrder& d) {
    const uint32_t nn = static_cast<uint32_t>(hs.nodes.size());
    std::vector<uint32_t> by_dev(d.n_slots, 0xFFFFFFFFu);
    for (uint32_t i = 0; i < nn; ++i) by_dev[d.node_new[i]] = i;
    d.tri_new.assign(hs.kd_tris.size(), 0xFFFFFFFFu);
    for (uint32_t dv = 0; dv < d.n_slots; ++dv) {
        const uint32_t i = by_dev[dv];
        if (i == 0xFFFFFFFFu || hs.nodes[i].axis) continue;
        d.leaf_order.push_back(i);
        for (uint32_t r = 0; r < hs.nodes[i].leaf_count; ++r) {
            const uint32_t k = hs.leaf_ids[hs.nodes[i].leaf_begin + r];
            if (d.tri_new[k] == 0xFFFFFFFFu) {
                d.tri_new[k] = static_cast<uint32_t>(d.tri_order.size());
                d.tri_order.push_back(k);
            }
        }
    }
    for (uint32_t k = 0; k < d.tri_new.size(); ++k)
        if (d.tri_new[k] == 0xFFFFFFFFu) {
            d.tri_new[k] = static_cast<uint32_t>(d.tri_order.size());
            d.tri_order.push_back(k);
        }
}

DeviceOrder device_order(const mcpt::HostScene& hs) {
    const uint32_t nn = static_cast<uint32_t>(hs.nodes.size());
    DeviceOrder d;
    d.node_new.assign(nn, 0xFFFFFFFFu);
    d.node_new[0] = 0;
    uint32_t pairs = 0;                  // pair m occupies device nodes 2m+1, 2m+2 (slots 2m+2, 2m+3)
    std::vector<uint32_t> queue{0}, list, frontier, next;
    for (size_t qi = 0; qi < queue.size(); ++qi) {
        list.clear();
        frontier.assign(1, queue[qi]);
        for (int lvl = 0; lvl < 3; ++lvl) {
            next.clear();
            for (uint32_t n : frontier)
                if (hs.nodes[n].axis) {
                    list.push_back(hs.nodes[n].left);
                    next.push_back(hs.nodes[n].left);
                    next.push_back(hs.nodes[n].left + 1);
                }
            frontier.swap(next);
        }
        for (uint32_t n : frontier)
            if (hs.nodes[n].axis) queue.push_back(n);
        if (list.empty()) continue;
        for (uint32_t L : list) {
            d.node_new[L] = 2 * pairs + 1;
            d.node_new[L + 1] = 2 * pairs + 2;
            ++pairs;
        }
    }
    d.n_slots = 2 * pairs + 1;
    order_leaves(hs, d);
    return d;
}

void build_image(mcpt_scene& s, bool force_global) {
    const mcpt::HostScene& hs = s.hs;
    const uint32_t nt = static_cast<uint32_t>(hs.kd_tris.size());
    const uint32_t nn = static_cast<uint32_t>(hs.nodes.size());
    const uint32_t nl = static_cast<uint32_t>(hs.leaf_ids.size());
    const uint32_t ng = static_cast<uint32_t>(hs.geoms.size());
    // the traversal's spill area holds 32 stack entries per lane (depth cap 32)
    if (hs.kd_depth < 0 || hs.kd_depth > 32) throw mcpt::Error{MCPT_E_INVALID, "KD tree deeper than 32"};
    for (uint32_t i = 0; i < nn; ++i)
        if (hs.nodes[i].axis && ((hs.nodes[i].left % 2u) != 1u || hs.nodes[i].right != hs.nodes[i].left + 1u ||
                                 hs.nodes[i].left + 1u >= nn || hs.nodes[i].left <= i))
            throw mcpt::Error{MCPT_E_INVALID, "KD sibling pair not at an odd index"};
    auto al16 = [](size_t x) { return (x + 15u) & ~size_t(15); };
    auto al128 = [](size_t x) { return (x + 127u) & ~size_t(127); };
    // Scenes that fit in LDS: 8-B node records in packed cluster order (every
    // LDS byte counts).  Larger scenes: 48-B sibling-pair records -- the two
    // node words plus both children's KD boxes as fp16 rounded outward, so the
    // traversal skips children the ray misses (child-box cull).
    DeviceOrder ord = device_order(hs);
    bool boxes = false;
    auto image_size = [&](const DeviceOrder& o, size_t& on, size_t& ol, size_t& og) {
        on = al128(size_t(nt) * 48);
        if (boxes) ol = al16(on + size_t((o.n_slots - 1) / 2) * 48);   // pair m: device nodes 2m+1, 2m+2
        else ol = al16(on + size_t(o.n_slots + 1) * 8);                 // node slot j = device node j-1
        og = al16(ol + size_t(nl) * 4);
        // (geometries never empty for a scene with triangles; the paired
        // triangle tests read the ref after a leaf's last one, so the leaf
        // section must never end the image)
        return al16(og + size_t(std::max<uint32_t>(ng, 1u)) * 64);
    };
    size_t off_nodes, off_leafs, off_geoms;
    size_t total = image_size(ord, off_nodes, off_leafs, off_geoms);
    if (mcpt::lds_bytes_in_lds(static_cast<uint32_t>(std::min<size_t>(total, 0xFFFFFFF0u)), 4) + 32 > mcpt::kMaxLds ||
        force_global) {
        boxes = true;
        total = image_size(ord, off_nodes, off_leafs, off_geoms);
    }
    const size_t off_tris = 0;
    if (total > 0xFFFFFFF0u) throw mcpt::Error{MCPT_E_UNSUPPORTED, "scene image exceeds 4 GiB"};
    if (ord.n_slots >= (1u << 29) || nl >= (1u << 30)) throw mcpt::Error{MCPT_E_UNSUPPORTED, "KD tree too large"};
    s.image.assign(total, 0);
    s.tri_order = ord.tri_order;
    unsigned char* img = s.image.data();
    for (uint32_t slot = 0; slot < nt; ++slot) {
        const uint32_t k = ord.tri_order[slot];
        const float* v = &hs.kd_verts[9 * size_t(k)];
        float rec[12] = {v[0], v[1], v[2], 0.0f,
                         v[0] - v[3], v[1] - v[4], v[2] - v[5], 0.0f,
                         v[0] - v[6], v[1] - v[7], v[2] - v[8], 0.0f};
        std::memcpy(&rec[3], &hs.kd_prio[k], 4);
        std::memcpy(&rec[7], &hs.kd_geom[k], 4);
        // the 2x2 minor (a-b).y (a-c).z - (a-c).y (a-b).z that Math.hpp:171-173's
        // det() forms for both A and tM (CUTracer.cu:72-83): ray-independent, so
        // stored once (same float operations as the kernel's, no contraction)
        rec[11] = rec[5] * rec[10] - rec[9] * rec[6];
        std::memcpy(img + off_tris + size_t(slot) * 48, rec, 48);
    }
    // leaf references, leaves in device order
    std::vector<uint32_t> leaf_begin_new(nn, 0);
    {
        uint32_t* refs = reinterpret_cast<uint32_t*>(img + off_leafs);
        uint32_t at = 0;
        for (uint32_t i : ord.leaf_order) {
            leaf_begin_new[i] = at;
            for (uint32_t r = 0; r < hs.nodes[i].leaf_count; ++r)
                refs[at++] = 3u * ord.tri_new[hs.leaf_ids[hs.nodes[i].leaf_begin + r]];   // record index
        }
    }
    for (uint32_t i = 0; i < nn; ++i) {
        const mcpt::KdNode& n = hs.nodes[i];
        uint32_t w[2];
        if (n.axis) {
            // LDS layout: the left child's device node index (its 8-B record
            // pair at slot index + 1); global layout: the 16-B offset 3m of the
            // children's 48-B pair record m (no index arithmetic per step)
            const uint32_t dl = ord.node_new[n.left];
            w[0] = ((n.axis - 1u) << 30) | (boxes ? 3u * ((dl - 1u) / 2u) : dl);
            std::memcpy(&w[1], &n.split, 4);
        } else {
            w[0] = (3u << 30) | leaf_begin_new[i];
            w[1] = n.leaf_count;
        }
        const uint32_t dv = ord.node_new[i];
        if (i == 0) {
            s.gpu.root_w[0] = w[0];
            s.gpu.root_w[1] = w[1];
            if (boxes) continue;              // the root has no pair record
        }
        if (!boxes) {
            std::memcpy(img + off_nodes + size_t(dv + 1) * 8, w, 8);
            continue;
        }
        // pair record: [w(left) w(right)] [box(left) box(right)] [pad]; boxes rounded outward
        const size_t m = (dv - 1) / 2, side = (dv - 1) % 2;
        unsigned char* rec = img + off_nodes + m * 48;
        std::memcpy(rec + side * 8, w, 8);
        uint16_t hb[6];
        for (int a = 0; a < 3; ++a) {
            hb[a] = mcpt::f32_to_f16_dir(n.bmin[a], -1);
            hb[3 + a] = mcpt::f32_to_f16_dir(n.bmax[a], +1);
        }
        std::memcpy(rec + 16 + side * 12, hb, 12);
    }
    for (uint32_t g = 0; g < ng; ++g) {
        const mcpt::Geometry& ge = hs.geoms[g];
        mcpt::GpuGeom gg{};
        gg.Ka[0] = ge.Ka.x; gg.Ka[1] = ge.Ka.y; gg.Ka[2] = ge.Ka.z;
        gg.Kd[0] = ge.Kd.x; gg.Kd[1] = ge.Kd.y; gg.Kd[2] = ge.Kd.z;
        gg.Ks[0] = ge.Ks.x; gg.Ks[1] = ge.Ks.y; gg.Ks[2] = ge.Ks.z;
        gg.Ns = ge.Ns; gg.Tr = ge.Tr; gg.Ni = ge.Ni;
        gg.Ns_u = ge.Ns > 0.0f ? (ge.Ns < 4294967040.0f ? static_cast<uint32_t>(ge.Ns) : 0xFFFFFF00u) : 0u;
        std::memcpy(img + off_geoms + size_t(g) * 64, &gg, 64);
    }
    mcpt::GpuScene& gs = s.gpu;
    gs.image_bytes = static_cast<uint32_t>(total);
    gs.off_tris = static_cast<uint32_t>(off_tris);
    gs.off_nodes = static_cast<uint32_t>(off_nodes);
    gs.off_leafs = static_cast<uint32_t>(off_leafs);
    gs.off_geoms = static_cast<uint32_t>(off_geoms);
    gs.node_boxes = boxes ? 1u : 0u;
    gs.n_tris = nt; gs.n_nodes = nn; gs.n_leafs = nl; gs.n_geoms = ng;
    if (nn) {
        for (int a = 0; a < 3; ++a) { gs.root_min[a] = hs.nodes[0].bmin[a]; gs.root_max[a] = hs.nodes[0].bmax[a]; }
    }
}

void ensure_buf(void*& p, size_t& have, size_t need) {
    if (have >= need && p) return;
    if (p) HIP_TRY(hipFree(p));
    p = nullptr;
    have = 0;
    HIP_TRY(hipMalloc(&p, need ? need : 16));
    have = need;
}

// A workspace buffer of scene s grown to `need` bytes.  Once the scene has been
// reserved (mcpt_scene_reserve), the old buffer is retired instead of freed --
// a HIP graph captured against it keeps valid memory (its replays use the old
// buffers, later renders the new ones) -- and on a capturing stream nothing is
// allocated at all: a captured render that needs more than the scene holds
// fails with MCPT_E_NOMEM before any launch (reserve for its params first).
void grow_ws(mcpt_scene& s, void*& p, size_t& have, size_t need, bool capturing) {
    if (have >= need && p) return;
    if (capturing)
        throw mcpt::Error{MCPT_E_NOMEM, "render needs more workspace than the scene holds while its stream is "
                                        "capturing a graph: call mcpt_scene_reserve with these params first"};
    if (p && s.reserved) {
        s.retired.push_back(p);
        p = nullptr;
        have = 0;
    }
    ensure_buf(p, have, need);
}

struct Plan {
    mcpt::KernelParams kp;
    size_t out_pixels;
    bool capturing = false;      // the render's stream is capturing a graph: nothing may be allocated
    int pipeline;
    int wf_streams;              // wavefront streams (wavefront_streams)
    uint32_t wf_capacity;        // paths per wavefront batch
    bool wf_batch_explicit;      // the caller asked for this batch (not shrunk to fit memory)
    int32_t wf_sort;             // wavefront material sort (mcpt_render_params::wf_sort)
    int32_t wf_refill;           // idle lanes before an extend wave refills
    uint32_t wf_group_shift;     // global-memory scenes: paths dealt to segments in groups of 2^k
    int64_t tail_per_lane;       // megakernel tail split: units per lane (< 0 off)
    int64_t tail_exact;          // megakernel tail split: exact units (> 0 overrides)
    uint64_t wf_mem_limit;       // mcpt_render_params::wf_mem_limit
    uint64_t work;               // paths of the render
};

int clamp_i(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// wavefront streams: 2-3 for scenes in LDS, 4 for scenes in global memory (C2
// 1024 spp, streams x batch: 2 x 2^27 11.48, 2 x 2^26 11.46, 4 x 2^27 11.52,
// 4 x 2^26 10.93; C4 1024 spp: 1 x 2^28 6.14, 2 x 2^28 8.07, 3 x 2^27 8.17,
// 4 x 2^27 8.28 G rays/s, means of 2-3 runs).  mcpt_render_params::wf_streams
// (1..4) overrides; 1 = every batch on the caller's stream.
// LDS scenes: 3 streams for frames of more than 2^29 paths (C2 after the
// id-only hit records: 2 x 2^28 13.48 / 13.45, 3 x 2^27 13.65 / 13.56,
// 3 x 2^30/9 13.65 / 13.59 G rays/s), 2 up to 2^29 (one rank's C2 share at
// N = 2, 2^29 paths: 136.1 ms on 2 x 2^27, 136.7 on 2 x 2^28, 143.3 on
// 3 x 2^27 -- four batches on three streams leave one alone at the end; at
// N = 8, 2^27 paths: 35.4 ms on 2 streams, 37.6 on 3)
int wavefront_streams(const mcpt_scene& s, uint64_t work, const mcpt_render_params* p) {
    const int n = p->wf_streams > 0 ? p->wf_streams
                                    : (s.gpu.node_boxes ? 4 : (work > (uint64_t(1) << 29) ? 3 : 2));
    return clamp_i(n, 1, mcpt::kMaxWfStreams);
}

// Device memory of one stream's wavefront workspace for batches of `cap`
// paths (prepare_wavefront carves it): two ray queues, radiance, per-bounce
// counters.  A queue is three float4 streams (origin + path id, direction +
// depth, throughput + RNG state) and the hit stream of 4-B triangle ids
// (wavefront.hip kQHIT): 3 x 16 + 4 B per slot and queue, 120 B per path with
// the radiance (the material sort too: it sorts in LDS).  Segments hold
// whole path groups (2^group_shift paths: 64 for LDS scenes, up to 2^14 for
// global-memory ones): up to one group of slots per segment beyond the paths.
struct WfLayout {
    size_t cap_slots, f4, queue, need;
};
WfLayout wf_layout(const mcpt_scene& s, const Plan& pl, uint64_t cap) {
    const mcpt::KernelParams& kp = pl.kp;
    const size_t nseg = static_cast<size_t>(mcpt::wavefront_segments(s.gpu, s.cus));
    const size_t queries = kp.mode == MCPT_MODE_QUINENGINE ? 3 * size_t(kp.max_depth) + 1 : size_t(kp.max_depth) + 1;
    const size_t bounces = (queries + 1) * nseg;
    auto al256 = [](size_t x) { return (x + 255) & ~size_t(255); };
    WfLayout l;
    l.cap_slots = size_t(cap) + (nseg << pl.wf_group_shift);
    l.f4 = l.cap_slots * 16;
    l.queue = al256(3 * l.f4 + 4 * l.cap_slots);
    l.need = al256(2 * l.queue + l.f4 + bounces * sizeof(mcpt::WfCounters) + 256);
    return l;
}

Plan make_plan(const mcpt_scene& s, const mcpt_render_params* p) {
    if (!p) throw mcpt::Error{MCPT_E_INVALID, "params is NULL"};
    if (p->width <= 0 || p->height <= 0) throw mcpt::Error{MCPT_E_INVALID, "width/height must be positive"};
    if (p->spp == 0) throw mcpt::Error{MCPT_E_INVALID, "spp must be > 0"};
    if (p->max_depth < 0 || p->max_depth > 1000) throw mcpt::Error{MCPT_E_INVALID, "max_depth out of range"};
    if (p->wf_streams < 0 || p->wf_streams > mcpt::kMaxWfStreams)
        throw mcpt::Error{MCPT_E_INVALID, "wf_streams must be 0 (automatic) or 1..4"};
    if (p->wf_refill < 0 || p->wf_refill > 64 || p->ready_thresh < 0 || p->ready_thresh > 64)
        throw mcpt::Error{MCPT_E_INVALID, "wf_refill / ready_thresh must be 0 (automatic) or 1..64"};
    if (p->wf_group_shift != 0 && (p->wf_group_shift < 6 || p->wf_group_shift > 14))
        throw mcpt::Error{MCPT_E_INVALID, "wf_group_shift must be 0 (automatic) or 6..14"};
    if (p->tail_units < 0) throw mcpt::Error{MCPT_E_INVALID, "tail_units must be >= 0"};
    // (every render path, one device or several, rejects an unknown gather)
    if (p->gather != MCPT_GATHER_PEER && p->gather != MCPT_GATHER_RCCL)
        throw mcpt::Error{MCPT_E_INVALID, "unknown gather"};
    const int T = p->tile > 0 ? p->tile : 8;
    if (T > 256) throw mcpt::Error{MCPT_E_INVALID, "tile too large"};
    const int sc = p->shard_count > 1 ? p->shard_count : 1;
    const int si = sc > 1 ? p->shard_index : 0;
    if (si < 0 || si >= sc) throw mcpt::Error{MCPT_E_INVALID, "shard_index out of range"};
    const uint64_t tiles_x = (uint64_t(p->width) + T - 1) / T, tiles_y = (uint64_t(p->height) + T - 1) / T;
    const uint64_t ntiles = tiles_x * tiles_y;
    const uint64_t owned = uint64_t(si) < ntiles ? (ntiles - uint64_t(si) + uint64_t(sc) - 1) / uint64_t(sc) : 0;
    const uint64_t npix = owned * uint64_t(T) * uint64_t(T);
    const uint32_t chunk = p->spp_chunk ? (p->spp_chunk < p->spp ? p->spp_chunk : p->spp) : p->spp;
    const uint64_t nchunks = (uint64_t(p->spp) + chunk - 1) / chunk;
    if (npix * nchunks >= 0xFFFFFFFFull) throw mcpt::Error{MCPT_E_UNSUPPORTED, "too many work units for one call"};

    Plan pl;
    mcpt::KernelParams& k = pl.kp;
    std::memset(&k, 0, sizeof k);
    k.scene = s.gpu;
    k.width = p->width; k.height = p->height;
    k.tile = T; k.tiles_x = static_cast<int32_t>(tiles_x);
    k.shard_count = sc; k.shard_index = si;
    k.packed = (p->packed || sc > 1) ? 1 : 0;
    k.npix_local = static_cast<uint32_t>(npix);
    k.spp = p->spp; k.spp_offset = p->spp_offset; k.chunk = chunk;
    k.nchunks = static_cast<uint32_t>(nchunks);
    k.total_units = static_cast<uint32_t>(npix * nchunks);
    k.div_npix = mcpt::FastDiv::make(std::max<uint32_t>(k.npix_local, 1));
    k.div_tt = mcpt::FastDiv::make(static_cast<uint32_t>(T * T));
    k.div_tiles_x = mcpt::FastDiv::make(static_cast<uint32_t>(tiles_x));
    k.div_tile = mcpt::FastDiv::make(static_cast<uint32_t>(T));
    k.div_chunk = mcpt::FastDiv::make(chunk);
    k.tail_units = k.total_units;         // no tail split unless prepare_workspace sets one
    k.total_items = k.total_units;
    k.max_depth = p->max_depth;
    k.lean = p->lean ? 1 : 0;
    k.illum = p->illum;
    const float a = p->fov_deg * 3.14159265359f / 360;   // CUTracer.cu:189,202
    k.tan_half_fov = static_cast<float>(std::tan(static_cast<double>(a)));
    k.h_over_w = 1.0 * static_cast<double>(static_cast<uint32_t>(p->height)) / static_cast<double>(static_cast<uint32_t>(p->width));
    k.inv_w_pow2 = (p->width > 0 && (p->width & (p->width - 1)) == 0) ? 1.0 / static_cast<double>(p->width) : 0.0;
    k.fresnel_kd = p->fresnel_kd ? 1 : 0;
    k.prev_count = p->prev_count;
    // camera basis (CUTracer.cu:349-359)
    Vf d = normal_of(Vf{p->dir[0], p->dir[1], p->dir[2]});
    Vf r = normal_of(cross_of(d, Vf{p->up[0], p->up[1], p->up[2]}));
    Vf u = normal_of(cross_of(r, d));
    for (int i = 0; i < 3; ++i) k.eye[i] = p->eye[i];
    k.fwd[0] = d.x; k.fwd[1] = d.y; k.fwd[2] = d.z;
    k.up[0] = u.x; k.up[1] = u.y; k.up[2] = u.z;
    k.right[0] = r.x; k.right[1] = r.y; k.right[2] = r.z;
    if (p->mode != MCPT_MODE_CVMCTRACER && p->mode != MCPT_MODE_QUINENGINE)
        throw mcpt::Error{MCPT_E_INVALID, "unknown mode"};
    k.mode = p->mode;
    k.best_init = FLT_MAX;
    if (p->mode == MCPT_MODE_QUINENGINE) {
        // rtx.hlsl:380 seeds TEA-16 with the 32-bit frame seed itself; t_best 10000 (:88);
        // camera GraphicsRTX.cpp:173-184 (PerspectiveFovRH: fov_deg is the vertical FOV)
        k.key = static_cast<uint32_t>(p->seed);
        k.best_init = 10000.0f;
        const float a = p->fov_deg * 3.14159265359f / 360;
        const float ys = static_cast<float>(1.0 / std::tan(static_cast<double>(a)));
        k.proj22 = ys;
        k.proj11 = ys / (static_cast<float>(p->width) / static_cast<float>(p->height));
    } else {
        k.key = tea16(static_cast<uint32_t>(p->seed), static_cast<uint32_t>(p->seed >> 32));
    }
    // lanes ready before a shading round: scenes in LDS 32 (sweep 16..48);
    // scenes in global memory 40 (C4: 24 5.15, 32 5.38, 40 5.50, 48 5.39 G rays/s)
    k.ready_thresh = p->ready_thresh > 0 ? p->ready_thresh : (s.gpu.node_boxes == 1 ? 40 : 32);
    pl.out_pixels = k.packed ? size_t(npix) : size_t(p->width) * size_t(p->height);
    if (p->pipeline != MCPT_PIPELINE_MEGAKERNEL && p->pipeline != MCPT_PIPELINE_WAVEFRONT)
        throw mcpt::Error{MCPT_E_INVALID, "unknown pipeline"};
    pl.pipeline = p->pipeline;
    pl.wf_sort = p->wf_sort ? 1 : 0;
    // idle lanes before an extend wave refills: 16 for scenes in LDS (C2 sweep
    // 8 / 16 / 24: 10.08 / 10.28 / 10.19 G rays/s), 8 for scenes in global
    // memory (C4 256 spp, 2..40: 6.18 / 6.20 (4-12) / 6.14 (16) / 5.79 (32) / 5.53)
    pl.wf_refill = p->wf_refill > 0 ? p->wf_refill : (s.gpu.node_boxes ? 8 : 16);
    // global-memory scenes keep whole image regions together per segment.
    // Round 4 (XCD-aware dealing, 7-entry stacks; C4 1024 spp, G rays/s):
    // 2^8 9.36, 2^9 8.39, 2^10 7.92 / 7.86, 2^11 9.70 / 9.73, 2^12 9.96 / 9.96 /
    // 9.98, 2^13 9.74, 2^14 9.83 / 9.87 / 9.85 (round 1, 256 spp: 2^14 best)
    pl.wf_group_shift = s.gpu.node_boxes ? static_cast<uint32_t>(p->wf_group_shift > 0 ? p->wf_group_shift : 12) : 6u;
    // tail split: 4 units per lane (a whole frame +0.3% over 6; rank 0 of 8
    // shards at 97.0% of ideal, 6: 96.5%, 8: 95.7%, 10: 94.8%)
    pl.tail_per_lane = p->tail_units_per_lane == 0 ? 4 : p->tail_units_per_lane;
    pl.tail_exact = p->tail_units;
    pl.wf_mem_limit = p->wf_mem_limit;
    {
        // default batch: big (120 B of queues per path and stream; fewer launches,
        // shorter relative tails).  One stream: C2 2^24 5.59, 2^25 6.43, 2^26 7.07,
        // 2^27 7.31, 2^28 7.24; C4 (256 spp) 2^24 2.90, 2^26 3.45, 2^28 4.31 G
        // rays/s.  Global-memory scenes on 4 streams: 2^27 each (see wavefront_streams);
        // LDS scenes on 2 streams: 2^28 each (C2 2 x 2^27 12.90, 2 x 2^28 13.03,
        // 3 x 2^27 13.06, 4 x 2^27 12.55 G rays/s, two rounds each; 86 GB of queues)
        const uint64_t work = std::max<uint64_t>(npix, 1) * std::max<uint64_t>(p->spp, chunk);
        pl.work = npix * p->spp;
        const int nstr = wavefront_streams(s, work, p);
        pl.wf_streams = nstr;
        const bool big = nstr == 1 || (!s.gpu.node_boxes && nstr == 2);
        uint64_t cap = p->wf_batch ? p->wf_batch : (big ? (1u << 28) : (1u << 27));
        // a default batch gives every stream a batch of its own (one rank's C2
        // share at 8 GPUs, 2^27 paths: one 2^27 batch 9.26, two 2^26 12.61, four
        // 2^25 12.13 G rays/s; the megakernel 11.22)
        if (!p->wf_batch && nstr > 1) cap = std::min<uint64_t>(cap, (work + nstr - 1) / nstr);
        cap = std::max<uint64_t>(cap, chunk);                        // at least one pixel per batch
        cap = std::min<uint64_t>(cap, work);
        cap = std::min<uint64_t>(cap, uint64_t(1) << 28);               // u32 slot arithmetic; 120 B per path
        pl.wf_capacity = static_cast<uint32_t>(cap);
        pl.wf_batch_explicit = p->wf_batch != 0;
    }
    return pl;
}

// Fit the wavefront's queues into device memory: the budget is
// wf_mem_limit, or 90% of what the device has free plus what this scene's
// workspace already holds.  A default batch is halved until every stream's
// queues fit (never below one pixel's chunk); an explicit batch that does not
// fit is an error, not a failed hipMalloc half-way through a render.  A scene
// reserved with mcpt_scene_reserve fits a default batch into its reservation
// (nothing is re-allocated inside a stream capture); if even the smallest
// batch does not fit there (a reservation made for a smaller render), the
// render grows the workspace from free memory like an unreserved scene --
// except on a capturing stream, where that would allocate, so it fails.
bool stream_capturing(hipStream_t st) {
    if (!st) return false;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing(st, &cs));
    return cs != hipStreamCaptureStatusNone;
}
void fit_wavefront(const mcpt_scene& s, Plan& pl) {
    if (pl.pipeline != MCPT_PIPELINE_WAVEFRONT) return;
    uint64_t budget = pl.wf_mem_limit;
    bool reserved = false;
    if (!budget) {
        size_t fr = 0, tot = 0;
        HIP_TRY(hipMemGetInfo(&fr, &tot));
        // what prepare_workspace will still allocate beside the queues (partial
        // sums, stack spill areas) comes out of the same free memory
        const mcpt::KernelParams& k = pl.kp;
        const size_t lanes = static_cast<size_t>(mcpt::total_lanes_for(s.gpu.image_bytes, s.cus));
        const size_t partial = size_t(k.nchunks) * k.npix_local * 16, spill = size_t(pl.wf_streams) * 32 * lanes * 16;
        const double others = double(partial > s.ws.partial_bytes ? partial - s.ws.partial_bytes : 0) +
                              double(spill > s.ws.spill_bytes ? spill - s.ws.spill_bytes : 0);
        const double avail = (static_cast<double>(fr) + static_cast<double>(s.ws.wf_bytes)) * 0.9 - others;
        budget = avail > 0 ? static_cast<uint64_t>(avail) : 0;
        reserved = s.wf_reserved && !pl.wf_batch_explicit;
    }
    auto need = [&](uint64_t cap) { return uint64_t(wf_layout(s, pl, cap).need) * uint64_t(pl.wf_streams); };
    auto fit = [&](uint64_t b) {
        uint64_t cap = pl.wf_capacity;
        if (!pl.wf_batch_explicit)
            while (need(cap) > b && cap / 2 >= pl.kp.chunk && cap > (uint64_t(1) << 16)) cap /= 2;
        return cap;
    };
    uint64_t cap = fit(reserved ? std::min<uint64_t>(budget, s.wf_reserved) : budget);
    if (reserved && need(cap) > s.wf_reserved) {
        if (pl.capturing) budget = std::min<uint64_t>(budget, s.wf_reserved);
        else cap = fit(budget);
    }
    if (need(cap) > budget) {
        char msg[256];
        std::snprintf(msg, sizeof msg,
                      "wavefront queues for batches of %llu paths need %.2f GB on %d stream(s); budget %.2f GB "
                      "(wf_mem_limit, the scene's reservation or 90%% of free device memory): lower wf_batch / wf_streams",
                      static_cast<unsigned long long>(cap), need(cap) / 1e9, pl.wf_streams, budget / 1e9);
        throw mcpt::Error{MCPT_E_NOMEM, msg};
    }
    pl.wf_capacity = static_cast<uint32_t>(cap);
}

// tail_split: the megakernel hands the last Plan::tail_per_lane (default 4)
// units per lane of the work-unit order out one sample at a time
// (KernelParams::tail_units).  Without it a lane's last whole unit (32 samples,
// ~3.5 ms) set the kernel's end: at 1024 spp, rank 0 of 8 ran 64.4 ms against
// 55.5 ideal (86%); split 2 / 4 / 6 / 8 / 12 per lane: 92 / 96 / 98 / 97 / 96%,
// 1-GPU frame unchanged (442 -> 440 ms at 6).
uint64_t tail_units_for(const mcpt_scene& s, const Plan& pl) {
    const mcpt::KernelParams& k = pl.kp;
    if (k.chunk <= 1) return 0;
    const uint64_t lanes = static_cast<uint64_t>(mcpt::total_lanes_for(s.gpu.image_bytes, s.cus));
    uint64_t tail = pl.tail_exact > 0 ? static_cast<uint64_t>(pl.tail_exact)
                                      : (pl.tail_per_lane > 0 ? static_cast<uint64_t>(pl.tail_per_lane) * lanes : 0);
    tail = std::min<uint64_t>(tail, k.total_units);
    // item indices and tail slots stay below 2^31
    while (tail && uint64_t(k.total_units - tail) + tail * k.chunk >= (uint64_t(1) << 31)) tail >>= 1;
    return tail;
}

void prepare_workspace(mcpt_scene& s, Plan& pl, bool tail_split = false, int spill_sets = 1) {
    mcpt::KernelParams& k = pl.kp;
    grow_ws(s, s.ws.partial, s.ws.partial_bytes, size_t(k.nchunks) * k.npix_local * 16, pl.capturing);
    if (!s.ws.small) {
        HIP_TRY(hipMalloc(&s.ws.small, 256));
        HIP_TRY(hipMemset(s.ws.small, 0, 256));
    }
    const size_t lanes = static_cast<size_t>(mcpt::total_lanes_for(s.gpu.image_bytes, s.cus));
    // (the wavefront's streams run extends concurrently: one spill area each)
    grow_ws(s, s.ws.spill, s.ws.spill_bytes, size_t(spill_sets) * 32 * lanes * 16, pl.capturing);
    k.partial = static_cast<float4*>(s.ws.partial);
    k.counter = static_cast<uint32_t*>(s.ws.small);
    k.stats = reinterpret_cast<unsigned long long*>(static_cast<char*>(s.ws.small) + 64);
    k.spill = static_cast<uint4*>(s.ws.spill);
    k.tail_units = k.total_units;
    k.total_items = k.total_units;
    k.tail_buf = nullptr;
    if (tail_split) {
        const uint64_t tail = tail_units_for(s, pl);
        if (tail) {
            grow_ws(s, s.ws.tail, s.ws.tail_bytes, size_t(tail) * k.chunk * 16, pl.capturing);
            k.tail_units = k.total_units - static_cast<uint32_t>(tail);
            k.total_items = k.tail_units + static_cast<uint32_t>(tail * k.chunk);
            k.tail_buf = static_cast<float4*>(s.ws.tail);
        }
    }
}

// wavefront workspace: 2 ray queues (o, d float4), hits, 4 class lists,
// path state and radiance, per-bounce counters -- carved from one buffer, once
// per stream (`sets`: batches rotate over the wavefront's streams, each with its own)
void prepare_wavefront(mcpt_scene& s, const Plan& pl, int sets, mcpt::WfParams* out) {
    const WfLayout l = wf_layout(s, pl, pl.wf_capacity);
    grow_ws(s, s.ws.wf, s.ws.wf_bytes, l.need * size_t(sets), pl.capturing);
    // a default-batch render that grew the queues past the reservation: the
    // grown queues are the reservation now (a later captured render of the same
    // params allocates nothing and must not be refused)
    if (s.reserved) s.wf_reserved = std::max(s.wf_reserved, s.ws.wf_bytes);
    for (int h = 0; h < sets; ++h) {
        char* b = static_cast<char*>(s.ws.wf) + size_t(h) * l.need;
        mcpt::WfParams& w = out[h];
        std::memset(&w, 0, sizeof w);
        w.q[0] = reinterpret_cast<float4*>(b); b += l.queue;
        w.q[1] = reinterpret_cast<float4*>(b); b += l.queue;
        w.radiance = reinterpret_cast<float4*>(b); b += l.f4;
        w.cnt = reinterpret_cast<mcpt::WfCounters*>(b);
        w.capacity = pl.wf_capacity;                   // paths per batch (pid range)
        w.slot_stride = static_cast<uint32_t>(l.cap_slots);
        w.refill_thresh = clamp_i(pl.wf_refill, 1, 64);
        w.group_shift = pl.wf_group_shift;
        w.sort = pl.wf_sort;
    }
}

// the wavefront's side streams and their fork / join events (created once per
// scene, outside any stream capture: mcpt_scene_reserve calls this too)
void ensure_wf_streams(mcpt_scene& s, int n) {
    if (n > 1 && !s.wf_fork) HIP_TRY(hipEventCreateWithFlags(&s.wf_fork, hipEventDisableTiming));
    for (int i = 1; i < n; i++) {
        if (!s.wf_stream[i]) HIP_TRY(hipStreamCreateWithFlags(&s.wf_stream[i], hipStreamNonBlocking));
        if (!s.wf_join[i]) HIP_TRY(hipEventCreateWithFlags(&s.wf_join[i], hipEventDisableTiming));
    }
}

void set_device(const mcpt_scene& s) {
    int cur = -1;
    HIP_TRY(hipGetDevice(&cur));
    if (cur != s.device) HIP_TRY(hipSetDevice(s.device));
}

void render_multi(mcpt_scene& s, const mcpt_render_params* p, float* d_fb, hipStream_t st);

bool multi_device(const mcpt_scene& s, const mcpt_render_params* p, const uint32_t* d_unit_counters) {
    // (an RCCL gather also runs for a one-device list: a one-rank communicator)
    return (!s.replicas.empty() || (p && p->gather == MCPT_GATHER_RCCL)) && p && p->shard_count <= 1 && !p->packed &&
           !d_unit_counters;
}

void ensure_capture_timing(mcpt_scene& s) {
    if (s.has_capture_timing) return;
    for (auto& ev : s.capture_timing.e) HIP_TRY(hipEventCreate(&ev));
    s.has_capture_timing = true;
}

void render_async(mcpt_scene& s, const mcpt_render_params* p, float* d_fb, hipStream_t st,
                  uint32_t* d_unit_counters = nullptr, bool raw_mean = false) {
    if (!s.on_device) throw mcpt::Error{MCPT_E_INVALID, "scene was created host-only"};
    if (!d_fb) throw mcpt::Error{MCPT_E_INVALID, "framebuffer is NULL"};
    if (multi_device(s, p, d_unit_counters)) {
        render_multi(s, p, d_fb, st);
        return;
    }
    set_device(s);
    Plan pl = make_plan(s, p);
    pl.capturing = stream_capturing(st);
    fit_wavefront(s, pl);
    pl.kp.raw_mean = raw_mean ? 1 : 0;
    // the tail split hands units out by sample, so per-unit counters need whole units
    const int wf_sets = pl.pipeline == MCPT_PIPELINE_WAVEFRONT ? pl.wf_streams : 1;
    prepare_workspace(s, pl, pl.pipeline == MCPT_PIPELINE_MEGAKERNEL && !d_unit_counters, wf_sets);
    pl.kp.unit_counters = d_unit_counters;
    Timing t;
    if (pl.capturing) {
        ensure_capture_timing(s);
        t = s.capture_timing;
    } else if (!s.free_timing.empty()) {
        t = s.free_timing.back();
        s.free_timing.pop_back();
    } else {
        for (auto& ev : t.e) HIP_TRY(hipEventCreate(&ev));
    }
    if (pl.pipeline == MCPT_PIPELINE_WAVEFRONT) {
        if (d_unit_counters) throw mcpt::Error{MCPT_E_UNSUPPORTED, "unit counters need the megakernel pipeline"};
        mcpt::WfParams wf[mcpt::kMaxWfStreams];
        prepare_wavefront(s, pl, wf_sets, wf);
        mcpt::WfStreams wst{};
        wst.n = wf_sets;
        wst.st[0] = st;
        ensure_wf_streams(s, wf_sets);
        wst.fork = s.wf_fork;
        for (int i = 1; i < wf_sets; i++) {
            wst.st[i] = s.wf_stream[i];
            wst.join[i] = s.wf_join[i];
        }
        const int queries = pl.kp.mode == MCPT_MODE_QUINENGINE ? 3 * pl.kp.max_depth + 1 : pl.kp.max_depth + 1;
        HIP_TRY(mcpt::launch_wavefront(pl.kp, wf, wst, s.cus, queries, t.e[0], t.e[1], t.e[2],
                                       reinterpret_cast<float4*>(d_fb), &s.last_variant));
    } else {
        HIP_TRY(mcpt::launch_render(pl.kp, s.cus, st, t.e[0], t.e[1], t.e[2], reinterpret_cast<float4*>(d_fb),
                                    &s.last_variant));
    }
    if (pl.capturing) return;   // timed and counted when replayed, not now
    s.pending.push_back(t);
    s.renders++;
}

void read_stats(mcpt_scene& s, mcpt_render_stats* out) {
    set_device(s);
    mcpt_render_stats r;
    std::memset(&r, 0, sizeof r);
    double kms = 0, rms = 0;
    for (auto& t : s.pending) {
        HIP_TRY(hipEventSynchronize(t.e[2]));
        float a = 0, b = 0;
        HIP_TRY(hipEventElapsedTime(&a, t.e[0], t.e[1]));
        HIP_TRY(hipEventElapsedTime(&b, t.e[1], t.e[2]));
        kms += a;
        rms += b;
        s.free_timing.push_back(t);
    }
    s.pending.clear();
    if (s.ws.small) {
        unsigned long long st[16];
        HIP_TRY(hipMemcpy(st, static_cast<char*>(s.ws.small) + 64, sizeof st, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemset(static_cast<char*>(s.ws.small) + 64, 0, sizeof st));
        if (st[8] | st[9] | st[10] | st[11])   // diagnostic builds (-DMCPT_PHASE_TIMING) only
            std::fprintf(stderr, "mcpt phase cycles (sum over waves): units %llu trav %llu shade %llu burst_iters %llu "
                         "scatter %llu\n", st[8], st[9], st[10], st[11], st[12]);
#ifdef MCPT_PHASE_TIMING
        {
            unsigned long long lu[6], lw[6];
            mcpt::read_lane_use(lu);
            mcpt::read_lane_use_wf(lw);
            for (int i = 0; i < 6; i++) lu[i] += lw[i];
            std::fprintf(stderr, "mcpt lane use: descent %.3f (%llu wave-iters) triangle %.3f (%llu) burst %.3f (%llu)\n",
                         lu[0] ? double(lu[1]) / (64.0 * lu[0]) : 0.0, lu[0], lu[2] ? double(lu[3]) / (64.0 * lu[2]) : 0.0,
                         lu[2], lu[4] ? double(lu[5]) / (64.0 * lu[4]) : 0.0, lu[4]);
        }
#endif
        r.rays = st[0]; r.paths = st[1]; r.inner_visits = st[2]; r.leaf_visits = st[3];
        r.leaf_refs = st[4]; r.tri_tests = st[5]; r.shades = st[6]; r.stack_spills = st[7];
    }
    r.renders = s.renders;
    r.devices = 1;
    s.renders = 0;
    r.kernel_ms = kms;
    r.reduce_ms = rms;
    r.variant = s.last_variant;
    if (out) *out = r;
}

// Multi-device render (mcpt_init with n > 1; the reference's Initialize(),
// CUTracer.cu:220-223, picked one device): shard r of n = the interleaved tiles
// t with t % n == r (the same partition as the one-process-per-GPU bench),
// rendered by device r into its packed means, peer-copied (xGMI DMA) into the
// primary's gather buffer, then unpermuted there with the running mean.  The
// RNG is keyed per (pixel, sample), so the image is the single-device one bit
// for bit.  Cross-device order: every shard waits for `start` (recorded on the
// caller's stream), the caller's stream waits for every shard's `done`.
// RCCL gather: one communicator per device of the list (ncclCommInitAll,
// rank r = the list's device r), made once per scene
void ensure_comms(mcpt_scene& s) {
    if (!s.comms.empty()) return;
    const Rccl& R = rccl();
    if (!R.load_error.empty()) throw mcpt::Error{MCPT_E_UNSUPPORTED, R.load_error};
    std::vector<int> devs{s.device};
    for (auto& rep : s.replicas) devs.push_back(rep->device);
    std::vector<ncclComm_t> comms(devs.size(), nullptr);
    NCCL_TRY(R.comm_init_all(comms.data(), static_cast<int>(devs.size()), devs.data()));
    s.comms = comms;
}

// packed pixels per shard slot of an n-way multi-device render (>= every shard's count)
uint64_t multi_slot(const Plan& full, const mcpt_render_params* p, int n) {
    const int T = full.kp.tile;
    const uint64_t ntiles = uint64_t(full.kp.tiles_x) * ((uint64_t(p->height) + T - 1) / T);
    return (ntiles + n - 1) / n * uint64_t(T) * uint64_t(T);
}

void render_multi(mcpt_scene& s, const mcpt_render_params* p, float* d_fb, hipStream_t st) {
    DeviceGuard guard;   // an error on a replica's device must not leave that device current
    set_device(s);
    const Plan full = make_plan(s, p);                  // validates p (gather included); row-major output
    const bool use_rccl = p->gather == MCPT_GATHER_RCCL;
    const int n = 1 + static_cast<int>(s.replicas.size());
    const int T = full.kp.tile;
    const uint64_t slot = multi_slot(full, p, n);
    if (slot * n >= (uint64_t(1) << 32)) throw mcpt::Error{MCPT_E_UNSUPPORTED, "image too large"};
    const bool cap = stream_capturing(st);
    grow_ws(s, s.gather, s.gather_bytes, size_t(n) * slot * 16, cap);
    if (use_rccl) {
        ensure_comms(s);
        // every rank sends `slot` pixels (ncclGather's equal counts; the shards'
        // own counts differ by at most one tile): rank 0 from gather_send
        grow_ws(s, s.gather_send, s.gather_send_bytes, size_t(slot) * 16, cap);
    }
    if (!s.start) HIP_TRY(hipEventCreateWithFlags(&s.start, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(s.start, st));
    auto shard = [&](int r) {
        mcpt_render_params pr = *p;
        pr.shard_count = n;
        pr.shard_index = r;
        pr.packed = 1;
        return pr;
    };
    for (int r = 1; r < n; ++r) {
        mcpt_scene& R = *s.replicas[size_t(r - 1)];
        set_device(R);
        const mcpt_render_params pr = shard(r);
        const size_t bytes = size_t(mcpt_shard_pixel_count(&pr)) * 16;
        grow_ws(R, R.ws.fb, R.ws.fb_bytes, use_rccl ? size_t(slot) * 16 : bytes, cap);
        HIP_TRY(hipStreamWaitEvent(R.stream, s.start, 0));
        render_async(R, &pr, static_cast<float*>(R.ws.fb), R.stream, nullptr, true);
        if (use_rccl) continue;                        // gathered below, all ranks in one group
        char* dst = static_cast<char*>(s.gather) + size_t(r) * slot * 16;
        if (R.device == s.device && !p->force_peer_copy)
            HIP_TRY(hipMemcpyAsync(dst, R.ws.fb, bytes, hipMemcpyDeviceToDevice, R.stream));
        else
            HIP_TRY(hipMemcpyPeerAsync(dst, s.device, R.ws.fb, R.device, bytes, R.stream));
        HIP_TRY(hipEventRecord(R.done, R.stream));
    }
    set_device(s);
    const mcpt_render_params p0 = shard(0);
    render_async(s, &p0, static_cast<float*>(use_rccl ? s.gather_send : s.gather), st, nullptr, true);
    if (use_rccl) {
        // ncclGather of every rank's `slot` packed pixels into devices[0]'s
        // gather buffer (rank r at r * slot), each on the stream its shard was
        // rendered on; one group, as one process drives every rank
        const Rccl& R = rccl();
        const size_t count = size_t(slot) * 4;
        NCCL_TRY(R.group_start());
        try {
            for (int r = 0; r < n; ++r) {
                const void* send = r ? s.replicas[size_t(r - 1)]->ws.fb : s.gather_send;
                hipStream_t rs = r ? s.replicas[size_t(r - 1)]->stream : st;
                NCCL_TRY(R.gather(send, r ? nullptr : s.gather, count, ncclFloat32, 0, s.comms[size_t(r)], rs));
            }
        } catch (...) {
            (void)R.group_end();
            throw;
        }
        NCCL_TRY(R.group_end());
        for (auto& rep : s.replicas) {
            set_device(*rep);
            HIP_TRY(hipEventRecord(rep->done, rep->stream));
        }
        set_device(s);
    }
    for (auto& R : s.replicas) HIP_TRY(hipStreamWaitEvent(st, R->done, 0));
    mcpt::GatherParams g{};
    g.src = static_cast<const float4*>(s.gather);
    g.fb = reinterpret_cast<float4*>(d_fb);
    g.slot = static_cast<uint32_t>(slot);
    g.width = p->width; g.height = p->height; g.tile = T; g.tiles_x = full.kp.tiles_x; g.nshards = n;
    g.prev_count = p->prev_count;
    g.mode = p->mode;
    HIP_TRY(mcpt::launch_gather(g, st));
}

// stats of a (multi-device) scene: counters summed over devices; kernel and
// reduce times the slowest device's (the devices run concurrently)
void read_stats_all(mcpt_scene& s, mcpt_render_stats* out) {
    mcpt_render_stats r;
    read_stats(s, &r);
    for (auto& R : s.replicas) {
        mcpt_render_stats q;
        read_stats(*R, &q);
        r.rays += q.rays; r.paths += q.paths; r.inner_visits += q.inner_visits; r.leaf_visits += q.leaf_visits;
        r.leaf_refs += q.leaf_refs; r.tri_tests += q.tri_tests; r.shades += q.shades;
        r.stack_spills += q.stack_spills;
        r.kernel_ms = std::max(r.kernel_ms, q.kernel_ms);
        r.reduce_ms = std::max(r.reduce_ms, q.reduce_ms);
    }
    r.devices = 1 + static_cast<int32_t>(s.replicas.size());
    set_device(s);
    if (out) *out = r;
}

// device copies of the scene image and the shading normals on `device`
void upload(mcpt_scene& s, int device, const std::vector<unsigned char>& image, const std::vector<float>& nrm) {
    HIP_TRY(hipSetDevice(device));
    s.device = device;
    HIP_TRY(hipDeviceGetAttribute(&s.cus, hipDeviceAttributeMultiprocessorCount, s.device));
    s.on_device = true;
    HIP_TRY(hipMalloc(&s.d_image, image.size()));
    HIP_TRY(hipMemcpy(s.d_image, image.data(), image.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&s.d_normals, nrm.size() * 4));
    HIP_TRY(hipMemcpy(s.d_normals, nrm.data(), nrm.size() * 4, hipMemcpyHostToDevice));
    s.gpu.image = static_cast<const unsigned char*>(s.d_image);
    s.gpu.normals = static_cast<const float4*>(s.d_normals);
}

}  // namespace

extern "C" {

int mcpt_abi_version(void) { return MCPT_ABI_VERSION; }

const char* mcpt_last_error(void) { return g_err.c_str(); }

int mcpt_init(const int32_t* devices, int32_t n) {
    return guarded([&]() -> int {
        if (n < 0 || (n > 0 && !devices)) return fail(MCPT_E_INVALID, "bad device list");
        if (n == 0) {                     // the current device, single-device scenes
            g_devices.clear();
            g_peer_ok = true;
            return MCPT_OK;
        }
        int count = 0;
        HIP_TRY(hipGetDeviceCount(&count));
        for (int i = 0; i < n; ++i)
            if (devices[i] < 0 || devices[i] >= count) return fail(MCPT_E_INVALID, "device ordinal out of range");
        // peer access between every pair of distinct listed devices, so the
        // multi-device gather's hipMemcpyPeerAsync is a direct xGMI DMA (without
        // it the runtime stages the copy through host memory); "already
        // enabled" is success, a pair without peer capability keeps the staged copy
        // (the guard restores the caller's device if a HIP call throws mid-loop)
        DeviceGuard guard;
        bool peer_ok = true;
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
                if (devices[i] == devices[j]) continue;
                int can = 0;
                HIP_TRY(hipDeviceCanAccessPeer(&can, devices[i], devices[j]));
                if (!can) {
                    peer_ok = false;
                    continue;
                }
                HIP_TRY(hipSetDevice(devices[i]));
                const hipError_t e = hipDeviceEnablePeerAccess(devices[j], 0);
                if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
                else HIP_TRY(e);
            }
        g_devices.assign(devices, devices + n);
        g_peer_ok = peer_ok;
        guard.prev = devices[0];          // success: devices[0] becomes current
        return MCPT_OK;
    });
}

int mcpt_device_count(int32_t* out) {
    return guarded([&]() -> int {
        if (!out) return fail(MCPT_E_INVALID, "out is NULL");
        int c = 0;
        HIP_TRY(hipGetDeviceCount(&c));
        *out = c;
        return MCPT_OK;
    });
}

void mcpt_render_params_quinengine(mcpt_render_params* p) {
    if (!p) return;
    mcpt_render_params_default(p);
    p->mode = MCPT_MODE_QUINENGINE;
    p->width = 640; p->height = 480;                 // the QE window (QE/Main.cpp:11, GraphicsRTX.hpp:34-35)
    p->spp = 1;                                       // one sample per pixel per frame (rtx.hlsl:373-404)
    p->max_depth = 5;                                 // sampleMC(..., 5) (rtx.hlsl:400)
    p->illum = 1.0f;                                  // no ILLUM factor
    p->fov_deg = 45.0f;                               // D3DX_PI / 4, vertical (GraphicsRTX.cpp:181)
    p->fresnel_kd = 0;                                // rtx.hlsl:345 (commented out)
    p->seed = 0;                                      // frame seed: the caller's mt19937(1234) draw
}

void mcpt_render_params_default(mcpt_render_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof *p);
    p->width = 800; p->height = 600;                 // CV/stdafx.h:41-42
    p->spp = 100;                                     // NUM_SAMPLES_PER_KERNEL
    p->max_depth = 7;                                 // CUTracer.cu:212
    p->illum = 10.0f;                                 // ILLUM
    p->fov_deg = 60.0f;                               // CUTracer.cu:189
    p->eye[0] = 0; p->eye[1] = 5; p->eye[2] = 17;     // scene 1 camera, CUTracer.cu:349-351
    p->dir[0] = 0; p->dir[1] = 0; p->dir[2] = -1;
    p->up[0] = 0; p->up[1] = 1; p->up[2] = 0;
    p->seed = 0x4D435054ull;
    p->fresnel_kd = 1;
    p->tile = 8;
    p->shard_count = 1;
}

int mcpt_model_create(const mcpt_model_desc* d, mcpt_model** out) {
    return guarded([&]() -> int {
        if (!d || !out) return fail(MCPT_E_INVALID, "NULL argument");
        if (d->n_vertices < 1 || d->n_normals < 1 || d->n_triangles < 1 || d->n_materials < 1 || d->n_groups < 0)
            return fail(MCPT_E_INVALID, "arrays must include the dummy element 0");
        if (!d->vertices || !d->normals || !d->triangles || !d->materials ||
            (d->n_groups > 0 && (!d->group_names || !d->group_offsets || !d->group_tris)))
            return fail(MCPT_E_INVALID, "NULL array");
        auto m = std::make_unique<mcpt_model>();
        mcpt::ObjModel& o = m->m;
        o.path = "<memory>";
        o.vertices.resize(size_t(d->n_vertices));
        for (int64_t i = 0; i < d->n_vertices; ++i)
            o.vertices[size_t(i)] = mcpt::Vec3{d->vertices[3 * i], d->vertices[3 * i + 1], d->vertices[3 * i + 2]};
        o.normals.resize(size_t(d->n_normals));
        for (int64_t i = 0; i < d->n_normals; ++i)
            o.normals[size_t(i)] = mcpt::Vec3{d->normals[3 * i], d->normals[3 * i + 1], d->normals[3 * i + 2]};
        o.n_texcoords = 1;
        o.triangles.resize(size_t(d->n_triangles));
        for (int64_t i = 0; i < d->n_triangles; ++i) {
            const int32_t* t = d->triangles + 10 * i;
            auto& dst = o.triangles[size_t(i)];
            for (int j = 0; j < 3; ++j) { dst.v[j] = t[j]; dst.t[j] = t[3 + j]; dst.n[j] = t[6 + j]; }
            dst.material = t[9];
            if (i > 0 && (t[9] < 0 || t[9] >= d->n_materials)) return fail(MCPT_E_INVALID, "material index out of range");
        }
        o.materials.resize(size_t(d->n_materials));
        for (int64_t i = 0; i < d->n_materials; ++i) {
            const double* q = d->materials + 12 * i;
            auto& mt = o.materials[size_t(i)];
            mt.Ka = mcpt::Vec3{float(q[0]), float(q[1]), float(q[2])};
            mt.Kd = mcpt::Vec3{float(q[3]), float(q[4]), float(q[5])};
            mt.Ks = mcpt::Vec3{float(q[6]), float(q[7]), float(q[8])};
            mt.Ns = q[9]; mt.Tr = q[10]; mt.Ni = q[11];
        }
        for (int64_t g = 0; g < d->n_groups; ++g) {
            const int64_t b = d->group_offsets[g], e = d->group_offsets[g + 1];
            if (b < 0 || e < b) return fail(MCPT_E_INVALID, "bad group offsets");
            auto& dst = o.groups[d->group_names[g] ? d->group_names[g] : ""];
            for (int64_t k = b; k < e; ++k) {
                if (d->group_tris[k] < 1 || d->group_tris[k] >= d->n_triangles)
                    return fail(MCPT_E_INVALID, "group triangle index out of range");
                dst.push_back(d->group_tris[k]);
            }
        }
        *out = m.release();
        return MCPT_OK;
    });
}

int mcpt_model_read_obj(const char* path, mcpt_model** out) {
    return guarded([&]() -> int {
        if (!path || !out) return fail(MCPT_E_INVALID, "path/out is NULL");
        auto m = std::make_unique<mcpt_model>();
        mcpt::read_obj(path, m->m);
        *out = m.release();
        return MCPT_OK;
    });
}

int mcpt_model_read_obj_ex(const char* path, int32_t flavor, mcpt_model** out) {
    return guarded([&]() -> int {
        if (!path || !out) return fail(MCPT_E_INVALID, "path/out is NULL");
        if (flavor != MCPT_OBJ_CVMCTRACER && flavor != MCPT_OBJ_TINYOBJ) return fail(MCPT_E_INVALID, "unknown flavor");
        auto m = std::make_unique<mcpt_model>();
        mcpt::read_obj(path, m->m, flavor);
        *out = m.release();
        return MCPT_OK;
    });
}

void mcpt_model_free(mcpt_model* m) { delete m; }

int mcpt_model_get_info(const mcpt_model* m, mcpt_model_info* out) {
    if (!m || !out) return fail(MCPT_E_INVALID, "NULL argument");
    out->n_vertices = static_cast<int64_t>(m->m.vertices.size());
    out->n_normals = static_cast<int64_t>(m->m.normals.size());
    out->n_texcoords = m->m.n_texcoords;
    out->n_triangles = static_cast<int64_t>(m->m.triangles.size());
    out->n_materials = static_cast<int64_t>(m->m.materials.size());
    out->n_groups = static_cast<int64_t>(m->m.groups.size());
    return MCPT_OK;
}

int mcpt_model_copy_vertices(const mcpt_model* m, float* out) {
    if (!m || !out) return fail(MCPT_E_INVALID, "NULL argument");
    for (size_t i = 0; i < m->m.vertices.size(); ++i) {
        out[3 * i] = m->m.vertices[i].x; out[3 * i + 1] = m->m.vertices[i].y; out[3 * i + 2] = m->m.vertices[i].z;
    }
    return MCPT_OK;
}

int mcpt_model_copy_normals(const mcpt_model* m, float* out) {
    if (!m || !out) return fail(MCPT_E_INVALID, "NULL argument");
    for (size_t i = 0; i < m->m.normals.size(); ++i) {
        out[3 * i] = m->m.normals[i].x; out[3 * i + 1] = m->m.normals[i].y; out[3 * i + 2] = m->m.normals[i].z;
    }
    return MCPT_OK;
}

int mcpt_model_copy_triangles(const mcpt_model* m, int32_t* out) {
    if (!m || !out) return fail(MCPT_E_INVALID, "NULL argument");
    for (size_t i = 0; i < m->m.triangles.size(); ++i) {
        const auto& t = m->m.triangles[i];
        for (int j = 0; j < 3; ++j) { out[10 * i + j] = t.v[j]; out[10 * i + 3 + j] = t.t[j]; out[10 * i + 6 + j] = t.n[j]; }
        out[10 * i + 9] = t.material;
    }
    return MCPT_OK;
}

int mcpt_model_copy_materials(const mcpt_model* m, double* out) {
    if (!m || !out) return fail(MCPT_E_INVALID, "NULL argument");
    for (size_t i = 0; i < m->m.materials.size(); ++i) {
        const auto& t = m->m.materials[i];
        double* o = out + 12 * i;
        o[0] = t.Ka.x; o[1] = t.Ka.y; o[2] = t.Ka.z; o[3] = t.Kd.x; o[4] = t.Kd.y; o[5] = t.Kd.z;
        o[6] = t.Ks.x; o[7] = t.Ks.y; o[8] = t.Ks.z; o[9] = t.Ns; o[10] = t.Tr; o[11] = t.Ni;
    }
    return MCPT_OK;
}

int mcpt_model_group(const mcpt_model* m, int64_t g, char* name_buf, int64_t name_cap, int64_t* n, int32_t* tris) {
    if (!m || g < 0 || g >= static_cast<int64_t>(m->m.groups.size())) return fail(MCPT_E_INVALID, "bad group index");
    auto it = m->m.groups.begin();
    std::advance(it, g);
    if (name_buf && name_cap > 0) std::snprintf(name_buf, static_cast<size_t>(name_cap), "%s", it->first.c_str());
    if (n) *n = static_cast<int64_t>(it->second.size());
    if (tris && !it->second.empty()) std::memcpy(tris, it->second.data(), it->second.size() * sizeof(int32_t));
    return MCPT_OK;
}

static int scene_create_impl(const mcpt_model* m, mcpt_scene** out, bool device, const char* kd_cache_dir = nullptr,
                             int32_t* cache_hit = nullptr, int32_t layout = MCPT_LAYOUT_AUTO,
                             int32_t kd_build = MCPT_KD_BUILD_REFERENCE) {
    return guarded([&]() -> int {
        if (!m || !out) return fail(MCPT_E_INVALID, "NULL argument");
        if (kd_build != MCPT_KD_BUILD_REFERENCE && kd_build != MCPT_KD_BUILD_SAH)
            return fail(MCPT_E_INVALID, "unknown kd_build");
        auto s = std::make_unique<mcpt_scene>();
        int hit = 0;
        mcpt::build_host_scene(m->m, s->hs, kd_cache_dir, &hit, kd_build);
        if (cache_hit) *cache_hit = hit;
        if (s->hs.kd_tris.empty()) return fail(MCPT_E_INVALID, "scene has no triangles");
        if (layout != MCPT_LAYOUT_AUTO && layout != MCPT_LAYOUT_GLOBAL) return fail(MCPT_E_INVALID, "unknown layout");
        build_image(*s, layout == MCPT_LAYOUT_GLOBAL);
        if (device) {
            const size_t nt = s->hs.kd_tris.size();
            std::vector<float> nrm(nt * 12, 0.0f);
            for (size_t k = 0; k < nt; ++k)          // image triangle order
                for (int j = 0; j < 3; ++j)
                    for (int c = 0; c < 3; ++c)
                        nrm[12 * k + 4 * j + c] = s->hs.kd_normals[9 * size_t(s->tri_order[k]) + 3 * j + c];
            int cur = 0;
            HIP_TRY(hipGetDevice(&cur));
            const std::vector<int> devs = g_devices.empty() ? std::vector<int>{cur} : g_devices;
            upload(*s, devs[0], s->image, nrm);
            // replicas for the further devices: same image, own workspace and stream
            for (size_t i = 1; i < devs.size(); ++i) {
                auto R = std::make_unique<mcpt_scene>();
                R->gpu = s->gpu;
                upload(*R, devs[i], s->image, nrm);
                HIP_TRY(hipStreamCreateWithFlags(&R->stream, hipStreamNonBlocking));
                HIP_TRY(hipEventCreateWithFlags(&R->done, hipEventDisableTiming));
                s->replicas.push_back(std::move(R));
            }
            HIP_TRY(hipSetDevice(devs[0]));
            s->peer_access = g_peer_ok;
        }
        *out = s.release();
        return MCPT_OK;
    });
}

int mcpt_scene_create(const mcpt_model* m, mcpt_scene** out) { return scene_create_impl(m, out, true); }
int mcpt_scene_create_host(const mcpt_model* m, mcpt_scene** out) { return scene_create_impl(m, out, false); }
int mcpt_scene_create_cached(const mcpt_model* m, const char* kd_cache_dir, int32_t host_only, mcpt_scene** out,
                             int32_t* cache_hit) {
    return scene_create_impl(m, out, host_only == 0, kd_cache_dir, cache_hit);
}
int mcpt_scene_create_ex(const mcpt_model* m, const mcpt_scene_options* o, mcpt_scene** out, int32_t* cache_hit) {
    const mcpt_scene_options d{nullptr, 0, MCPT_LAYOUT_AUTO, MCPT_KD_BUILD_REFERENCE};
    if (!o) o = &d;
    const char* dir = o->kd_cache_dir && o->kd_cache_dir[0] ? o->kd_cache_dir : nullptr;
    return scene_create_impl(m, out, o->host_only == 0, dir, cache_hit, o->layout, o->kd_build);
}

void mcpt_scene_destroy(mcpt_scene* s) { delete s; }

int mcpt_scene_get_info(const mcpt_scene* s, mcpt_scene_info* out) {
    if (!s || !out) return fail(MCPT_E_INVALID, "NULL argument");
    out->n_geometries = static_cast<int64_t>(s->hs.geoms.size());
    out->n_triangles = static_cast<int64_t>(s->hs.kd_tris.size());
    out->n_nodes = static_cast<int64_t>(s->hs.nodes.size());
    out->n_leaf_refs = static_cast<int64_t>(s->hs.leaf_ids.size());
    out->kd_depth = s->hs.kd_depth;
    out->lds_bytes = s->gpu.node_boxes ? 0 : s->gpu.image_bytes;
    out->node_boxes = s->gpu.node_boxes;
    out->device = s->device;
    out->n_devices = s->on_device ? 1 + static_cast<int64_t>(s->replicas.size()) : 0;
    out->kd_build = s->hs.kd_build;
    return MCPT_OK;
}

int mcpt_scene_copy_kd(const mcpt_scene* s, uint32_t* nodes, uint32_t* leaf_ids, int32_t* kd_tris, float* geoms) {
    if (!s) return fail(MCPT_E_INVALID, "NULL scene");
    const auto& hs = s->hs;
    if (nodes)
        for (size_t i = 0; i < hs.nodes.size(); ++i) {
            const auto& n = hs.nodes[i];
            uint32_t* o = nodes + 12 * i;
            o[0] = n.left; o[1] = n.right; o[2] = n.axis;
            std::memcpy(&o[3], &n.split, 4);
            std::memcpy(&o[4], n.bmin, 12);
            std::memcpy(&o[7], n.bmax, 12);
            o[10] = n.leaf_begin; o[11] = n.leaf_count;
        }
    if (leaf_ids && !hs.leaf_ids.empty()) std::memcpy(leaf_ids, hs.leaf_ids.data(), hs.leaf_ids.size() * 4);
    if (kd_tris) std::memcpy(kd_tris, hs.kd_tris.data(), hs.kd_tris.size() * 4);
    if (geoms)
        for (size_t g = 0; g < hs.geoms.size(); ++g) {
            const auto& e = hs.geoms[g];
            float* o = geoms + 14 * g;
            o[0] = e.Ka.x; o[1] = e.Ka.y; o[2] = e.Ka.z; o[3] = e.Kd.x; o[4] = e.Kd.y; o[5] = e.Kd.z;
            o[6] = e.Ks.x; o[7] = e.Ks.y; o[8] = e.Ks.z; o[9] = e.Ns; o[10] = e.Tr; o[11] = e.Ni;
            o[12] = static_cast<float>(e.start); o[13] = static_cast<float>(e.count);
        }
    return MCPT_OK;
}

int mcpt_render_device(mcpt_scene* s, const mcpt_render_params* p, float* d_fb_rgba, void* hip_stream) {
    return guarded([&]() -> int {
        if (!s) return fail(MCPT_E_INVALID, "NULL scene");
        render_async(*s, p, d_fb_rgba, static_cast<hipStream_t>(hip_stream));
        return MCPT_OK;
    });
}

int mcpt_render_stats_read(mcpt_scene* s, mcpt_render_stats* out) {
    return guarded([&]() -> int {
        if (!s || !s->on_device) return fail(MCPT_E_INVALID, "scene is not on a device");
        read_stats_all(*s, out);
        return MCPT_OK;
    });
}

static int render_sync(mcpt_scene* s, const mcpt_render_params* p, float* fb_rgb, mcpt_render_stats* stats,
                       uint32_t* unit_counters) {
    return guarded([&]() -> int {
        if (!s || !fb_rgb) return fail(MCPT_E_INVALID, "NULL argument");
        if (!s->on_device) return fail(MCPT_E_INVALID, "scene was created host-only");
        set_device(*s);
        Plan pl = make_plan(*s, p);
        const size_t npx = pl.out_pixels;
        ensure_buf(s->ws.fb, s->ws.fb_bytes, npx * 16);
        std::vector<float> rgba(npx * 4, 0.0f);
        if (p->prev_count > 0) {
            for (size_t i = 0; i < npx; ++i)
                for (int c = 0; c < 3; ++c) rgba[4 * i + c] = fb_rgb[3 * i + c];
            HIP_TRY(hipMemcpy(s->ws.fb, rgba.data(), npx * 16, hipMemcpyHostToDevice));
        } else {
            HIP_TRY(hipMemset(s->ws.fb, 0, npx * 16));
        }
        read_stats_all(*s, nullptr);   // start a fresh record
        void* d_uc = nullptr;
        const size_t uc_bytes = size_t(pl.kp.total_units) * 16;
        if (unit_counters) {
            HIP_TRY(hipMalloc(&d_uc, uc_bytes ? uc_bytes : 16));
            HIP_TRY(hipMemset(d_uc, 0, uc_bytes ? uc_bytes : 16));
        }
        render_async(*s, p, static_cast<float*>(s->ws.fb), nullptr, static_cast<uint32_t*>(d_uc));
        HIP_TRY(hipStreamSynchronize(nullptr));
        if (unit_counters) {
            HIP_TRY(hipMemcpy(unit_counters, d_uc, uc_bytes, hipMemcpyDeviceToHost));
            HIP_TRY(hipFree(d_uc));
        }
        HIP_TRY(hipMemcpy(rgba.data(), s->ws.fb, npx * 16, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < npx; ++i)
            for (int c = 0; c < 3; ++c) fb_rgb[3 * i + c] = rgba[4 * i + c];
        read_stats_all(*s, stats);
        return MCPT_OK;
    });
}

int mcpt_render(mcpt_scene* s, const mcpt_render_params* p, float* fb_rgb, mcpt_render_stats* stats) {
    return render_sync(s, p, fb_rgb, stats, nullptr);
}

int mcpt_intersect(mcpt_scene* s, int64_t n, const float* o, const float* d, float t_max, int32_t* tri_out,
                   float* hit_out, mcpt_render_stats* stats) {
    return guarded([&]() -> int {
        if (!s || n < 0 || (n && (!o || !d || !tri_out || !hit_out))) return fail(MCPT_E_INVALID, "NULL argument");
        if (!s->on_device) return fail(MCPT_E_INVALID, "scene was created host-only");
        if (n >= (int64_t(1) << 31) / 3) return fail(MCPT_E_UNSUPPORTED, "too many rays for one call");
        set_device(*s);
        mcpt_render_stats st;
        std::memset(&st, 0, sizeof st);
        st.devices = 1;
        if (n) {
            const size_t N = static_cast<size_t>(n);
            // one allocation: o, d, hits (3 floats each), slots, counters, then the
            // 16-B aligned stack spill area (32 entries per ray)
            const size_t stats_off = (N * 40 + 15) & ~size_t(15), spill_off = stats_off + 64;
            char* buf = nullptr;
            HIP_TRY(hipMalloc(reinterpret_cast<void**>(&buf), spill_off + N * 32 * 16));
            struct Free { char* p; ~Free() { (void)hipFree(p); } } guard{buf};
            mcpt::QueryParams q{};
            q.scene = s->gpu;
            q.o = reinterpret_cast<float*>(buf);
            q.d = q.o + 3 * N;
            q.hit = reinterpret_cast<float*>(buf) + 6 * N;
            q.slot = reinterpret_cast<int32_t*>(buf + 36 * N);
            q.stats = reinterpret_cast<unsigned long long*>(buf + stats_off);
            q.spill = reinterpret_cast<uint4*>(buf + spill_off);
            q.n = static_cast<uint32_t>(n);
            q.best_init = t_max;
            HIP_TRY(hipMemcpy(buf, o, N * 12, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(buf + N * 12, d, N * 12, hipMemcpyHostToDevice));
            HIP_TRY(hipMemset(q.stats, 0, 64));
            HIP_TRY(mcpt::launch_query(q, nullptr));
            HIP_TRY(hipDeviceSynchronize());
            std::vector<int32_t> slot(N);
            unsigned long long c[8];
            HIP_TRY(hipMemcpy(slot.data(), q.slot, N * 4, hipMemcpyDeviceToHost));
            HIP_TRY(hipMemcpy(hit_out, q.hit, N * 12, hipMemcpyDeviceToHost));
            HIP_TRY(hipMemcpy(c, q.stats, 64, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < N; ++i)
                tri_out[i] = slot[i] < 0 ? -1 : static_cast<int32_t>(s->tri_order[static_cast<size_t>(slot[i])]);
            st.rays = c[0]; st.inner_visits = c[2]; st.leaf_visits = c[3]; st.leaf_refs = c[4];
            st.tri_tests = c[5]; st.stack_spills = c[7];
        }
        if (stats) *stats = st;
        return MCPT_OK;
    });
}

int mcpt_render_unit_counters(mcpt_scene* s, const mcpt_render_params* p, float* fb_rgb, uint32_t* unit_counters) {
    if (!unit_counters) return fail(MCPT_E_INVALID, "unit_counters is NULL");
    return render_sync(s, p, fb_rgb, nullptr, unit_counters);
}

int64_t mcpt_shard_pixel_count(const mcpt_render_params* p) {
    if (!p || p->width <= 0 || p->height <= 0) return fail(MCPT_E_INVALID, "bad params");
    const int64_t T = p->tile > 0 ? p->tile : 8;
    const int64_t sc = p->shard_count > 1 ? p->shard_count : 1, si = sc > 1 ? p->shard_index : 0;
    if (si < 0 || si >= sc) return fail(MCPT_E_INVALID, "shard_index out of range");
    const int64_t ntiles = ((p->width + T - 1) / T) * ((p->height + T - 1) / T);
    const int64_t owned = si < ntiles ? (ntiles - si + sc - 1) / sc : 0;
    return owned * T * T;
}

int mcpt_shard_pixels(const mcpt_render_params* p, int32_t* xy) {
    const int64_t n = mcpt_shard_pixel_count(p);
    if (n < 0) return static_cast<int>(n);
    if (!xy) return fail(MCPT_E_INVALID, "xy is NULL");
    const int64_t T = p->tile > 0 ? p->tile : 8;
    const int64_t sc = p->shard_count > 1 ? p->shard_count : 1, si = sc > 1 ? p->shard_index : 0;
    const int64_t tiles_x = (p->width + T - 1) / T;
    for (int64_t v = 0; v < n; ++v) {
        const int64_t k = v / (T * T), w = v % (T * T);
        const int64_t t = si + k * sc;
        const int64_t x = (t % tiles_x) * T + w % T, y = (t / tiles_x) * T + w / T;
        const bool in = x < p->width && y < p->height;
        xy[2 * v] = in ? static_cast<int32_t>(x) : -1;
        xy[2 * v + 1] = in ? static_cast<int32_t>(y) : -1;
    }
    return MCPT_OK;
}

int mcpt_scene_reserve(mcpt_scene* s, const mcpt_render_params* p) {
    return guarded([&]() -> int {
        if (!s || !s->on_device) return fail(MCPT_E_INVALID, "scene is not on a device");
        DeviceGuard guard;
        auto reserve = [&](mcpt_scene& sc, const mcpt_render_params* q) {
            set_device(sc);
            sc.reserved = true;
            ensure_capture_timing(sc);   // (events exist before any capture)
            Plan pl = make_plan(sc, q);
            fit_wavefront(sc, pl);
            const int sets = pl.pipeline == MCPT_PIPELINE_WAVEFRONT ? pl.wf_streams : 1;
            prepare_workspace(sc, pl, pl.pipeline == MCPT_PIPELINE_MEGAKERNEL, sets);
            if (pl.pipeline == MCPT_PIPELINE_WAVEFRONT) {
                mcpt::WfParams wf[mcpt::kMaxWfStreams];
                prepare_wavefront(sc, pl, sets, wf);
                sc.wf_reserved = std::max(sc.wf_reserved, sc.ws.wf_bytes);
                ensure_wf_streams(sc, sets);   // streams and events exist before any capture
            }
        };
        if (!multi_device(*s, p, nullptr)) {
            reserve(*s, p);
            return MCPT_OK;
        }
        const int n = 1 + static_cast<int>(s->replicas.size());
        const bool use_rccl = p->gather == MCPT_GATHER_RCCL;
        set_device(*s);
        const uint64_t slot = multi_slot(make_plan(*s, p), p, n);
        for (int r = 0; r < n; ++r) {
            mcpt_render_params pr = *p;
            pr.shard_count = n; pr.shard_index = r; pr.packed = 1;
            mcpt_scene& sc = r ? *s->replicas[size_t(r - 1)] : *s;
            reserve(sc, &pr);
            if (r) ensure_buf(sc.ws.fb, sc.ws.fb_bytes, use_rccl ? size_t(slot) * 16
                                                                  : size_t(mcpt_shard_pixel_count(&pr)) * 16);
        }
        set_device(*s);
        // the gather buffer: n slots of the largest shard (shard 0 owns the most tiles)
        ensure_buf(s->gather, s->gather_bytes, size_t(n) * size_t(slot) * 16);
        if (use_rccl) {   // the communicators and rank 0's send buffer exist before any capture
            ensure_comms(*s);
            ensure_buf(s->gather_send, s->gather_send_bytes, size_t(slot) * 16);
        }
        if (!s->start) HIP_TRY(hipEventCreateWithFlags(&s->start, hipEventDisableTiming));
        return MCPT_OK;
    });
}

int mcpt_plan_query(mcpt_scene* s, const mcpt_render_params* p, mcpt_plan_info* out) {
    return guarded([&]() -> int {
        if (!s || !s->on_device || !p || !out) return fail(MCPT_E_INVALID, "NULL argument or host-only scene");
        DeviceGuard guard;
        // a multi-device render: the plan of devices[0]'s shard (the largest)
        mcpt_render_params q = *p;
        const bool multi = multi_device(*s, p, nullptr);
        if (multi) {
            q.shard_count = 1 + static_cast<int32_t>(s->replicas.size());
            q.shard_index = 0;
            q.packed = 1;
        }
        set_device(*s);
        Plan pl = make_plan(*s, &q);
        const uint32_t unfitted = pl.wf_capacity;
        fit_wavefront(*s, pl);
        mcpt_plan_info r;
        std::memset(&r, 0, sizeof r);
        const uint32_t img = s->gpu.image_bytes;
        const bool wf = pl.pipeline == MCPT_PIPELINE_WAVEFRONT;
        r.pipeline = pl.pipeline;
        if (wf) r.variant = (!s->gpu.node_boxes && mcpt::lds_bytes_in_lds(img, 4) + 32 <= mcpt::kMaxLds) ? 4 : 5;
        else if (s->gpu.node_boxes) r.variant = 3;
        else r.variant = mcpt::lds_bytes_in_lds(img, 8) <= mcpt::kMaxLds ? 1 : (mcpt::lds_bytes_in_lds(img, 4) <= mcpt::kMaxLds ? 2 : 3);
        r.wf_streams = wf ? pl.wf_streams : 0;
        r.wf_batch = wf ? pl.wf_capacity : 0;
        r.wf_batch_default = wf ? unfitted : 0;
        r.wf_refill = wf ? pl.wf_refill : 0;
        r.wf_group_shift = wf ? static_cast<int32_t>(pl.wf_group_shift) : 0;
        r.ready_thresh = wf ? 0 : pl.kp.ready_thresh;
        r.tail_units = wf ? 0 : static_cast<int32_t>(tail_units_for(*s, pl));
        r.work_paths = pl.work;
        const uint64_t lanes = static_cast<uint64_t>(mcpt::total_lanes_for(img, s->cus));
        uint64_t ws = uint64_t(pl.kp.nchunks) * pl.kp.npix_local * 16 + 256 +
                      uint64_t(wf ? pl.wf_streams : 1) * 32 * lanes * 16;
        if (wf) {
            r.wf_queue_bytes = uint64_t(wf_layout(*s, pl, pl.wf_capacity).need) * uint64_t(pl.wf_streams);
            ws += r.wf_queue_bytes;
        }
        else ws += uint64_t(r.tail_units) * pl.kp.chunk * 16;
        r.workspace_bytes = ws;
        size_t fr = 0, tot = 0;
        HIP_TRY(hipMemGetInfo(&fr, &tot));
        r.device_free_bytes = fr;
        r.devices = multi ? q.shard_count : 1;
        r.peer_access = s->peer_access ? 1 : 0;
        *out = r;
        return MCPT_OK;
    });
}

}  // extern "C"
