// mcpt_pw_tracer.hpp -- header-only drop-in for the reference's tracer module.
//
// Replaces CVMCTracer/CVMCTracer/CUDA/CUTracer.h (namespace PW::Tracer):
//     cudaError_t Initialize();                                   CUTracer.h:9
//     cudaError_t CreateGeometry(const PW::FileReader::ObjModel*); CUTracer.h:10
//     cudaError_t DestroyGeometry();                               CUTracer.h:11
//     cudaError_t RenderScene(const PWint sceneID, PWVector3f*);   CUTracer.h:12
// with the same names, argument meaning and call order as CVMCTracer/main.cpp
// uses them, implemented over the C ABI in mcpt.h (link -lmcpt).  The model
// and colour types are template parameters so this header compiles against the
// reference's own ObjModel / PWVector3f without including CUDA headers.
// Return value: 0 on success, a negative MCPT_E_* code otherwise
// (mcpt_last_error() has the message); the reference returned cudaError_t.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "mcpt.h"

namespace PW {
namespace Tracer {

namespace detail {
inline mcpt_scene*& scene() {      // the reference keeps the scene in module globals (CUTracer.cu:30-37)
    static mcpt_scene* s = nullptr;
    return s;
}
inline int32_t& gather() {           // how a multi-device render's shards reach devices[0]
    static int32_t g = MCPT_GATHER_PEER;
    return g;
}
}  // namespace detail

inline int Initialize() {            // CUTracer.cu:220-223: cudaSetDevice(0)
    const int32_t dev = 0;
    return mcpt_init(&dev, 1);
}

// Multi-GPU extension (no reference counterpart: the reference ran on one GPU):
// scenes created afterwards are replicated on every listed device and each
// RenderScene launch is split into interleaved tiles across them, gathered to
// devices[0] -- the same image as Initialize() gives (mcpt.h, mcpt_init).
inline int Initialize(const std::vector<int32_t>& devices) {
    return mcpt_init(devices.data(), static_cast<int32_t>(devices.size()));
}

// RenderScene's gather for such a device list: one RCCL collective over the
// list (ncclCommInitAll + ncclGather into devices[0]) instead of peer copies
// (mcpt_render_params::gather); also valid for a one-device list.
inline void UseRcclGather(bool on) { detail::gather() = on ? MCPT_GATHER_RCCL : MCPT_GATHER_PEER; }

// ObjModelT: PW::FileReader::ObjModel (ObjReader.hpp:37-63): m_vertices, m_normals
// (x,y,z floats), m_triangles (m_vertexIndex[3], m_textureIndex[3], m_normalIndex[3],
// materialIndex), m_materials (Ka/Kd/Ks .x .y .z, Ns, Tr, Ni), m_groups (map name ->
// .m_triangleIndices).
template <class ObjModelT>
int CreateGeometry(const ObjModelT* model) {   // CUTracer.cu:225-314 (+ KD build)
    if (!model) return MCPT_E_INVALID;
    std::vector<float> v, n;
    for (const auto& p : model->m_vertices) { v.push_back(p.x); v.push_back(p.y); v.push_back(p.z); }
    for (const auto& p : model->m_normals) { n.push_back(p.x); n.push_back(p.y); n.push_back(p.z); }
    std::vector<int32_t> t;
    for (const auto& tr : model->m_triangles) {
        for (int j = 0; j < 3; ++j) t.push_back(tr.m_vertexIndex[j]);
        for (int j = 0; j < 3; ++j) t.push_back(tr.m_textureIndex[j]);
        for (int j = 0; j < 3; ++j) t.push_back(tr.m_normalIndex[j]);
        t.push_back(tr.materialIndex);
    }
    std::vector<double> m;
    for (const auto& mt : model->m_materials) {
        const double q[12] = {mt.Ka.x, mt.Ka.y, mt.Ka.z, mt.Kd.x, mt.Kd.y, mt.Kd.z,
                              mt.Ks.x, mt.Ks.y, mt.Ks.z, (double)mt.Ns, (double)mt.Tr, (double)mt.Ni};
        m.insert(m.end(), q, q + 12);
    }
    std::vector<std::string> names;
    std::vector<const char*> cnames;
    std::vector<int64_t> offs{0};
    std::vector<int32_t> gt;
    for (const auto& kv : model->m_groups) {
        names.push_back(kv.first);
        for (auto id : kv.second.m_triangleIndices) gt.push_back(static_cast<int32_t>(id));
        offs.push_back(static_cast<int64_t>(gt.size()));
    }
    for (const auto& s : names) cnames.push_back(s.c_str());
    mcpt_model_desc d;
    d.vertices = v.data(); d.n_vertices = static_cast<int64_t>(v.size() / 3);
    d.normals = n.data(); d.n_normals = static_cast<int64_t>(n.size() / 3);
    d.triangles = t.data(); d.n_triangles = static_cast<int64_t>(t.size() / 10);
    d.materials = m.data(); d.n_materials = static_cast<int64_t>(m.size() / 12);
    d.group_names = cnames.data(); d.group_offsets = offs.data(); d.group_tris = gt.data();
    d.n_groups = static_cast<int64_t>(names.size());
    mcpt_model* mm = nullptr;
    int rc = mcpt_model_create(&d, &mm);
    if (rc != MCPT_OK) return rc;
    if (detail::scene()) mcpt_scene_destroy(detail::scene());
    detail::scene() = nullptr;
    rc = mcpt_scene_create(mm, &detail::scene());
    mcpt_model_free(mm);
    return rc;
}

inline int DestroyGeometry() {       // CUTracer.cu:316-338, freeing what was allocated
    if (detail::scene()) mcpt_scene_destroy(detail::scene());
    detail::scene() = nullptr;
    return MCPT_OK;
}

// RenderScene (CUTracer.cu:340-404): num_kernels launches of spp_per_kernel samples,
// hostcolor (width*height PWVector3f, row-major y*W+x) holds the running mean after
// every launch (prevCount semantics, CUTracer.cu:215-217).  Camera of sceneID as
// CUTracer.cu:347-374.  No OpenCV window / PNG side effects.
// Summation order: by default the reference's -- each launch sums all of its
// spp_per_kernel samples of a pixel in sample order, then divides
// (CUTracer.cu:192-214; spp_chunk = 0).  A positive spp_chunk sums chunks of
// that many samples first and the chunk sums in order (an explicit deviation:
// the same image within fp32 rounding, not bit for bit).
template <class Vec3T>
int RenderScene(const int sceneID, Vec3T* hostcolor, int width = 800, int height = 600,
                int num_kernels = 100, int spp_per_kernel = 100, int spp_chunk = 0) {
    static_assert(sizeof(Vec3T) == 3 * sizeof(float), "hostcolor must be 3 packed floats per pixel");
    if (!detail::scene()) return MCPT_E_INVALID;
    mcpt_render_params p;
    mcpt_render_params_default(&p);
    p.width = width;
    p.height = height;
    p.spp = static_cast<uint32_t>(spp_per_kernel);
    p.spp_chunk = static_cast<uint32_t>(spp_chunk > 0 ? spp_chunk : 0);
    p.gather = detail::gather();
    p.eye[2] = (sceneID == 1) ? 17.0f : 23.0f;
    for (int k = 0; k < num_kernels; ++k) {
        p.spp_offset = static_cast<uint32_t>(k * spp_per_kernel);
        p.prev_count = static_cast<uint32_t>(k);
        int rc = mcpt_render(detail::scene(), &p, reinterpret_cast<float*>(hostcolor), nullptr);
        if (rc != MCPT_OK) return rc;
    }
    return MCPT_OK;
}

}  // namespace Tracer
}  // namespace PW
