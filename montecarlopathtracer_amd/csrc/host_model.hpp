// host_model.hpp -- host-side scene model, geometry table and KD tree.
//
// ObjModel mirrors CVMCTracer/CVMCTracer/Framework/ObjReader.hpp:37-63 (dummy
// element 0 in every array, groups in std::map order).  Geometry mirrors the
// per-group record CreateGeometry uploads (CUTracer.cu:277-311, Geometry.h:30-35).
// KdTree holds the QuinEngine KD tree (Utils/KDTree.hpp:58-287) in the BFS
// order of its GPU upload (RTX/ShaderResource.hpp:128-179).
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace mcpt {

struct Vec3 {
    float x = 0, y = 0, z = 0;
};

struct ObjTriangle {                  // ObjReader.hpp:12-18
    int32_t v[3] = {0, 0, 0};
    int32_t t[3] = {0, 0, 0};
    int32_t n[3] = {0, 0, 0};
    int32_t material = 0;
};

struct ObjMaterial {                  // ObjReader.hpp:20-30
    std::string name;
    Vec3 Ka, Kd, Ks;
    double Ns = 1.0, Tr = 0.0, Ni = 1.0;
};

struct ObjModel {
    std::string path;
    std::vector<Vec3> vertices;
    int64_t n_texcoords = 0;
    std::vector<Vec3> normals;
    std::vector<ObjTriangle> triangles;
    std::vector<ObjMaterial> materials;
    std::map<std::string, std::vector<int32_t>> groups;
};

// Throws mcpt::Error on failure.  flavor MCPT_OBJ_CVMCTRACER (0): the
// CVMCTracer ObjReader (read_obj_cv); MCPT_OBJ_TINYOBJ (1): tinyobjloader as
// QuinEngine uses it (host_model.cpp read_obj_tinyobj).
void read_obj(const std::string& path, ObjModel& out, int flavor = 0);
void read_obj_cv(const std::string& path, ObjModel& out);

struct Geometry {                     // Geometry.h:14-35
    Vec3 Ka, Kd, Ks;
    float Ns, Tr, Ni;
    uint32_t start, count;
};

struct KdNode {                       // CSKDTree (Structure.hpp:213-223) minus the 64-slot cap
    uint32_t left = 0xFFFFFFFFu, right = 0xFFFFFFFFu;
    float bmin[3], bmax[3];
    uint32_t axis = 0;                // 0 leaf, 1..3 split axis
    float split = 0.0f;
    uint32_t leaf_begin = 0, leaf_count = 0;
};

struct HostScene {
    std::vector<Geometry> geoms;
    std::vector<int32_t> kd_tris;     // kd id -> OBJ triangle index (ascending)
    std::vector<uint32_t> kd_geom;    // kd id -> geometry index
    std::vector<uint32_t> kd_prio;    // kd id -> brute-force iteration rank (tie-break)
    std::vector<float> kd_verts;      // kd id -> 9 floats a,b,c
    std::vector<float> kd_normals;    // kd id -> 9 floats n0,n1,n2
    std::vector<KdNode> nodes;
    std::vector<uint32_t> leaf_ids;
    int kd_depth = 0;
    int kd_build = 0;                 // MCPT_KD_BUILD_*
};

// CreateGeometry semantics + KD build; throws mcpt::Error.  With a cache
// directory the KD tree is read from / written to it (kd_cache.cpp);
// *cache_hit (if given) = 1 when it was read, 0 when built.
// kd_build: MCPT_KD_BUILD_REFERENCE (KDTree.hpp) or MCPT_KD_BUILD_SAH.
void build_host_scene(const ObjModel& m, HostScene& out, const char* kd_cache_dir = nullptr,
                      int* cache_hit = nullptr, int kd_build = 0);
// on-disk KD cache (kd_cache.cpp): load returns false unless a valid file exists
// (files are keyed by the vertices and the build rule)
bool kd_cache_load(const std::string& dir, const std::vector<float>& tri_verts, std::vector<KdNode>& nodes,
                   std::vector<uint32_t>& leaf_ids, int& depth, int kd_build = 0);
bool kd_cache_store(const std::string& dir, const std::vector<float>& tri_verts, const std::vector<KdNode>& nodes,
                    const std::vector<uint32_t>& leaf_ids, int depth, int kd_build = 0);
// KD build only over kd_verts (KDTree.hpp semantics, or the SAH rule of
// MCPT_KD_BUILD_SAH); fills nodes/leaf_ids/kd_depth.
void build_kdtree(const std::vector<float>& tri_verts, std::vector<KdNode>& nodes,
                  std::vector<uint32_t>& leaf_ids, int& depth, int kd_build = 0);

struct Error {
    int code;
    std::string msg;
};

}  // namespace mcpt
