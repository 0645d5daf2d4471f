// Drop-in check: code written against the reference's PW::Tracer API (the call
// sequence of CVMCTracer/main.cpp:16-18) compiled against include/mcpt_pw_tracer.hpp.
// ObjModel here is a minimal stand-in with the reference's member names; the
// data comes from the library's own reader.
// Usage: pw_tracer_dropin scene.obj out.bin [devices, e.g. 0,0 -> Initialize({0, 0})]
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

#include "mcpt_pw_tracer.hpp"

struct Vec3 { float x, y, z; };
struct Tri { int m_vertexIndex[3], m_textureIndex[3], m_normalIndex[3], materialIndex; };
struct Mat { Vec3 Ka, Kd, Ks; double Ns, Tr, Ni; };
struct Group { std::vector<int> m_triangleIndices; };
struct ObjModel {
    std::vector<Vec3> m_vertices, m_normals;
    std::vector<Tri> m_triangles;
    std::vector<Mat> m_materials;
    std::map<std::string, Group> m_groups;
};

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    mcpt_model* mm = nullptr;
    if (mcpt_model_read_obj(argv[1], &mm) != MCPT_OK) { std::printf("read: %s\n", mcpt_last_error()); return 1; }
    mcpt_model_info info;
    mcpt_model_get_info(mm, &info);
    ObjModel model;
    std::vector<float> v(3 * info.n_vertices), n(3 * info.n_normals);
    std::vector<int32_t> t(10 * info.n_triangles);
    std::vector<double> m(12 * info.n_materials);
    mcpt_model_copy_vertices(mm, v.data());
    mcpt_model_copy_normals(mm, n.data());
    mcpt_model_copy_triangles(mm, t.data());
    mcpt_model_copy_materials(mm, m.data());
    for (int64_t i = 0; i < info.n_vertices; ++i) model.m_vertices.push_back({v[3 * i], v[3 * i + 1], v[3 * i + 2]});
    for (int64_t i = 0; i < info.n_normals; ++i) model.m_normals.push_back({n[3 * i], n[3 * i + 1], n[3 * i + 2]});
    for (int64_t i = 0; i < info.n_triangles; ++i) {
        Tri tr;
        for (int j = 0; j < 3; ++j) { tr.m_vertexIndex[j] = t[10 * i + j]; tr.m_textureIndex[j] = t[10 * i + 3 + j]; tr.m_normalIndex[j] = t[10 * i + 6 + j]; }
        tr.materialIndex = t[10 * i + 9];
        model.m_triangles.push_back(tr);
    }
    for (int64_t i = 0; i < info.n_materials; ++i) {
        const double* q = &m[12 * i];
        model.m_materials.push_back({{(float)q[0], (float)q[1], (float)q[2]}, {(float)q[3], (float)q[4], (float)q[5]},
                                     {(float)q[6], (float)q[7], (float)q[8]}, q[9], q[10], q[11]});
    }
    for (int64_t g = 0; g < info.n_groups; ++g) {
        char name[256];
        int64_t cnt = 0;
        mcpt_model_group(mm, g, name, sizeof name, &cnt, nullptr);
        std::vector<int32_t> ids(cnt);
        mcpt_model_group(mm, g, name, sizeof name, &cnt, ids.data());
        model.m_groups[name].m_triangleIndices.assign(ids.begin(), ids.end());
    }
    mcpt_model_free(mm);

    const int W = 40, H = 30;
    std::vector<Vec3> hostcolor(W * H);
    std::vector<int32_t> devices;
    for (const char* c = argc > 3 ? argv[3] : ""; *c;) {
        char* end = nullptr;
        devices.push_back(static_cast<int32_t>(std::strtol(c, &end, 10)));
        c = *end ? end + 1 : end;
    }
    const int init = devices.empty() ? PW::Tracer::Initialize() : PW::Tracer::Initialize(devices);
    if (argc > 5 && std::string(argv[5]) == "rccl") PW::Tracer::UseRcclGather(true);
    if (init != 0 || PW::Tracer::CreateGeometry(&model) != 0 ||
        PW::Tracer::RenderScene(1, hostcolor.data(), W, H, 3, argc > 4 ? std::atoi(argv[4]) : 4) != 0) {
        std::printf("tracer: %s\n", mcpt_last_error());
        return 1;
    }
    PW::Tracer::DestroyGeometry();
    FILE* f = std::fopen(argv[2], "wb");
    std::fwrite(hostcolor.data(), sizeof(Vec3), hostcolor.size(), f);
    std::fclose(f);
    std::printf("ok\n");
    return 0;
}
