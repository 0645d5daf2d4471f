// tinyobj_dump.cpp -- dumps what the reference's vendored tinyobjloader v1.1.1
// (MCRT/QuinEngine/3rdparty/include/tiny_obj_loader.h, used by QuinModel,
// QE/Utils/Structure.hpp:9-12) reads from an OBJ/MTL pair.
// TEST INFRASTRUCTURE ONLY: built by oracle/ref/Makefile into oracle/_ref/,
// run by tests/golden/make_golden.py to produce committed fixtures.
//
// Output (little-endian binary): magic "TOBJ", then
//   u32 nv, f32[nv*3] vertices; u32 nn, f32[nn*3] normals;
//   u32 nshapes; per shape: u32 name_len, name bytes, u32 nidx, i32[nidx*3] (v,t,n),
//   u32 nface, i32[nface] material ids;
//   u32 nmat; per material: u32 name_len, name, f32[3] ambient, f32[3] diffuse,
//   f32[3] specular, f32 shininess, f32 dissolve, f32 ior.
#define TINYOBJLOADER_IMPLEMENTATION
#include "tiny_obj_loader.h"

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

static void w32(FILE* f, uint32_t v) { fwrite(&v, 4, 1, f); }
static void wstr(FILE* f, const std::string& s) { w32(f, (uint32_t)s.size()); fwrite(s.data(), 1, s.size(), f); }

int main(int argc, char** argv) {
    if (argc != 4) { fprintf(stderr, "usage: %s scene.obj mtl_dir out.bin\n", argv[0]); return 2; }
    tinyobj::attrib_t attr;
    std::vector<tinyobj::shape_t> shapes;
    std::vector<tinyobj::material_t> mats;
    std::string err;
    bool ok = tinyobj::LoadObj(&attr, &shapes, &mats, &err, argv[1], argv[2]);
    if (!ok) { fprintf(stderr, "LoadObj failed: %s\n", err.c_str()); return 1; }
    FILE* f = fopen(argv[3], "wb");
    if (!f) return 1;
    fwrite("TOBJ", 1, 4, f);
    w32(f, (uint32_t)(attr.vertices.size() / 3));
    fwrite(attr.vertices.data(), 4, attr.vertices.size(), f);
    w32(f, (uint32_t)(attr.normals.size() / 3));
    fwrite(attr.normals.data(), 4, attr.normals.size(), f);
    w32(f, (uint32_t)shapes.size());
    for (const auto& s : shapes) {
        wstr(f, s.name);
        w32(f, (uint32_t)s.mesh.indices.size());
        for (const auto& ix : s.mesh.indices) {
            int32_t t[3] = {ix.vertex_index, ix.texcoord_index, ix.normal_index};
            fwrite(t, 4, 3, f);
        }
        w32(f, (uint32_t)s.mesh.material_ids.size());
        fwrite(s.mesh.material_ids.data(), 4, s.mesh.material_ids.size(), f);
    }
    w32(f, (uint32_t)mats.size());
    for (const auto& m : mats) {
        wstr(f, m.name);
        fwrite(m.ambient, 4, 3, f);
        fwrite(m.diffuse, 4, 3, f);
        fwrite(m.specular, 4, 3, f);
        fwrite(&m.shininess, 4, 1, f);
        fwrite(&m.dissolve, 4, 1, f);
        fwrite(&m.ior, 4, 1, f);
    }
    fclose(f);
    return 0;
}
