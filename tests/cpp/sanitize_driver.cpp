// sanitize_driver.cpp -- host-side inputs of libmcpt under AddressSanitizer +
// UndefinedBehaviorSanitizer (scripts/sanitize.sh builds it).  No GPU calls.
//
// Every untrusted-input path of the host code, through the C ABI:
//   * OBJ/MTL reader (ObjReader.cpp:8-259 semantics) on the bundled scenes and
//     on every file of a malformed corpus: each must load or fail with an error
//     code, never crash or touch memory it does not own;
//   * CreateGeometry + KD build (host-only scenes) on whatever loaded;
//   * mcpt_model_create on in-memory descriptors with bad counts/indices;
//   * the on-disk KD cache (kd_cache.cpp) on truncated, bit-flipped and
//     header-forged files: every load must either be rejected (rebuild) or
//     give the tree the builder gives, bit for bit.
// Usage: sanitize_driver <scratch dir> <scene.obj>... -- <corpus file>...
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "mcpt.h"

namespace {

int failures = 0;

#define CHECK(cond)                                                              \
    do {                                                                         \
        if (!(cond)) {                                                           \
            std::printf("CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                          \
        }                                                                        \
    } while (0)

struct Kd {
    std::vector<uint32_t> nodes, leafs;
    std::vector<int32_t> tris;
    bool operator==(const Kd& o) const { return nodes == o.nodes && leafs == o.leafs && tris == o.tris; }
};

Kd kd_of(mcpt_scene* s) {
    mcpt_scene_info i;
    CHECK(mcpt_scene_get_info(s, &i) == MCPT_OK);
    Kd k;
    k.nodes.resize(size_t(i.n_nodes) * 12);
    k.leafs.resize(size_t(i.n_leaf_refs) + 1);
    k.tris.resize(size_t(i.n_triangles));
    std::vector<float> geoms(size_t(i.n_geometries) * 14 + 1);
    CHECK(mcpt_scene_copy_kd(s, k.nodes.data(), k.leafs.data(), k.tris.data(), geoms.data()) == MCPT_OK);
    return k;
}

// read a model and build a host scene; returns the model's load code
int load_and_build(const std::string& path, bool verbose) {
    std::fflush(stdout);
    mcpt_model* m = nullptr;
    const int rc = mcpt_model_read_obj(path.c_str(), &m);
    if (rc != MCPT_OK) {
        CHECK(m == nullptr && rc < 0 && std::strlen(mcpt_last_error()) > 0);
        if (verbose) std::printf("  %-40s read -> %d (%s)\n", path.c_str(), rc, mcpt_last_error());
        return rc;
    }
    mcpt_model_info mi;
    CHECK(mcpt_model_get_info(m, &mi) == MCPT_OK);
    std::vector<float> v(size_t(mi.n_vertices) * 3), n(size_t(mi.n_normals) * 3);
    std::vector<int32_t> t(size_t(mi.n_triangles) * 10);
    std::vector<double> mt(size_t(mi.n_materials) * 12);
    CHECK(mcpt_model_copy_vertices(m, v.data()) == MCPT_OK);
    CHECK(mcpt_model_copy_normals(m, n.data()) == MCPT_OK);
    CHECK(mcpt_model_copy_triangles(m, t.data()) == MCPT_OK);
    CHECK(mcpt_model_copy_materials(m, mt.data()) == MCPT_OK);
    for (int64_t g = 0; g < mi.n_groups; ++g) {
        char name[64];
        int64_t cnt = 0;
        CHECK(mcpt_model_group(m, g, name, sizeof name, &cnt, nullptr) == MCPT_OK);
        std::vector<int32_t> ids(size_t(cnt) + 1);
        CHECK(mcpt_model_group(m, g, name, sizeof name, &cnt, ids.data()) == MCPT_OK);
    }
    mcpt_scene* s = nullptr;
    const int sc = mcpt_scene_create_host(m, &s);
    if (sc == MCPT_OK) {
        (void)kd_of(s);
        mcpt_scene_destroy(s);
    }
    if (verbose)
        std::printf("  %-40s read ok (%lld tris), scene -> %d %s\n", path.c_str(), (long long)mi.n_triangles, sc,
                    sc ? mcpt_last_error() : "");
    mcpt_model_free(m);
    return rc;
}

void bad_descriptors() {
    const float v[12] = {0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 1, 0};
    const float n[6] = {0, 0, 0, 0, 0, 1};
    int32_t t[20] = {0};
    t[10] = 1; t[11] = 2; t[12] = 3; t[16] = 1; t[17] = 1; t[18] = 1; t[19] = 0;
    const double mats[12] = {0, 0, 0, .5, .5, .5, 0, 0, 0, 1, 0, 1};
    const char* names[1] = {"g"};
    int64_t offs[2] = {0, 1};
    int32_t gt[1] = {1};
    mcpt_model_desc d = {v, 4, n, 2, t, 2, mats, 1, names, offs, gt, 1};
    mcpt_model* m = nullptr;
    CHECK(mcpt_model_create(&d, &m) == MCPT_OK);
    mcpt_scene* s = nullptr;
    CHECK(mcpt_scene_create_host(m, &s) == MCPT_OK);
    mcpt_scene_destroy(s);
    mcpt_model_free(m);
    auto rejects = [&](mcpt_model_desc bad) {
        mcpt_model* mm = nullptr;
        const int rc = mcpt_model_create(&bad, &mm);
        if (rc == MCPT_OK) {                 // accepted by the model: the scene must reject it
            mcpt_scene* ss = nullptr;
            const int sc = mcpt_scene_create_host(mm, &ss);
            CHECK(sc != MCPT_OK);
            if (sc == MCPT_OK) mcpt_scene_destroy(ss);
            mcpt_model_free(mm);
        }
    };
    mcpt_model_desc b = d; b.n_vertices = 0; rejects(b);
    b = d; b.vertices = nullptr; rejects(b);
    b = d; b.n_groups = -1; rejects(b);
    int64_t offs_bad[2] = {1, 0};
    b = d; b.group_offsets = offs_bad; rejects(b);
    int32_t gt_bad[1] = {5};
    b = d; b.group_tris = gt_bad; rejects(b);
    int32_t t_bad[20];
    std::memcpy(t_bad, t, sizeof t);
    t_bad[11] = 99;                           // vertex index past the array
    b = d; b.triangles = t_bad; rejects(b);
    std::memcpy(t_bad, t, sizeof t);
    t_bad[17] = -3;                           // negative normal index
    b = d; b.triangles = t_bad; rejects(b);
    std::memcpy(t_bad, t, sizeof t);
    t_bad[19] = 7;                            // material past the array
    b = d; b.triangles = t_bad; rejects(b);
    CHECK(mcpt_model_create(nullptr, &m) != MCPT_OK);
    CHECK(mcpt_model_read_obj(nullptr, &m) != MCPT_OK);
    CHECK(mcpt_scene_create_host(nullptr, &s) != MCPT_OK);
    mcpt_render_params p;
    mcpt_render_params_default(&p);
    p.width = 37; p.height = 29; p.tile = 8; p.shard_count = 3; p.shard_index = 2;
    const int64_t np = mcpt_shard_pixel_count(&p);
    std::vector<int32_t> xy(size_t(np) * 2);
    CHECK(np > 0 && mcpt_shard_pixels(&p, xy.data()) == MCPT_OK);
    p.shard_index = 3;
    CHECK(mcpt_shard_pixel_count(&p) < 0);
}

std::string read_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    std::ostringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

void write_file(const std::string& path, const std::string& data) {
    std::ofstream f(path, std::ios::binary | std::ios::trunc);
    f.write(data.data(), std::streamsize(data.size()));
}

// the KD cache on corrupted / forged files
void kd_cache(const std::string& scratch, const std::string& scene) {
    const std::string dir = scratch + "/kd";
    std::string cmd = "rm -rf '" + dir + "' && mkdir -p '" + dir + "'";
    if (std::system(cmd.c_str()) != 0) { ++failures; return; }
    mcpt_model* m = nullptr;
    CHECK(mcpt_model_read_obj(scene.c_str(), &m) == MCPT_OK);
    if (!m) return;
    mcpt_scene* s = nullptr;
    int32_t hit = -1;
    CHECK(mcpt_scene_create_cached(m, dir.c_str(), 1, &s, &hit) == MCPT_OK && hit == 0);
    const Kd ref = kd_of(s);
    mcpt_scene_destroy(s);
    std::string file;
    {
        FILE* p = popen(("ls '" + dir + "'").c_str(), "r");
        char buf[256] = {0};
        if (p && std::fgets(buf, sizeof buf, p)) file = dir + "/" + std::string(buf, std::strcspn(buf, "\n"));
        if (p) pclose(p);
    }
    CHECK(!file.empty());
    const std::string good = read_file(file);
    CHECK(good.size() > 72);
    std::mt19937 rng(12345);
    int accepted = 0, rejected = 0;
    auto trial = [&](const std::string& data) {
        write_file(file, data);
        mcpt_scene* t = nullptr;
        int32_t h = -1;
        CHECK(mcpt_scene_create_cached(m, dir.c_str(), 1, &t, &h) == MCPT_OK);
        if (!t) return;
        CHECK(kd_of(t) == ref);               // a load that passes the checks is the builder's tree
        (h ? accepted : rejected)++;
        mcpt_scene_destroy(t);
    };
    for (size_t cut : {size_t(0), size_t(7), size_t(71), size_t(72), size_t(100), good.size() / 2, good.size() - 1})
        trial(good.substr(0, std::min(cut, good.size())));
    trial(good + std::string(1, '\0'));
    for (int i = 0; i < 200; ++i) {           // single bit flips anywhere
        std::string d = good;
        const size_t at = std::uniform_int_distribution<size_t>(0, d.size() - 1)(rng);
        d[at] = char(d[at] ^ (1 << (rng() % 8)));
        trial(d);
    }
    for (int i = 0; i < 100; ++i) {           // random header words (sizes, depth, keys)
        std::string d = good;
        const size_t at = 8 + 4 * std::uniform_int_distribution<size_t>(0, 15)(rng);
        const uint32_t w = i % 3 == 0 ? 0xFFFFFFFFu : (i % 3 == 1 ? uint32_t(rng()) : uint32_t(rng() % 64));
        std::memcpy(&d[at], &w, 4);
        trial(d);
    }
    {   // header announcing 2^31 - 1 nodes on a short file: rejected before allocating
        std::string d = good;
        const uint64_t big = (uint64_t(1) << 31) - 1;
        std::memcpy(&d[40], &big, 8);
        trial(d);
    }
    trial(good);
    CHECK(accepted >= 1);                     // the untouched file (and flips in padding) load
    std::printf("  kd cache: %d loads accepted (identical tree), %d rejected and rebuilt\n", accepted, rejected);
    mcpt_model_free(m);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s scratch scene.obj... -- corpus...\n", argv[0]);
        return 2;
    }
    const std::string scratch = argv[1];
    std::vector<std::string> scenes, corpus;
    bool in_corpus = false;
    for (int i = 2; i < argc; ++i) {
        if (std::strcmp(argv[i], "--") == 0) { in_corpus = true; continue; }
        (in_corpus ? corpus : scenes).push_back(argv[i]);
    }
    std::printf("scenes:\n");
    for (const auto& s : scenes) CHECK(load_and_build(s, true) == MCPT_OK);
    std::printf("malformed corpus (%zu files):\n", corpus.size());
    for (const auto& c : corpus) (void)load_and_build(c, true);
    std::printf("descriptors:\n");
    bad_descriptors();
    std::printf("kd cache:\n");
    if (!scenes.empty()) kd_cache(scratch, scenes.front());
    std::printf("%s (%d failed checks)\n", failures ? "FAILED" : "clean", failures);
    return failures ? 1 : 0;
}
