// kd_cache.cpp -- on-disk cache of the host KD build.
//
// The KD build (KDTree.hpp:58-287 semantics, host_model.cpp build_kdtree) is
// a pure function of the kd-ordered triangle vertices: for the 70 k-triangle
// C4 mesh it takes ~1.5 s of every process start, the rest of scene creation
// ~0.1 s.  The cache keys a file on two independent 64-bit hashes of those
// vertex bytes (plus the builder version) and stores the flattened nodes,
// leaf ids and depth.  A file is used only if its header, both keys, the
// payload checksum and a structural check (valid_tree: sibling pairs in
// range, a tree of depth <= 32 equal to the header's, leaf ranges and ids in
// range) all pass -- anything else rebuilds and rewrites it, so a stale,
// truncated or foreign file can cost time but never change or break a render.  Writes go
// to a temporary file renamed into place (concurrent processes see either
// the old file or the whole new one).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <unistd.h>

#include "host_model.hpp"
#include "../../include/mcpt.h"

namespace mcpt {
namespace {

// bump whenever build_kdtree's output for the same input can change; the SAH
// rule (MCPT_KD_BUILD_SAH) has its own id, so its files never match a
// reference-rule lookup and vice versa
constexpr uint32_t kBuilderVersion = 1;
constexpr uint32_t kSahBuilderVersion = 0x5A480001u;
uint32_t builder_id(int kd_build) { return kd_build == MCPT_KD_BUILD_SAH ? kSahBuilderVersion : kBuilderVersion; }
constexpr char kMagic[8] = {'M', 'C', 'P', 'T', 'K', 'D', 'C', '1'};
constexpr uint32_t kNodeWords = 12;   // left right bmin[3] bmax[3] axis split leaf_begin leaf_count
constexpr int32_t kMaxKdDepth = 32;   // build_kdtree's cap (KDTree.hpp:103-106)

struct Header {
    char magic[8];
    uint32_t version, node_words;
    uint64_t n_tris, key_a, key_b;
    uint64_t n_nodes, n_leaf_ids;
    int32_t depth;
    uint32_t pad;
    uint64_t payload_hash;
};
static_assert(sizeof(Header) == 72, "cache header layout");

// FNV-1a 64 over bytes from a given offset basis
uint64_t fnv1a(const void* data, size_t n, uint64_t h) {
    const unsigned char* p = static_cast<const unsigned char*>(data);
    for (size_t i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 0x100000001B3ull;
    }
    return h;
}

void keys(const std::vector<float>& tv, uint32_t builder, uint64_t& a, uint64_t& b) {
    const uint64_t n = tv.size() / 9;
    a = fnv1a(&builder, 4, fnv1a(&n, 8, 0xCBF29CE484222325ull));
    a = fnv1a(tv.data(), tv.size() * 4, a);
    b = fnv1a(&n, 8, fnv1a(&builder, 4, 0x84222325CBF29CE4ull));
    // second key over the words in reverse order: independent of the first
    for (size_t i = tv.size(); i-- > 0;) b = fnv1a(&tv[i], 4, b);
}

std::string path_for(const std::string& dir, uint64_t key_a) {
    char name[64];
    std::snprintf(name, sizeof name, "/mcpt-kd-%016llx.bin", static_cast<unsigned long long>(key_a));
    return dir + name;
}

void pack(const std::vector<KdNode>& nodes, std::vector<uint32_t>& words) {
    words.resize(nodes.size() * kNodeWords);
    for (size_t i = 0; i < nodes.size(); ++i) {
        const KdNode& n = nodes[i];
        uint32_t* w = &words[i * kNodeWords];
        w[0] = n.left;
        w[1] = n.right;
        std::memcpy(w + 2, n.bmin, 12);
        std::memcpy(w + 5, n.bmax, 12);
        w[8] = n.axis;
        std::memcpy(w + 9, &n.split, 4);
        w[10] = n.leaf_begin;
        w[11] = n.leaf_count;
    }
}

// Structure the consumers rely on: capi.cpp device_order/build_image read
// nodes[left + 1] as the right sibling and write node_new[left + 1]; the
// traversal's stack spill area holds 32 entries per lane (the builder's depth
// cap, KDTree.hpp:103-106).  So: every inner node's children are the pair
// (left, left + 1) with left odd and both in range, every node but the root
// has exactly one parent (a tree, no shared subtrees), the real depth equals
// the header's and is <= 32, and leaf ranges / ids stay inside their arrays.
// The keys and checksums are public, so a crafted file must fail here.
bool valid_tree(const std::vector<uint32_t>& w, const std::vector<uint32_t>& leaf_ids, uint64_t n_tris,
                int32_t depth) {
    const size_t nn = w.size() / kNodeWords;
    if (nn == 0 || depth < 0 || depth > kMaxKdDepth) return false;
    std::vector<uint8_t> parents(nn, 0);
    std::vector<int32_t> node_depth(nn, -1);
    node_depth[0] = 0;
    int32_t max_depth = 0;
    for (size_t i = 0; i < nn; ++i) {
        const uint32_t* n = &w[i * kNodeWords];
        if (n[8] > 3) return false;
        if (node_depth[i] < 0) return false;     // unreachable (children point forward: parents come first)
        max_depth = std::max(max_depth, node_depth[i]);
        if (n[8]) {
            const uint64_t L = n[0];
            if (L <= i || (L & 1u) != 1u || uint64_t(n[1]) != L + 1 || L + 1 >= nn) return false;
            if (parents[L]++ || parents[L + 1]++) return false;
            node_depth[L] = node_depth[L + 1] = node_depth[i] + 1;
            if (node_depth[i] + 1 > kMaxKdDepth) return false;
        } else if (uint64_t(n[10]) + n[11] > leaf_ids.size()) {
            return false;
        }
    }
    if (max_depth != depth) return false;
    for (uint32_t id : leaf_ids)
        if (id >= n_tris) return false;
    return true;
}

}  // namespace

bool kd_cache_load(const std::string& dir, const std::vector<float>& tv, std::vector<KdNode>& nodes,
                   std::vector<uint32_t>& leaf_ids, int& depth, int kd_build) {
    const uint32_t builder = builder_id(kd_build);
    uint64_t ka, kb;
    keys(tv, builder, ka, kb);
    FILE* f = std::fopen(path_for(dir, ka).c_str(), "rb");
    if (!f) return false;
    Header h{};
    std::vector<uint32_t> w, ids;
    bool ok = std::fread(&h, sizeof h, 1, f) == 1 && std::memcmp(h.magic, kMagic, 8) == 0 &&
              h.version == builder && h.node_words == kNodeWords && h.n_tris == tv.size() / 9 &&
              h.key_a == ka && h.key_b == kb && h.n_nodes > 0 && h.n_nodes < (1ull << 31) &&
              h.n_leaf_ids < (1ull << 31) && h.depth >= 0 && h.depth <= kMaxKdDepth;
    if (ok) {
        // the payload must be exactly what the header announces: checked against
        // the file size before anything is allocated (a crafted header cannot make
        // the reader reserve up to 2^31 x 48 B)
        const uint64_t want = sizeof(Header) + h.n_nodes * kNodeWords * 4 + h.n_leaf_ids * 4;
        ok = std::fseek(f, 0, SEEK_END) == 0 && std::ftell(f) >= 0 && uint64_t(std::ftell(f)) == want &&
             std::fseek(f, long(sizeof(Header)), SEEK_SET) == 0;
    }
    if (ok) {
        w.resize(size_t(h.n_nodes) * kNodeWords);
        ids.resize(size_t(h.n_leaf_ids));
        ok = std::fread(w.data(), 4, w.size(), f) == w.size() && std::fread(ids.data(), 4, ids.size(), f) == ids.size();
        char extra;
        ok = ok && std::fread(&extra, 1, 1, f) == 0;   // exactly the payload, nothing after it
    }
    std::fclose(f);
    if (!ok) return false;
    const uint64_t ph = fnv1a(ids.data(), ids.size() * 4, fnv1a(w.data(), w.size() * 4, 0xCBF29CE484222325ull));
    if (ph != h.payload_hash || !valid_tree(w, ids, h.n_tris, h.depth)) return false;
    nodes.assign(size_t(h.n_nodes), KdNode());
    for (size_t i = 0; i < nodes.size(); ++i) {
        const uint32_t* s = &w[i * kNodeWords];
        KdNode& n = nodes[i];
        n.left = s[0];
        n.right = s[1];
        std::memcpy(n.bmin, s + 2, 12);
        std::memcpy(n.bmax, s + 5, 12);
        n.axis = s[8];
        std::memcpy(&n.split, s + 9, 4);
        n.leaf_begin = s[10];
        n.leaf_count = s[11];
    }
    leaf_ids.swap(ids);
    depth = h.depth;
    return true;
}

bool kd_cache_store(const std::string& dir, const std::vector<float>& tv, const std::vector<KdNode>& nodes,
                    const std::vector<uint32_t>& leaf_ids, int depth, int kd_build) {
    Header h{};
    std::memcpy(h.magic, kMagic, 8);
    h.version = builder_id(kd_build);
    h.node_words = kNodeWords;
    h.n_tris = tv.size() / 9;
    keys(tv, h.version, h.key_a, h.key_b);
    h.n_nodes = nodes.size();
    h.n_leaf_ids = leaf_ids.size();
    h.depth = depth;
    std::vector<uint32_t> w;
    pack(nodes, w);
    h.payload_hash = fnv1a(leaf_ids.data(), leaf_ids.size() * 4, fnv1a(w.data(), w.size() * 4, 0xCBF29CE484222325ull));
    const std::string path = path_for(dir, h.key_a);
    const std::string tmp = path + ".tmp." + std::to_string(static_cast<long long>(getpid()));
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return false;
    bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 && std::fwrite(w.data(), 4, w.size(), f) == w.size() &&
              std::fwrite(leaf_ids.data(), 4, leaf_ids.size(), f) == leaf_ids.size();
    ok = (std::fclose(f) == 0) && ok;
    if (ok) ok = std::rename(tmp.c_str(), path.c_str()) == 0;
    if (!ok) std::remove(tmp.c_str());
    return ok;
}

}  // namespace mcpt
