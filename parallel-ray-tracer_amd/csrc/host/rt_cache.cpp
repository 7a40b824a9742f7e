// rt_cache.cpp — binary scene cache: triangles_load's and bvh_build's outputs stored as
// raw records, so that re-loading an unchanged scene reads ~100 B per triangle instead of parsing text
// (871k triangles: ~0.85 s parse + ~1.8 s heuristic-3 build) — results byte-identical by construction.
//
// File: "PRTCACHE" | u32 version | u32 kind | u64 key | u64 count | u64 extra | payload | u64 check
// key = hash of everything the result depends on (file bytes; triangles + heuristic + RNG state);
// check = hash of the payload. Anything that does not match (stale, foreign, truncated, corrupt) is
// ignored and rebuilt: the cache can only ever return what the uncached call would.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt_host.h"

namespace {

constexpr char MAGIC[8] = {'P', 'R', 'T', 'C', 'A', 'C', 'H', 'E'};
constexpr uint32_t VERSION = 1, KIND_TRIS = 1, KIND_BVH = 2;

// 64-bit multiply-xorshift hash over 8-byte words (fast; not cryptographic — it detects change)
uint64_t mix(uint64_t h, uint64_t v) {
    h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 0xBF58476D1CE4E5B9ull;
    return h ^ (h >> 31);
}
uint64_t hash_bytes(const void* p, size_t n, uint64_t h) {
    const unsigned char* b = (const unsigned char*)p;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t v;
        std::memcpy(&v, b + i, 8);
        h = mix(h, v);
    }
    uint64_t t = 0;
    std::memcpy(&t, b + i, n - i);
    return mix(mix(h, t), n);
}

bool read_file(const char* path, std::vector<unsigned char>& out) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    out.resize(sz > 0 ? (size_t)sz : 0);
    const bool ok = sz >= 0 && std::fread(out.data(), 1, out.size(), f) == out.size();
    std::fclose(f);
    return ok;
}

struct Header {
    char magic[8];
    uint32_t version, kind;
    uint64_t key, count, extra;
};

// payload of a valid cache entry of `kind` and `key`, or false
bool cache_get(const char* path, uint32_t kind, uint64_t key, std::vector<unsigned char>& payload, Header& h) {
    std::vector<unsigned char> all;
    if (!path || !read_file(path, all) || all.size() < sizeof(Header) + 8) return false;
    std::memcpy(&h, all.data(), sizeof h);
    if (std::memcmp(h.magic, MAGIC, 8) || h.version != VERSION || h.kind != kind || h.key != key) return false;
    const size_t n = all.size() - sizeof(Header) - 8;
    uint64_t check;
    std::memcpy(&check, all.data() + sizeof(Header) + n, 8);
    if (hash_bytes(all.data() + sizeof(Header), n, 7) != check) return false;
    payload.assign(all.begin() + sizeof(Header), all.begin() + sizeof(Header) + n);
    return true;
}

void cache_put(const char* path, uint32_t kind, uint64_t key, uint64_t count, uint64_t extra,
               const std::vector<const void*>& parts, const std::vector<size_t>& sizes) {
    if (!path) return;
    const std::string tmp = std::string(path) + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return;  // a cache that cannot be written is simply not used
    Header h;
    std::memcpy(h.magic, MAGIC, 8);
    h.version = VERSION;
    h.kind = kind;
    h.key = key;
    h.count = count;
    h.extra = extra;
    bool ok = std::fwrite(&h, sizeof h, 1, f) == 1;
    std::vector<unsigned char> payload;
    for (size_t i = 0; i < parts.size(); i++)
        payload.insert(payload.end(), (const unsigned char*)parts[i], (const unsigned char*)parts[i] + sizes[i]);
    const uint64_t check = hash_bytes(payload.data(), payload.size(), 7);
    ok = ok && std::fwrite(payload.data(), 1, payload.size(), f) == payload.size();
    ok = ok && std::fwrite(&check, 8, 1, f) == 1;
    ok = std::fclose(f) == 0 && ok;
    if (ok) std::rename(tmp.c_str(), path);  // atomic replace: readers never see a half-written cache
    else std::remove(tmp.c_str());
}

}  // namespace

extern "C" int rth_triangles_load_cached(const char* obj, const char* mtl, const char* cache, rt_triangle** out,
                                         size_t* n, int* from_cache) {
    if (!obj || !mtl || !out || !n) return RT_E_ARG;
    if (from_cache) *from_cache = 0;
    std::vector<unsigned char> ob, mb;
    if (!read_file(obj, ob)) return rth_triangles_load(obj, mtl, out, n);  // the loader reports the error
    const bool have_mtl = read_file(mtl, mb);
    uint64_t key = hash_bytes(ob.data(), ob.size(), 1);
    key = have_mtl ? hash_bytes(mb.data(), mb.size(), key) : mix(key, 0xA11CE);
    std::vector<unsigned char> pl;
    Header h;
    if (cache && cache_get(cache, KIND_TRIS, key, pl, h) && pl.size() == h.count * sizeof(rt_triangle)) {
        rt_triangle* t = (rt_triangle*)std::malloc(std::max<size_t>(pl.size(), 1));
        if (!t) return RT_E_NOMEM;
        std::memcpy(t, pl.data(), pl.size());
        *out = t;
        *n = h.count;
        if (from_cache) *from_cache = 1;
        return RT_OK;
    }
    const int rc = rth_triangles_load(obj, mtl, out, n);
    if (rc == RT_OK) cache_put(cache, KIND_TRIS, key, *n, 0, {*out}, {*n * sizeof(rt_triangle)});
    return rc;
}

extern "C" int rth_bvh_build_cached(const rt_triangle* tris, size_t n, int heuristic, rth_rng* g, const char* cache,
                                    rt_bvh_node** nodes, int* bvh_len, int** tri_idx, rth_bvh_stats* stats,
                                    int* from_cache) {
    if (!tris || !nodes || !bvh_len || !tri_idx) return RT_E_ARG;
    if (from_cache) *from_cache = 0;
    uint64_t key = hash_bytes(tris, n * sizeof(rt_triangle), 2);
    key = mix(key, (uint64_t)(int64_t)heuristic);
    key = g ? hash_bytes(g, sizeof *g, key) : mix(key, 0x5EED);
    std::vector<unsigned char> pl;
    Header h;
    if (cache && cache_get(cache, KIND_BVH, key, pl, h)) {
        const size_t len = h.count;
        const size_t need = len * sizeof(rt_bvh_node) + n * sizeof(int) + sizeof(rth_bvh_stats) + sizeof(rth_rng);
        if (pl.size() == need && len > 0) {
            rt_bvh_node* nd = (rt_bvh_node*)std::malloc(len * sizeof(rt_bvh_node));
            int* ix = (int*)std::malloc(std::max<size_t>(n, 1) * sizeof(int));
            if (!nd || !ix) {
                std::free(nd);
                std::free(ix);
                return RT_E_NOMEM;
            }
            const unsigned char* p = pl.data();
            std::memcpy(nd, p, len * sizeof(rt_bvh_node));
            p += len * sizeof(rt_bvh_node);
            std::memcpy(ix, p, n * sizeof(int));
            p += n * sizeof(int);
            if (stats) std::memcpy(stats, p, sizeof(rth_bvh_stats));
            p += sizeof(rth_bvh_stats);
            if (g) std::memcpy(g, p, sizeof(rth_rng));  // the RNG continues as after a real build
            *nodes = nd;
            *bvh_len = (int)len;
            *tri_idx = ix;
            if (from_cache) *from_cache = 1;
            return RT_OK;
        }
    }
    rth_bvh_stats st{};
    const int rc = rth_bvh_build(tris, n, heuristic, g, nodes, bvh_len, tri_idx, &st);
    if (rc != RT_OK) return rc;
    if (stats) *stats = st;
    rth_rng after{};
    if (g) after = *g;
    cache_put(cache, KIND_BVH, key, (uint64_t)*bvh_len, 0, {*nodes, *tri_idx, &st, &after},
              {(size_t)*bvh_len * sizeof(rt_bvh_node), n * sizeof(int), sizeof st, sizeof after});
    return RT_OK;
}
