// librt_host.so — host half of the drop-in (include/rt_host.h): scene loader, camera, BVH builders,
// random-triangle mode and BMP writer of the reference cpu/ renderer, restated in C++17.
//
// Floating point: this file must be compiled with -ffp-contract=off and without -ffast-math: every
// expression keeps the reference's operand order, so the triangles (normals, centroids), camera
// constants and BVH boxes are bit-identical to what the reference computes (tests/test_host.py).
#include "rt_host.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

// ------------------------------------------------------------------ vec (cpu/src/vec.c:4-69)
inline rt_vec3 V(float x, float y, float z) { return rt_vec3{x, y, z}; }
inline float dot(const rt_vec3& a, const rt_vec3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float mag(const rt_vec3& a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
inline rt_vec3 mul(const rt_vec3& a, float s) { return V(a.x * s, a.y * s, a.z * s); }
inline rt_vec3 add(const rt_vec3& a, const rt_vec3& b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
inline rt_vec3 sub(const rt_vec3& a, const rt_vec3& b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
inline rt_vec3 dv(const rt_vec3& a, float s) { return V(a.x / s, a.y / s, a.z / s); }
inline rt_vec3 cross(const rt_vec3& a, const rt_vec3& b) {
    return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline rt_vec3 normalize(const rt_vec3& a) { return dv(a, mag(a)); }
inline rt_vec3 vmin(const rt_vec3& a, const rt_vec3& b) {
    return V(std::fmin(a.x, b.x), std::fmin(a.y, b.y), std::fmin(a.z, b.z));
}
inline rt_vec3 vmax(const rt_vec3& a, const rt_vec3& b) {
    return V(std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z));
}
inline float comp(const rt_vec3& a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// fgets(buf, 256) line chunking, cpu/src/triangle.c:26-47
bool read_chunks(const char* path, std::vector<std::string>& out) {
    FILE* f = std::fopen(path, "r");
    if (!f) return false;
    char buf[256];
    while (std::fgets(buf, sizeof buf, f)) out.emplace_back(buf);
    std::fclose(f);
    return true;
}

struct Material {
    char name[256];
    rt_vec3 kd, ks, kr;
};

}  // namespace

// ------------------------------------------------------------------ rng (glibc random_r TYPE_3)
extern "C" void rth_srand(rth_rng* g, unsigned seed) {
    // glibc srandom_r: r[0] = seed (0 -> 1); r[i] = 16807 * r[i-1] mod (2^31 - 1); 310 discarded outputs
    int32_t r[344];
    r[0] = seed == 0 ? 1 : (int32_t)seed;
    for (int i = 1; i < 31; i++) {
        int64_t v = (16807LL * r[i - 1]) % 2147483647LL;
        if (v < 0) v += 2147483647LL;
        r[i] = (int32_t)v;
    }
    for (int i = 31; i < 34; i++) r[i] = r[i - 31];
    for (int i = 34; i < 344; i++) r[i] = (int32_t)((uint32_t)r[i - 31] + (uint32_t)r[i - 3]);
    for (int i = 0; i < 34; i++) g->r[i] = r[310 + i];
    g->pos = 0;  // next index into the 34-entry ring (holds r[k-34 .. k-1])
}

extern "C" int rth_rand(rth_rng* g) {
    // r[k] = r[k-31] + r[k-3]; ring slot k % 34 holds r[k-34]
    int k = g->pos;
    int32_t v = (int32_t)((uint32_t)g->r[(k + 3) % 34] + (uint32_t)g->r[(k + 31) % 34]);
    g->r[k] = v;
    g->pos = (k + 1) % 34;
    return (int)((uint32_t)v >> 1);
}

// ------------------------------------------------------------------ triangles / lights
extern "C" void rth_triangle_init(rt_triangle* t, const rt_vec3* a, const rt_vec3* b, const rt_vec3* c,
                                  const rt_vec3* ks, const rt_vec3* kd, const rt_vec3* kr) {
    // cpu/src/triangle.c:6-24
    t->coords[0] = *a;
    t->coords[1] = *b;
    t->coords[2] = *c;
    t->ks = *ks;
    t->kd = *kd;
    t->kr = *kr;
    rt_vec3 e1 = sub(t->coords[1], t->coords[0]);
    rt_vec3 e2 = sub(t->coords[2], t->coords[0]);
    t->norm[0] = normalize(cross(e1, e2));
    t->norm[1] = normalize(cross(e2, e1));
    t->centroid[0] = (t->coords[0].x + t->coords[1].x + t->coords[2].x) / 3.0f;
    t->centroid[1] = (t->coords[0].y + t->coords[1].y + t->coords[2].y) / 3.0f;
    t->centroid[2] = (t->coords[0].z + t->coords[1].z + t->coords[2].z) / 3.0f;
}

extern "C" int rth_triangles_load(const char* objname, const char* mtlname, rt_triangle** out, size_t* n) {
    if (!objname || !mtlname || !out || !n) return RT_E_ARG;
    std::vector<std::string> ol, ml;
    if (!read_chunks(objname, ol)) {
        std::printf("cannot load %s\n", objname);  // triangle.c:29
        return RT_E_IO;
    }
    if (!read_chunks(mtlname, ml)) {
        std::printf("cannot load %s\n", mtlname);
        return RT_E_IO;
    }
    std::vector<rt_vec3> verts;
    verts.reserve(ol.size());
    for (const std::string& l : ol)  // triangle.c:82-87
        if (l.size() >= 2 && l[0] == 'v' && l[1] == ' ') {
            rt_vec3 v{0, 0, 0};
            std::sscanf(l.c_str(), "v %f %f %f", &v.x, &v.y, &v.z);
            verts.push_back(v);
        }
    std::vector<Material> mats;  // triangle.c:54-72, max 128, unset keys = 0
    for (size_t i = 0; i < ml.size(); i++) {
        if (std::strncmp(ml[i].c_str(), "newmtl", 6) == 0 && mats.size() < 128) {
            Material m;
            std::memset(&m, 0, sizeof m);
            std::sscanf(ml[i].c_str(), "newmtl %255s", m.name);
            for (size_t j = i + 1; j < i + 6 && j < ml.size(); j++) {
                const char* s = ml[j].c_str();
                if (std::strncmp(s, "Kd", 2) == 0) std::sscanf(s, "Kd %f %f %f", &m.kd.x, &m.kd.y, &m.kd.z);
                else if (std::strncmp(s, "Ks", 2) == 0) std::sscanf(s, "Ks %f %f %f", &m.ks.x, &m.ks.y, &m.ks.z);
                else if (std::strncmp(s, "Kr", 2) == 0) std::sscanf(s, "Kr %f %f %f", &m.kr.x, &m.kr.y, &m.kr.z);
            }
            mats.push_back(m);
        }
    }
    rt_vec3 cks{0, 0, 0}, ckd{0, 0, 0}, ckr{0, 0, 0};  // triangle.c:92
    std::vector<rt_triangle> tris;
    for (const std::string& l : ol) {  // triangle.c:96-115
        if (std::strncmp(l.c_str(), "usemtl", 6) == 0) {
            char name[256] = {0};
            std::sscanf(l.c_str(), "usemtl %255s", name);
            for (const Material& m : mats)
                if (std::strcmp(name, m.name) == 0) {
                    ckd = m.kd;
                    cks = m.ks;
                    ckr = m.kr;
                    break;
                }
        } else if (!l.empty() && l[0] == 'f') {
            int a = 0, b = 0, c = 0;
            std::sscanf(l.c_str(), "f %d %d %d", &a, &b, &c);
            if (a < 1 || b < 1 || c < 1 || (size_t)a > verts.size() || (size_t)b > verts.size() ||
                (size_t)c > verts.size())
                return RT_E_ARG;  // the reference reads out of bounds here; we refuse instead
            rt_triangle t;
            rth_triangle_init(&t, &verts[a - 1], &verts[b - 1], &verts[c - 1], &cks, &ckd, &ckr);
            tris.push_back(t);
        }
    }
    rt_triangle* buf = (rt_triangle*)std::malloc(sizeof(rt_triangle) * (tris.empty() ? 1 : tris.size()));
    if (!buf) return RT_E_NOMEM;
    if (!tris.empty()) std::memcpy(buf, tris.data(), sizeof(rt_triangle) * tris.size());
    *out = buf;
    *n = tris.size();
    return RT_OK;
}

extern "C" int rth_lights_load(const char* path, rt_light** out, size_t* n) {
    if (!path || !out || !n) return RT_E_ARG;
    FILE* f = std::fopen(path, "r");  // light.c:9-13
    if (!f) {
        std::printf("cannot open %s\n", path);
        return RT_E_IO;
    }
    std::vector<rt_light> ls;
    char line[256];
    while (std::fgets(line, sizeof line, f)) {  // light.c:18-24
        rt_light l;
        std::memset(&l, 0, sizeof l);
        std::sscanf(line, "%f %f %f %f %f %f", &l.pos.x, &l.pos.y, &l.pos.z, &l.kl.x, &l.kl.y, &l.kl.z);
        ls.push_back(l);
    }
    std::fclose(f);
    rt_light* buf = (rt_light*)std::malloc(sizeof(rt_light) * (ls.empty() ? 1 : ls.size()));
    if (!buf) return RT_E_NOMEM;
    if (!ls.empty()) std::memcpy(buf, ls.data(), sizeof(rt_light) * ls.size());
    *out = buf;
    *n = ls.size();
    return RT_OK;
}

extern "C" int rth_triangles_random(size_t n, rth_rng* g, rt_triangle** out) {
    // cpu/src/main.c:116-130: a in [-5,5)^3, b = a + r1, c = b + r2; ks = 1, kd = kr = 0
    if (!g || !out) return RT_E_ARG;
    rt_triangle* t = (rt_triangle*)std::malloc(sizeof(rt_triangle) * (n ? n : 1));
    if (!t) return RT_E_NOMEM;
    const float RM = (float)RAND_MAX;
    for (size_t i = 0; i < n; i++) {
        rt_vec3 v0{0.0f, 0.0f, 0.0f}, v1{1.0f, 1.0f, 1.0f};
        float r[9];
        for (int k = 0; k < 9; k++) r[k] = (float)rth_rand(g) / RM;
        rt_vec3 r0{r[0], r[1], r[2]}, r1{r[3], r[4], r[5]}, r2{r[6], r[7], r[8]};
        rt_vec3 a = mul(r0, 10);
        a.x -= 5;
        a.y -= 5;
        a.z -= 5;
        rt_vec3 b = add(a, r1);
        rt_vec3 c = add(b, r2);
        rth_triangle_init(&t[i], &a, &b, &c, &v1, &v0, &v0);
    }
    *out = t;
    return RT_OK;
}

// ------------------------------------------------------------------ BVH (cpu/src/bvh.c)
namespace {

struct Builder {
    const rt_triangle* tris;
    int n;
    int heuristic;
    rth_rng* g;
    std::vector<rt_bvh_node> bvh;
    std::vector<int> idx;
    int len = 1;
    rth_bvh_stats st{};

    void grow(rt_vec3& mn, rt_vec3& mx, int t) const {  // bvh.c:61-71
        for (int k = 0; k < 3; k++) {
            mn = vmin(mn, tris[t].coords[k]);
            mx = vmax(mx, tris[t].coords[k]);
        }
    }
    // partition key: centroid[axis]; "centroid[3]" is the next float of triangle_t, ks.r
    float key(int t, int axis) const { return axis == 3 ? tris[t].ks.x : tris[t].centroid[axis]; }
    void leaf_stats(const rt_bvh_node& p, int depth) {  // bvh.c:87-94
        st.leaves++;
        st.avg_leaf += p.tr_len;
        st.min_leaf = std::min(st.min_leaf, p.tr_len);
        st.max_leaf = std::max(st.max_leaf, p.tr_len);
        st.max_depth = std::max(st.max_depth, depth);
    }

    // bvh.c:78-267, reference heuristics 0, 1, 3, 6 (recursive descent, children allocated in pairs)
    void split(int ni, int depth) {
        rt_bvh_node* p = &bvh[ni];
        if (len >= 2 * n) return;  // "BVH SPLIT: MAX SIZE REACHED", bvh.c:80-83
        if (depth == 32 || p->tr_len <= 2) {
            if (!p->tr_len) p->child = 0;
            leaf_stats(*p, depth);
            return;
        }
        int ci = len;
        len += 2;
        rt_bvh_node* L = &bvh[ci];
        rt_bvh_node* R = &bvh[ci + 1];
        L->child = p->child;
        L->min = V(1e10f, 1e10f, 1e10f);
        L->max = V(-1e10f, -1e10f, -1e10f);
        R->child = p->child;
        R->min = V(1e10f, 1e10f, 1e10f);
        R->max = V(-1e10f, -1e10f, -1e10f);
        int axis = 0;
        float pos = 0;
        rt_vec3 center = mul(add(p->min, p->max), 0.5f);  // aabb_center, bvh.c:38-41
        rt_vec3 size = sub(p->max, p->min);
        if (heuristic == 6) {  // bvh.c:138-177
            float best = FLT_MAX;
            for (int a = 0; a < 3; a++)
                for (int i = 0; i < 32; i++) {
                    rt_vec3 lmn = V(FLT_MAX, FLT_MAX, FLT_MAX), lmx = V(FLT_MIN, FLT_MIN, FLT_MIN);
                    rt_vec3 rmn = lmn, rmx = lmx;
                    float sp = comp(p->min, a) + comp(size, a) * ((float)i / 32);
                    int cl = 0, cr = 0;
                    for (int j = p->child; j < p->child + p->tr_len; j++) {
                        int t = idx[j];
                        if (tris[t].centroid[a] < sp) {
                            grow(lmn, lmx, t);
                            cl++;
                        } else {
                            grow(rmn, rmx, t);
                            cr++;
                        }
                    }
                    rt_vec3 sl = sub(lmx, lmn), sr = sub(rmx, rmn);
                    float score = cl * dot(sl, sl) + cr * dot(sr, sr);  // aabb_area = |diag|^2, bvh.c:43-46
                    if (score < best) {
                        best = score;
                        axis = a;
                        pos = sp;
                    }
                }
        } else if (heuristic == 3) {  // bvh.c:228-241
            bool okA = false, okB = false;
            while (!okA || !okB) {
                okA = okB = false;
                axis = rth_rand(g) % 4;
                if (axis == 3) {
                    // rand() % 4 == 3 reads center.arr[3], size.arr[3] and centroid[3] past their arrays
                    // (bvh.c:229-231,237,247). Restated as the reference's O-strict build (gcc -O2) lays
                    // them out: center.arr[3] = size.x, size.arr[3] = (min + max).x, centroid[3] = ks.r.
                    pos = size.x;
                    pos += ((float)rth_rand(g) / (float)RAND_MAX - 0.5f) * (p->min.x + p->max.x);
                } else {
                    pos = comp(center, axis);
                    pos += ((float)rth_rand(g) / (float)RAND_MAX - 0.5f) * (comp(size, axis));
                }
                for (int i = p->child; i < p->child + p->tr_len && (!okA || !okB); i++) {
                    bool inA = key(idx[i], axis) < pos;
                    okA |= inA;
                    okB |= !inA;
                }
            }
        } else {  // 0: axis 0 centre, 1: largest axis centre (bvh.c:214-223)
            axis = 0;
            if (heuristic == 1) {
                if (size.y > size.x) axis = 1;
                if (size.z > size.x && size.z > size.y) axis = 2;
            }
            pos = comp(center, axis);
        }
        for (int i = p->child; i < p->child + p->tr_len; i++) {  // bvh.c:244-259
            int t = idx[i];
            bool inA = key(t, axis) < pos;
            rt_bvh_node* c = inA ? L : R;
            grow(c->min, c->max, t);
            c->tr_len += 1;
            if (inA) {
                int sw = L->child + L->tr_len - 1;
                std::swap(idx[i], idx[sw]);
                R->child += 1;
            }
        }
        p->child = ci;
        p->tr_len = 0;
        split(ci, depth + 1);
        split(ci + 1, depth + 1);
    }

    // ---- RTH_BVH_BINNED_SAH: O(n log n) binned SAH (surface area), leaves <= 4 (8 if cheaper),
    // depth <= 32. Same output layout as the reference builder.
    static float area(const rt_vec3& mn, const rt_vec3& mx) {
        float dx = mx.x - mn.x, dy = mx.y - mn.y, dz = mx.z - mn.z;
        if (dx < 0 || dy < 0 || dz < 0) return 0.0f;
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
    // depth cap 24: the fast kernels stack only deferred far children, at most depth entries (26 slots)
    static constexpr int SAH_MAX_DEPTH = 24;
    std::vector<float> cen;  // centroid x,y,z per triangle (copied from triangle_t.centroid)
    std::vector<float> tb;   // per-triangle box lo.xyz, hi.xyz (the SAH path only; plain min/max)
    static rt_vec3 fmin3(const rt_vec3& a, const rt_vec3& b) {
        return V(std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z));
    }
    static rt_vec3 fmax3(const rt_vec3& a, const rt_vec3& b) {
        return V(std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z));
    }
    void grow_sah(rt_vec3& mn, rt_vec3& mx, int t) const {
        const float* b = &tb[6 * (size_t)t];
        mn.x = std::min(mn.x, b[0]);
        mn.y = std::min(mn.y, b[1]);
        mn.z = std::min(mn.z, b[2]);
        mx.x = std::max(mx.x, b[3]);
        mx.y = std::max(mx.y, b[4]);
        mx.z = std::max(mx.z, b[5]);
    }

    void sah_split(int ni, int depth) {
        rt_bvh_node* p = &bvh[ni];
        const int first = p->child, cnt = p->tr_len;
        if (cnt <= 2 || depth == SAH_MAX_DEPTH || len + 2 > 2 * n) {
            leaf_stats(*p, depth);
            return;
        }
        // centroid bounds
        float cmn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, cmx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (int i = first; i < first + cnt; i++)
            for (int a = 0; a < 3; a++) {
                float c = cen[3 * idx[i] + a];
                cmn[a] = std::min(cmn[a], c);
                cmx[a] = std::max(cmx[a], c);
            }
        // 32 bins, or about one per triangle in small nodes (the per-node sweeps dominate otherwise)
        constexpr int NBMAX = 32;
        const int NB = cnt >= NBMAX ? NBMAX : std::max(4, cnt);
        float best = FLT_MAX;
        int best_axis = -1, best_bin = -1;
        for (int a = 0; a < 3; a++) {
            float ext = cmx[a] - cmn[a];
            if (!(ext > 0)) continue;
            rt_vec3 bmn[NBMAX], bmx[NBMAX];
            int bc[NBMAX] = {0};
            for (int b = 0; b < NB; b++) {
                bmn[b] = V(FLT_MAX, FLT_MAX, FLT_MAX);
                bmx[b] = V(-FLT_MAX, -FLT_MAX, -FLT_MAX);
            }
            const float sc = NB / ext;
            for (int i = first; i < first + cnt; i++) {
                int t = idx[i];
                int b = std::min(NB - 1, (int)((cen[3 * t + a] - cmn[a]) * sc));
                bc[b]++;
                grow_sah(bmn[b], bmx[b], t);
            }
            float rA[NBMAX];
            int rN[NBMAX];
            rt_vec3 mn = V(FLT_MAX, FLT_MAX, FLT_MAX), mx = V(-FLT_MAX, -FLT_MAX, -FLT_MAX);
            int acc = 0;
            for (int b = NB - 1; b > 0; b--) {
                acc += bc[b];
                mn = fmin3(mn, bmn[b]);
                mx = fmax3(mx, bmx[b]);
                rA[b] = area(mn, mx);
                rN[b] = acc;
            }
            mn = V(FLT_MAX, FLT_MAX, FLT_MAX);
            mx = V(-FLT_MAX, -FLT_MAX, -FLT_MAX);
            acc = 0;
            for (int b = 0; b < NB - 1; b++) {
                acc += bc[b];
                mn = fmin3(mn, bmn[b]);
                mx = fmax3(mx, bmx[b]);
                if (acc == 0 || rN[b + 1] == 0) continue;
                float cost = area(mn, mx) * acc + rA[b + 1] * rN[b + 1];
                if (cost < best) {
                    best = cost;
                    best_axis = a;
                    best_bin = b;
                }
            }
        }
        // SAH termination: traversal cost 1, intersection cost 1 (in units of parent area)
        float leaf_cost = (float)cnt * area(p->min, p->max);
        int mid;
        if (best_axis < 0) {  // all centroids coincide: object-median split
            if (cnt <= 4) {
                leaf_stats(*p, depth);
                return;
            }
            mid = first + cnt / 2;
        } else {
            if (cnt <= 8 && best + area(p->min, p->max) >= leaf_cost) {
                leaf_stats(*p, depth);
                return;
            }
            const int a = best_axis;
            const float ext = cmx[a] - cmn[a], sc = NB / ext, lo = cmn[a];
            int* beg = idx.data() + first;
            int* m = std::partition(beg, beg + cnt, [&](int t) {
                return std::min(NB - 1, (int)((cen[3 * t + a] - lo) * sc)) <= best_bin;
            });
            mid = (int)(m - idx.data());
            if (mid == first || mid == first + cnt) mid = first + cnt / 2;
        }
        int ci = len;
        len += 2;
        p = &bvh[ni];
        rt_bvh_node* L = &bvh[ci];
        rt_bvh_node* R = &bvh[ci + 1];
        L->child = first;
        L->tr_len = mid - first;
        R->child = mid;
        R->tr_len = first + cnt - mid;
        for (rt_bvh_node* c : {L, R}) {
            c->min = V(1e10f, 1e10f, 1e10f);
            c->max = V(-1e10f, -1e10f, -1e10f);
            for (int i = c->child; i < c->child + c->tr_len; i++) grow_sah(c->min, c->max, idx[i]);
        }
        p->child = ci;
        p->tr_len = 0;
        sah_split(ci, depth + 1);
        sah_split(ci + 1, depth + 1);
    }
};

}  // namespace

extern "C" int rth_bvh_build(const rt_triangle* tris, size_t n, int heuristic, rth_rng* g, rt_bvh_node** nodes,
                             int* bvh_len, int** tri_idx, rth_bvh_stats* stats) {
    if (!n) {
        std::printf("no triangles, cannot build bvh.\n");  // bvh.c:361-364
        return RT_E_EMPTY;
    }
    if (!tris || !nodes || !bvh_len || !tri_idx || n > (size_t)(1 << 29)) return RT_E_ARG;
    if (heuristic != 0 && heuristic != 1 && heuristic != 3 && heuristic != 6 && heuristic != RTH_BVH_BINNED_SAH)
        return RT_E_ARG;
    if (heuristic == 3 && !g) return RT_E_ARG;
    Builder b;
    b.tris = tris;
    b.n = (int)n;
    b.heuristic = heuristic;
    b.g = g;
    b.st.min_leaf = INT32_MAX;
    b.st.max_leaf = INT32_MIN;
    b.bvh.assign(2 * n + 2, rt_bvh_node{});  // bvh.c:370-371 (memset 0)
    b.idx.resize(n);
    for (size_t i = 0; i < n; i++) b.idx[i] = (int)i;
    rt_bvh_node& root = b.bvh[0];  // bvh.c:372-377
    root.tr_len = (int)n;
    root.min = V(1e10f, 1e10f, 1e10f);
    root.max = V(-1e10f, -1e10f, -1e10f);
    for (size_t i = 0; i < n; i++) b.grow(root.min, root.max, (int)i);
    if (heuristic == RTH_BVH_BINNED_SAH) {
        b.cen.resize(3 * n);
        b.tb.resize(6 * n);
        for (size_t i = 0; i < n; i++) {
            for (int a = 0; a < 3; a++) b.cen[3 * i + a] = tris[i].centroid[a];
            rt_vec3 mn = tris[i].coords[0], mx = tris[i].coords[0];
            for (int k = 1; k < 3; k++) {
                const rt_vec3& c = tris[i].coords[k];
                mn = V(std::min(mn.x, c.x), std::min(mn.y, c.y), std::min(mn.z, c.z));
                mx = V(std::max(mx.x, c.x), std::max(mx.y, c.y), std::max(mx.z, c.z));
            }
            const float v[6] = {mn.x, mn.y, mn.z, mx.x, mx.y, mx.z};
            std::memcpy(&b.tb[6 * i], v, sizeof v);
        }
        b.sah_split(0, 0);
    } else {
        b.split(0, 0);
    }
    rt_bvh_node* out = (rt_bvh_node*)std::malloc(sizeof(rt_bvh_node) * b.len);
    int* ti = (int*)std::malloc(sizeof(int) * n);
    if (!out || !ti) {
        std::free(out);
        std::free(ti);
        return RT_E_NOMEM;
    }
    std::memcpy(out, b.bvh.data(), sizeof(rt_bvh_node) * b.len);
    std::memcpy(ti, b.idx.data(), sizeof(int) * n);
    *nodes = out;
    *bvh_len = b.len;
    *tri_idx = ti;
    if (stats) {
        *stats = b.st;
        stats->avg_leaf = b.st.leaves ? b.st.avg_leaf / b.st.leaves : 0.0;
    }
    return RT_OK;
}

// ------------------------------------------------------------------ camera (cam.c, main.c)
extern "C" int rth_camera(int W, int H, rt_camera* out) {
    if (W <= 0 || H <= 0 || !out) return RT_E_ARG;
    const double PI = 3.14159265358979323846;
    const rt_vec3 pos{0, -9, 3};
    float fov_arg = (float)(PI / 3.2);                 // cam_init(&cam, &pos, M_PI/3.2)
    float fov = (float)(1.0 / std::tan(fov_arg / 2.0f));  // cam.c:8: 1.0/tanf(fov/2.0f)
    // tanf: std::tan(float) is tanf
    rt_vec3 rot{(float)(-PI / 12), 0, 0};              // main.c:106
    float ar = (float)W / H;
    rt_vec3 sp[3] = {V(-1 * ar, fov, +1), V(+1 * ar, fov, +1), V(-1 * ar, fov, -1)};  // cam.c:36-38
    for (rt_vec3& p : sp) {
        rt_vec3 t = p;  // cam_rotateY, cam.c:23-27
        p.x = t.x * std::cos(rot.y) + t.z * std::sin(rot.y);
        p.z = -t.x * std::sin(rot.y) + t.z * std::cos(rot.y);
        t = p;  // cam_rotateX, cam.c:17-21
        p.y = t.y * std::cos(rot.x) - t.z * std::sin(rot.x);
        p.z = t.y * std::sin(rot.x) + t.z * std::cos(rot.x);
        t = p;  // cam_rotateZ, cam.c:29-33
        p.x = t.x * std::cos(rot.z) - t.y * std::sin(rot.z);
        p.y = t.x * std::sin(rot.z) + t.y * std::cos(rot.z);
        p = add(p, pos);  // cam.c:44-46
    }
    out->pos = pos;
    out->ul = sp[0];
    out->inc_x = dv(sub(sp[1], sp[0]), (float)W);  // main.c:247-248
    out->inc_y = dv(sub(sp[2], sp[0]), (float)H);  // main.c:249-250
    return RT_OK;
}

// ------------------------------------------------------------------ BMP (cpu/src/bmp_writer.c)
extern "C" int rth_bmp_header(int W, int H, uint8_t* buf) {
    if (W <= 0 || H <= 0 || !buf) return RT_E_ARG;
    const int row = W * 4, hdr = 14 + 40;
    const size_t fsz = (size_t)hdr + (size_t)row * H;
    std::memset(buf, 0, hdr);
    int file_size = (int)fsz, hs = hdr, dib = 40;
    uint16_t planes = 1, bpp = 32;
    uint32_t comp = 0;
    buf[0] = 'B';  // bmp_writer.c:97-104
    buf[1] = 'M';
    std::memcpy(buf + 0x02, &file_size, 4);
    std::memcpy(buf + 0x0A, &hs, 4);
    std::memcpy(buf + 0x0E, &dib, 4);  // bmp_writer.c:107-120
    std::memcpy(buf + 0x12, &W, 4);
    std::memcpy(buf + 0x16, &H, 4);
    std::memcpy(buf + 0x1A, &planes, 2);
    std::memcpy(buf + 0x1C, &bpp, 2);
    std::memcpy(buf + 0x1E, &comp, 4);
    return RT_OK;
}

extern "C" int rth_bmp_encode(const float* rgb, int W, int H, uint8_t* buf, size_t cap) {
    if (!rgb || W <= 0 || H <= 0 || !buf) return RT_E_ARG;
    const int row = W * 4, hdr = 14 + 40;
    const size_t fsz = (size_t)hdr + (size_t)row * H;
    if (cap < fsz) return RT_E_ARG;
    rth_bmp_header(W, H, buf);
    for (int y = 0; y < H; y++) {  // bottom-up, bmp_writer.c:131-143
        const float* src = rgb + (size_t)(H - 1 - y) * W * 3;
        uint8_t* dst = buf + hdr + (size_t)y * row;
        for (int x = 0; x < W; x++) {
            uint8_t r = (uint8_t)(src[3 * x] * 255.0f);  // vec_to_bgra, bmp_writer.c:88-95
            uint8_t g = (uint8_t)(src[3 * x + 1] * 255.0f);
            uint8_t b = (uint8_t)(src[3 * x + 2] * 255.0f);
            uint32_t px = b | (g << 8) | (r << 16) | (255u << 24);
            std::memcpy(dst + 4 * x, &px, 4);
        }
    }
    return RT_OK;
}

extern "C" int rth_bmp_write(const float* rgb, int W, int H, const char* path) {
    if (!rgb || W <= 0 || H <= 0 || !path) return RT_E_ARG;
    size_t fsz = 54 + (size_t)W * H * 4;
    std::vector<uint8_t> buf(fsz);
    int rc = rth_bmp_encode(rgb, W, H, buf.data(), fsz);
    if (rc) return rc;
    FILE* f = std::fopen(path, "wb");
    if (!f) return RT_E_IO;
    size_t w = std::fwrite(buf.data(), 1, fsz, f);
    std::fclose(f);
    return w == fsz ? RT_OK : RT_E_IO;
}

extern "C" void rth_free(void* p) { std::free(p); }
