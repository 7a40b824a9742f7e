// rt_wide.cpp — the fast walk's 8-wide quantised BVH (device layout: rt_device.hpp, DWide).
//
// Built from any reference-layout binary BVH (bvh_t[] + tri_idx, cpu/src/bvh.c:360-388), normally
// this library's binned SAH. The binary tree is collapsed top-down: a wide node starts from the two
// children of a binary node and repeatedly opens its largest-area interior child until it has 8
// children (Wald et al. / Ylitie et al. style collapse). Leaves are cut to <= 4 triangles so that a
// wide node's leaf triangles fit a 32-bit mask (8 slots x 4).
//
// Conservativeness: each child box is first grown by `inflate` (the same margin the binary fast walk
// uses, >= the reciprocal-FMA slab test's rounding reach), then quantised OUTWARD to 8 bits per
// plane on a per-node power-of-two grid. Every plane is checked with the device's own decode,
// fmaf(scale, q, p) (scale * q is exact, so this is p + scale * q rounded once), and moved outward
// until the decoded box contains the grown box.
//
// Slot order: children sit in the slot of the octant they occupy relative to the node centre
// (bit 0 = +x, bit 1 = +y, bit 2 = +z), so that a ray visiting slots in the order k ^ octant(ray)
// for k = 0..7 meets them roughly front to back without sorting.
#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <unordered_map>
#include <vector>

#include "rt_host.h"

namespace {

struct Box {
    float lo[3], hi[3];
};

Box empty_box() {
    Box b;
    for (int a = 0; a < 3; a++) {
        b.lo[a] = INFINITY;
        b.hi[a] = -INFINITY;
    }
    return b;
}

void grow(Box& b, const Box& o) {
    for (int a = 0; a < 3; a++) {
        b.lo[a] = std::min(b.lo[a], o.lo[a]);
        b.hi[a] = std::max(b.hi[a], o.hi[a]);
    }
}

float area(const Box& b) {
    const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}

constexpr int LEAF_MAX = 4;
constexpr int WIDTH = 8;

struct BNode {
    Box b;
    int l = -1, r = -1;      // interior: children (BNode indices); leaf: l == -1
    int first = 0, cnt = 0;  // leaf: range of `idx`
};

struct WBuilder {
    const rt_triangle* T = nullptr;
    int n = 0;
    std::vector<int> idx;
    std::vector<BNode> bn;
    float inflate = 0.0f;

    Box tri_box(int t) const {
        Box b = empty_box();
        for (const rt_vec3& c : T[t].coords) {
            const float v[3] = {c.x, c.y, c.z};
            for (int a = 0; a < 3; a++) {
                b.lo[a] = std::min(b.lo[a], v[a]);
                b.hi[a] = std::max(b.hi[a], v[a]);
            }
        }
        return b;
    }

    // a leaf range, cut by object median on the widest centroid axis until <= LEAF_MAX triangles (nodes into out:
    // bn, or a subtree's own vector when subtrees are made in parallel -- they sort disjoint ranges of idx)
    int leaf(std::vector<BNode>& out, int first, int cnt) {
        if (cnt <= LEAF_MAX) {
            BNode x;
            x.first = first;
            x.cnt = cnt;
            x.b = empty_box();
            for (int i = first; i < first + cnt; i++) grow(x.b, tri_box(idx[i]));
            out.push_back(x);
            return (int)out.size() - 1;
        }
        float cl[3] = {INFINITY, INFINITY, INFINITY}, ch[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = first; i < first + cnt; i++)
            for (int a = 0; a < 3; a++) {
                cl[a] = std::min(cl[a], T[idx[i]].centroid[a]);
                ch[a] = std::max(ch[a], T[idx[i]].centroid[a]);
            }
        int ax = 0;
        for (int a = 1; a < 3; a++)
            if (ch[a] - cl[a] > ch[ax] - cl[ax]) ax = a;
        std::stable_sort(idx.begin() + first, idx.begin() + first + cnt,
                         [&](int u, int v) { return T[u].centroid[ax] < T[v].centroid[ax]; });
        const int h = cnt / 2;
        const int l = leaf(out, first, h), r = leaf(out, first + h, cnt - h);
        return inner(out, l, r);
    }

    int inner(std::vector<BNode>& bn, int l, int r) {
        BNode x;
        x.l = l;
        x.r = r;
        x.b = bn[l].b;
        grow(x.b, bn[r].b);
        // the subtree's triangles as one range of idx (every reference-layout builder partitions in place);
        // cnt = -1: not contiguous, never merged into one leaf
        const BNode &L = bn[l], &R = bn[r];
        if (L.cnt >= 0 && R.cnt >= 0 && (L.first + L.cnt == R.first || R.first + R.cnt == L.first)) {
            x.first = std::min(L.first, R.first);
            x.cnt = L.cnt + R.cnt;
        } else {
            x.cnt = -1;
        }
        bn.push_back(x);
        return (int)bn.size() - 1;
    }

    // ---- SAH-optimal collapse (Ylitie et al. 2017, §3.1): cost(n, i) = cheapest way to hang subtree n
    // off a parent using at most i slots — as one leaf slot (<= LEAF_MAX triangles), as one wide node,
    // or by distributing the slots over n's two children. Costs are surface area x (C_node per wide-node
    // visit, 1 per triangle test).
    struct Dp {  // one node's costs, side by side (the collapse reads them node by node, in no memory order)
        float cost[WIDTH + 1];
        signed char split[WIDTH + 1];  // dist(n, i): slots given to the left child
        char as_leaf;                  // cost(n, 1) is the leaf form
    };
    std::unique_ptr<Dp[]> dp;  // (uninitialised: every node's entry is written before it is read)
    void sah_begin() { dp.reset(new Dp[bn.size()]); }
    // nodes [n0, n1) of bn, whose children precede them within the range or in ranges already costed
    void sah_costs(size_t n0, size_t n1, float c_node) {
        for (size_t n = n0; n < n1; n++) {  // children precede parents in bn
            const BNode& B = bn[n];
            Dp& D = dp[n];
            const float A = area(B.b);
            const float leaf = (B.cnt > 0 && B.cnt <= LEAF_MAX) ? A * (float)B.cnt : INFINITY;
            if (B.l < 0) {
                for (int i = 1; i <= WIDTH; i++) D.cost[i] = leaf;
                D.as_leaf = 1;
                continue;
            }
            const Dp &L = dp[B.l], &R = dp[B.r];
            float dist[WIDTH + 1];
            for (int j = 2; j <= WIDTH; j++) {
                float best = INFINITY;
                int bk = 1;
                for (int k = 1; k < j; k++) {
                    const float c = L.cost[k] + R.cost[j - k];
                    if (c < best) {
                        best = c;
                        bk = k;
                    }
                }
                dist[j] = best;
                D.split[j] = (signed char)bk;
            }
            const float node = c_node * A + dist[WIDTH];
            D.as_leaf = leaf <= node;
            D.cost[1] = std::min(leaf, node);
            for (int i = 2; i <= WIDTH; i++) D.cost[i] = std::min(D.cost[1], dist[i]);
        }
    }
    // the slots of subtree n given i of them: (bnode, as-leaf) pairs
    void collect(int n, int i, std::vector<std::pair<int, bool>>& out) const {
        const BNode& B = bn[n];
        const Dp& D = dp[n];
        if (B.l < 0 || i == 1 || D.cost[i] == D.cost[1]) {
            out.push_back({n, B.l < 0 || D.as_leaf != 0});
            return;
        }
        const int k = D.split[i];
        collect(B.l, k, out);
        collect(B.r, i - k, out);
    }

    // reference-layout node i -> BNode index in out (-1: empty subtree); top: the subtrees already made, by their
    // reference node (made in parallel, then appended to bn)
    int make(std::vector<BNode>& out, const rt_bvh_node* B, int nn, int i, int depth, bool& bad,
             const std::unordered_map<int, int>* top = nullptr) {
        if (top) {
            const auto f = top->find(i);
            if (f != top->end()) return f->second;
        }
        if (i < 0 || i >= nn || depth > 64) {
            bad = true;
            return -1;
        }
        const rt_bvh_node& p = B[i];
        if (p.tr_len > 0) {
            if (p.child < 0 || (long long)p.child + p.tr_len > n) {
                bad = true;
                return -1;
            }
            return leaf(out, p.child, p.tr_len);
        }
        if (p.child == 0) return -1;
        const int l = make(out, B, nn, p.child, depth + 1, bad, top);
        const int r = make(out, B, nn, p.child + 1, depth + 1, bad, top);
        if (l < 0) return r;
        if (r < 0) return l;
        return inner(out, l, r);
    }
};

// A plane is decoded as fmaf(2^e, QBIAS + q, p): QBIAS + q (1024 .. 1279) is an f16 integer whose bits are 0x6400 | q,
// so the device forms two such halves from two plane bytes with one v_perm_b32 and feeds them to v_fma_mix_f32, which
// converts the half exactly inside the FMA (rt_kernels.hpp wide_node): one perm per two planes instead of a byte
// conversion per plane, the same single rounding. The grid's origin p therefore lies QBIAS steps below the node.
constexpr int QBIAS = 1024;
inline float fma_decode(float scale, int q, float p) { return std::fmaf(scale, (float)(QBIAS + q), p); }
// the largest float <= x
inline float round_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -INFINITY);
    return f;
}

inline uint32_t f2u(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

// Quantise one axis of up to 8 child boxes (already grown) on the grid pb + 2^e * (QBIAS + q), q in 0..255.
// Returns the grid's exponent e (-126 .. 110); pb receives the grid's origin, qlo/qhi the planes.
int quantise_axis(const float* lo, const float* hi, int k, float& pb, int* qlo, int* qhi) {
    float p = INFINITY, top = -INFINITY;
    for (int c = 0; c < k; c++) {
        p = std::min(p, lo[c]);
        top = std::max(top, hi[c]);
    }
    const double ext = (double)top - (double)p;
    int e = ext > 0 ? (int)std::ceil(std::log2(ext / 255.0)) : -126;
    e = std::max(-126, std::min(e, 100));  // (QBIAS * 2^e stays finite)
    for (;; e++) {
        const float scale = std::ldexp(1.0f, e);
        pb = round_down((double)p - (double)QBIAS * scale);  // q = 0 decodes to the lowest plane or below it
        bool ok = true;
        for (int c = 0; c < k && ok; c++) {
            int a = (int)std::floor(((double)lo[c] - (double)pb) / scale) - QBIAS;
            a = std::max(0, std::min(a, 255));
            while (a > 0 && fma_decode(scale, a, pb) > lo[c]) a--;
            int b = (int)std::ceil(((double)hi[c] - (double)pb) / scale) - QBIAS;
            b = std::max(0, b);
            while (b <= 255 && fma_decode(scale, b, pb) < hi[c]) b++;
            if (b > 255 || fma_decode(scale, a, pb) > lo[c]) ok = false;
            qlo[c] = a;
            qhi[c] = b;
        }
        if (ok || e >= 110) return e;
    }
}

}  // namespace

extern "C" int rth_wbvh_build(const rt_bvh_node* bvh, int n_nodes, const int* tri_idx, const rt_triangle* tris,
                              int n_tris, float inflate, uint32_t** nodes_out, int** tri_order_out,
                              rth_wbvh_info* info) {
    return rth_wbvh_build_cost(bvh, n_nodes, tri_idx, tris, n_tris, inflate, 0.0f, nodes_out, tri_order_out, info);
}

extern "C" int rth_wbvh_build_cost(const rt_bvh_node* bvh, int n_nodes, const int* tri_idx, const rt_triangle* tris,
                                   int n_tris, float inflate, float c_node, uint32_t** nodes_out, int** tri_order_out,
                                   rth_wbvh_info* info) {
    if (!bvh || n_nodes <= 0 || !tri_idx || !tris || n_tris <= 0 || !nodes_out || !tri_order_out ||
        !(inflate >= 0.0f))
        return RT_E_ARG;
    WBuilder w;
    w.T = tris;
    w.n = n_tris;
    w.inflate = inflate;
    w.idx.assign(tri_idx, tri_idx + n_tris);
    for (int t : w.idx)
        if (t < 0 || t >= n_tris) return RT_E_ARG;
    w.bn.reserve(2 * (size_t)n_tris + 2);
    const int nthreads = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
    // the binary tree in parallel: the reference layout's top levels, breadth first, down to ~8 subtrees per thread
    // (leaves and empty slots stay in the frontier); each subtree into its own vector on the threads, appended to bn
    // in frontier order (children still precede parents), then the top above them -- the tree a one-thread make()
    // makes, node for node, in another order of bn
    struct Front {
        int i, depth;
    };
    std::vector<Front> front{{0, 0}};
    if (n_tris >= 4096 && nthreads > 1) {
        for (size_t q = 0; q < front.size() && front.size() < 8 * (size_t)nthreads;) {
            const Front f = front[q];
            const bool inner_node = f.i >= 0 && f.i < n_nodes && bvh[f.i].tr_len <= 0 && bvh[f.i].child > 0 &&
                                    bvh[f.i].child < n_nodes - 1 && f.depth < 64;
            if (!inner_node) {
                q++;
                continue;
            }
            front.erase(front.begin() + (long)q);
            front.push_back({bvh[f.i].child, f.depth + 1});
            front.push_back({bvh[f.i].child + 1, f.depth + 1});
        }
    }
    {  // (a malformed layout naming one node twice: one thread, as before)
        std::vector<int> ids;
        for (const Front& f : front) ids.push_back(f.i);
        std::sort(ids.begin(), ids.end());
        if (std::adjacent_find(ids.begin(), ids.end()) != ids.end()) front.assign(1, Front{0, 0});
    }
    std::vector<std::vector<BNode>> part(front.size());
    std::vector<int> proot(front.size(), -1);
    std::vector<char> pbad(front.size(), 0);
    auto run_tasks = [&](size_t n, auto&& fn) {  // fn(k) for k < n, taken one at a time by the threads
        std::atomic<size_t> next{0};
        auto worker = [&] {
            for (size_t k; (k = next.fetch_add(1)) < n;) fn(k);
        };
        const int nt = (int)std::min<size_t>((size_t)nthreads, n);
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; t++) pool.emplace_back(worker);
        worker();
        for (std::thread& th : pool) th.join();
    };
    bool bad = false;
    int root;
    std::vector<size_t> pbase(front.size() + 1, 0);
    if (front.size() == 1) {
        root = w.make(w.bn, bvh, n_nodes, 0, 0, bad);
    } else {
        run_tasks(front.size(), [&](size_t k) {
            bool b = false;
            proot[k] = w.make(part[k], bvh, n_nodes, front[k].i, front[k].depth, b);
            pbad[k] = b;
        });
        std::unordered_map<int, int> top;
        for (size_t k = 0; k < front.size(); k++) {
            bad = bad || pbad[k];
            pbase[k + 1] = pbase[k] + part[k].size();
            top[front[k].i] = proot[k] >= 0 ? proot[k] + (int)pbase[k] : -1;
        }
        w.bn.resize(pbase[front.size()]);
        run_tasks(front.size(), [&](size_t k) {  // (the subtrees' nodes into place, their children's indices moved)
            const int off = (int)pbase[k];
            BNode* dst = w.bn.data() + pbase[k];
            for (const BNode& x : part[k]) {
                *dst = x;
                if (x.l >= 0) {
                    dst->l += off;
                    dst->r += off;
                }
                dst++;
            }
            std::vector<BNode>().swap(part[k]);
        });
        root = w.make(w.bn, bvh, n_nodes, 0, 0, bad, &top);
    }
    if (bad || root < 0) return RT_E_ARG;
    // collapse policy: SAH-optimal, a wide-node visit priced at 2 triangle tests (the best of 2 / 3 / 4 in the
    // measured sweep — dragon -3.5 % vs 4, car_boxed even; the greedy largest-area collapse: +1.6 % / +3 %;
    // DESIGN.md §3). The subtrees' ranges of bn on the threads, then the top.
    const float cn = c_node > 0.0f ? c_node : 2.0f;
    w.sah_begin();
    if (front.size() > 1)
        run_tasks(front.size(), [&](size_t k) { w.sah_costs(pbase[k], pbase[k + 1], cn); });
    w.sah_costs(pbase[front.size()], w.bn.size(), cn);

    // breadth-first: interior children of a wide node get consecutive indices. Level by level: every node of a level
    // is formed independently (its children, slots, quantised planes) on the build's threads, then the level's
    // child / triangle bases follow by prefix sums in queue order -- the layout a one-node-at-a-time queue makes.
    struct Item {
        int b, depth;
    };
    struct Out {  // one wide node before its bases are known
        uint32_t W[20];
        int kid[WIDTH];      // per slot: the child's BNode (-1: empty)
        char leaf[WIDTH];    // per slot: a leaf slot
        int n_inner, n_tri;  // interior slots, leaf triangles
    };
    auto form = [&](const Item& it, Out& o) {
        const BNode& B = w.bn[it.b];
        std::pair<int, bool> c2[WIDTH];
        int k = 0;
        if (B.l < 0 || w.dp[it.b].as_leaf) {
            c2[k++] = {it.b, true};  // a leaf root
        } else {  // the cost-optimal distribution of this node's 8 slots
            std::vector<std::pair<int, bool>> tmp;
            tmp.reserve(WIDTH);
            w.collect(B.l, w.dp[it.b].split[WIDTH], tmp);
            w.collect(B.r, WIDTH - w.dp[it.b].split[WIDTH], tmp);
            for (auto& pr : tmp) c2[k++] = pr;
        }
        // octant slots: greedy on cost = -dot(centre offset, slot direction)
        Box all = empty_box();
        for (int c = 0; c < k; c++) grow(all, w.bn[c2[c].first].b);
        float pc[3];
        for (int a = 0; a < 3; a++) pc[a] = 0.5f * (all.lo[a] + all.hi[a]);
        int kid_in[WIDTH];
        for (int s2 = 0; s2 < WIDTH; s2++) kid_in[s2] = -1;
        bool done[WIDTH] = {false};
        for (int round = 0; round < k; round++) {
            float bc = INFINITY;
            int bk = -1, bs = -1;
            for (int c = 0; c < k; c++) {
                if (done[c]) continue;
                const Box& cb = w.bn[c2[c].first].b;
                for (int s2 = 0; s2 < WIDTH; s2++) {
                    if (kid_in[s2] >= 0) continue;
                    float cost = 0.0f;
                    for (int a = 0; a < 3; a++) {
                        const float off = 0.5f * (cb.lo[a] + cb.hi[a]) - pc[a];
                        cost -= ((s2 >> a) & 1) ? off : -off;
                    }
                    if (cost < bc) {
                        bc = cost;
                        bk = c;
                        bs = s2;
                    }
                }
            }
            done[bk] = true;
            kid_in[bs] = bk;
        }
        // quantise (grown boxes) per axis over the occupied slots
        float lo[3][WIDTH], hi[3][WIDTH];
        int qlo[3][WIDTH], qhi[3][WIDTH];
        int ks = 0;
        int slot_list[WIDTH];
        for (int s2 = 0; s2 < WIDTH; s2++)
            if (kid_in[s2] >= 0) {
                const Box& cb = w.bn[c2[kid_in[s2]].first].b;
                for (int a = 0; a < 3; a++) {
                    lo[a][ks] = cb.lo[a] - inflate;
                    hi[a][ks] = cb.hi[a] + inflate;
                }
                slot_list[ks++] = s2;
            }
        float p[3];
        int eb[3];
        for (int a = 0; a < 3; a++) eb[a] = quantise_axis(lo[a], hi[a], ks, p[a], qlo[a], qhi[a]);
        uint32_t* W = o.W;
        std::memset(W, 0, sizeof o.W);
        W[0] = f2u(p[0]);
        W[1] = f2u(p[1]);
        W[2] = f2u(p[2]);
        uint32_t imask = 0;
        for (int s2 = 0; s2 < WIDTH; s2++)
            if (kid_in[s2] >= 0 && !c2[kid_in[s2]].second) imask |= 1u << s2;
        // the exponents as signed bytes: the walks scale 1/d by them with one v_ldexp_f32 each
        W[3] = (uint32_t)(uint8_t)(int8_t)eb[0] | ((uint32_t)(uint8_t)(int8_t)eb[1] << 8) |
               ((uint32_t)(uint8_t)(int8_t)eb[2] << 16) | (imask << 24);
        uint8_t q8[6][WIDTH];
        for (int s2 = 0; s2 < WIDTH; s2++) {  // empty slots: an inverted box (never selected: meta 0, imask 0)
            for (int a = 0; a < 3; a++) {
                q8[a][s2] = 255;
                q8[3 + a][s2] = 0;
            }
            o.kid[s2] = kid_in[s2] >= 0 ? c2[kid_in[s2]].first : -1;
            o.leaf[s2] = kid_in[s2] >= 0 && c2[kid_in[s2]].second;
        }
        o.n_inner = o.n_tri = 0;
        for (int j = 0; j < ks; j++) {
            const int s2 = slot_list[j];
            for (int a = 0; a < 3; a++) {
                q8[a][s2] = (uint8_t)qlo[a][j];
                q8[3 + a][s2] = (uint8_t)qhi[a][j];
            }
            if (o.leaf[s2]) o.n_tri += w.bn[o.kid[s2]].cnt;
            else o.n_inner++;
        }
        // per axis a, four words: word j = qlo[2j], qhi[2j], qlo[2j + 1], qhi[2j + 1] (one slot pair's two planes
        // side by side, so that a single byte permute picks a pair's near or far planes by the ray's sign)
        for (int a = 0; a < 3; a++)
            for (int j = 0; j < WIDTH / 2; j++)
                W[8 + 4 * a + j] = (uint32_t)q8[a][2 * j] | ((uint32_t)q8[3 + a][2 * j] << 8) |
                                   ((uint32_t)q8[a][2 * j + 1] << 16) | ((uint32_t)q8[3 + a][2 * j + 1] << 24);
    };
    auto parallel = [&](size_t n, auto&& fn) {  // fn(i) for i < n, in contiguous chunks over the threads
        const int nt = (int)std::min<size_t>((size_t)nthreads, (n + 255) / 256);
        if (nt <= 1) {
            for (size_t i = 0; i < n; i++) fn(i);
            return;
        }
        std::vector<std::thread> pool;
        for (int t = 0; t < nt; t++)
            pool.emplace_back([&, t] {
                for (size_t i = n * t / nt; i < n * (t + 1) / nt; i++) fn(i);
            });
        for (std::thread& th : pool) th.join();
    };
    std::vector<Item> level{{root, 1}};
    std::vector<uint32_t> words;
    std::vector<int> order(n_tris, -1);
    size_t n_wide = 0, n_order = 0;
    int depth = 0, max_kids = 0;
    std::vector<Out> outs;
    while (!level.empty()) {
        depth = std::max(depth, level[0].depth);
        outs.resize(level.size());
        parallel(level.size(), [&](size_t i) { form(level[i], outs[i]); });
        // bases in queue order: this level's children follow every node queued so far
        size_t next_node = n_wide + level.size(), next_tri = n_order;
        std::vector<size_t> cbase(level.size()), tbase(level.size());
        std::vector<Item> nxt;
        for (size_t i = 0; i < level.size(); i++) {
            cbase[i] = next_node;
            tbase[i] = next_tri;
            next_node += (size_t)outs[i].n_inner;
            next_tri += (size_t)outs[i].n_tri;
            int kc = 0;
            for (int s2 = 0; s2 < WIDTH; s2++)
                if (outs[i].kid[s2] >= 0) {
                    kc++;
                    if (!outs[i].leaf[s2]) nxt.push_back({outs[i].kid[s2], level[i].depth + 1});
                }
            max_kids = std::max(max_kids, kc);
        }
        if (next_tri > (size_t)n_tris) return RT_E_ARG;  // a triangle referenced twice
        words.resize(20 * (n_wide + level.size()));
        parallel(level.size(), [&](size_t i) {
            Out& o = outs[i];
            o.W[4] = (uint32_t)cbase[i];
            o.W[5] = (uint32_t)tbase[i];
            uint8_t meta[WIDTH] = {0};
            int off = 0;
            for (int s2 = 0; s2 < WIDTH; s2++)
                if (o.kid[s2] >= 0 && o.leaf[s2]) {
                    const BNode& c = w.bn[o.kid[s2]];
                    meta[s2] = (uint8_t)((c.cnt << 5) | off);
                    for (int t = c.first; t < c.first + c.cnt; t++) order[tbase[i] + (size_t)off++] = w.idx[t];
                }
            std::memcpy(&o.W[6], meta, 8);
            std::memcpy(&words[20 * (n_wide + i)], o.W, sizeof o.W);
        });
        n_wide += level.size();
        n_order = next_tri;
        level.swap(nxt);
    }
    order.resize(n_order);
    if ((int)order.size() != n_tris) return RT_E_ARG;  // a triangle referenced twice or never
    uint32_t* nodes = (uint32_t*)std::malloc(sizeof(uint32_t) * words.size());
    int* ord = (int*)std::malloc(sizeof(int) * order.size());
    if (!nodes || !ord) {
        std::free(nodes);
        std::free(ord);
        return RT_E_NOMEM;
    }
    std::memcpy(nodes, words.data(), sizeof(uint32_t) * words.size());
    std::memcpy(ord, order.data(), sizeof(int) * order.size());
    *nodes_out = nodes;
    *tri_order_out = ord;
    if (info) {
        info->n_nodes = (int)(words.size() / 20);
        info->n_tris = (int)order.size();
        info->depth = depth;
        info->max_children = max_kids;
    }
    return RT_OK;
}
