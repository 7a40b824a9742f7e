// rt_treelet.hpp — treelet restructuring of the GPU-built binary BVH (Karras & Aila 2013, "Fast parallel construction of
// high-quality bounding volume hierarchies"), host-only and free of HIP so that tests/c/treelet_test.cpp can check it
// with g++ alone.
//
// PLOC (rt_build.hpp) merges nearest neighbours of a Morton-ordered list; its trees are good but locally suboptimal.
// For every internal node, children first, the treelet of its up to TREELET leaves (grown by opening the leaf of
// largest surface area) is rebuilt in the topology of least SAH cost, found by dynamic programming over the subsets
// of those leaves; the treelet's leaves (whole subtrees) and its root's box are unchanged, so the tree stays a valid
// BVH of the same triangles. The fast walk returns the reference's answer on any conservative BVH, so
// the tree's shape changes only how many nodes a ray visits.
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <thread>
#include <vector>

namespace rtt {

struct Box {
    float lo[3], hi[3];
};
inline Box join(const Box& a, const Box& b) {
    Box r;
    for (int k = 0; k < 3; k++) {
        r.lo[k] = std::min(a.lo[k], b.lo[k]);
        r.hi[k] = std::max(a.hi[k], b.hi[k]);
    }
    return r;
}
inline double area(const Box& b) {
    const double x = (double)b.hi[0] - b.lo[0], y = (double)b.hi[1] - b.lo[1], z = (double)b.hi[2] - b.lo[2];
    return 2.0 * (x * y + y * z + z * x);
}

// A binary tree as PLOC leaves it: leaves 0 .. n-1, internal nodes n .. 2n-2 with children left[i - n], right[i - n];
// box[id] for every node.
struct Tree {
    int n = 0, root = 0;
    std::vector<int> left, right;
    std::vector<Box> box;
};

#ifndef PRT_TREELET_LEAVES
#define PRT_TREELET_LEAVES 7
#endif
constexpr int TREELET = PRT_TREELET_LEAVES;  // leaves per treelet (2^7 subsets)
#ifndef PRT_TREELET_CI
#define PRT_TREELET_CI 1.2
#endif
constexpr double C_INNER = PRT_TREELET_CI, C_LEAF = 1.0;  // the SAH prices of the paper

// SAH cost of every subtree (bottom-up): C_INNER * area of each internal node + C_LEAF * area of each leaf
inline std::vector<double> subtree_costs(const Tree& T, const std::vector<int>& post) {
    std::vector<double> c(T.box.size(), 0.0);
    for (int i = 0; i < T.n; i++) c[i] = C_LEAF * area(T.box[i]);
    for (int id : post) c[id] = C_INNER * area(T.box[id]) + c[T.left[id - T.n]] + c[T.right[id - T.n]];
    return c;
}
// the internal nodes, children before parents
inline std::vector<int> post_order(const Tree& T) {
    std::vector<int> out;
    if (T.root < T.n) return out;
    out.reserve(T.n);
    std::vector<int> st{T.root};
    while (!st.empty()) {  // pre-order visiting the right child first; reversed, every child precedes its parent
        const int id = st.back();
        st.pop_back();
        out.push_back(id);
        const int l = T.left[id - T.n], r = T.right[id - T.n];
        if (l >= T.n) st.push_back(l);
        if (r >= T.n) st.push_back(r);
    }
    std::reverse(out.begin(), out.end());
    return out;
}

// The treelet of internal node N rebuilt in its least-cost topology (one step of a pass; children first). Touches only
// N's subtree: N, the treelet's internal nodes, and their costs. `scratch` holds the subset tables (one per thread).
struct TreeletScratch {
    std::vector<double> sa, copt;
    std::vector<int> part;
    std::vector<Box> sbox;
    TreeletScratch() : sa(1 << TREELET), copt(1 << TREELET), part(1 << TREELET), sbox(1 << TREELET) {}
};
inline void optimize_node(Tree& T, std::vector<double>& cost, int N, TreeletScratch& S) {
    std::vector<double>& sa = S.sa;
    std::vector<double>& copt = S.copt;
    std::vector<int>& part = S.part;
    std::vector<Box>& sbox = S.sbox;
    // N's cost from its children's current costs: a treelet rebuilt below N since the pass began lowered them
    // (post order: every child is final here), and the test below must compare against the tree as it now is
    cost[N] = C_INNER * area(T.box[N]) + cost[T.left[N - T.n]] + cost[T.right[N - T.n]];
    // the treelet: open the leaf of largest area until TREELET leaves (or none can be opened)
    int leaves[TREELET], inner[TREELET];
    int nl = 2, ni = 1;
    leaves[0] = T.left[N - T.n];
    leaves[1] = T.right[N - T.n];
    inner[0] = N;
    while (nl < TREELET) {
        int best = -1;
        double ba = -1.0;
        for (int i = 0; i < nl; i++)
            if (leaves[i] >= T.n && area(T.box[leaves[i]]) > ba) {
                ba = area(T.box[leaves[i]]);
                best = i;
            }
        if (best < 0) break;
        const int id = leaves[best];
        inner[ni++] = id;
        leaves[best] = T.left[id - T.n];
        leaves[nl++] = T.right[id - T.n];
    }
    if (nl < 3) return;
    const int full = (1 << nl) - 1;
    // least-cost topology over the treelet's leaves (subsets in increasing order: every proper subset first)
    for (int S2 = 1; S2 <= full; S2++) {
        const int lo = S2 & -S2;
        if (S2 == lo) {
            const int i = __builtin_ctz((unsigned)S2);
            sbox[S2] = T.box[leaves[i]];
            copt[S2] = cost[leaves[i]];
            continue;
        }
        sbox[S2] = join(sbox[S2 ^ lo], sbox[lo]);
        sa[S2] = area(sbox[S2]);
        double bc = 1e300;
        int bp = 0;
        for (int P = (S2 - 1) & S2; P; P = (P - 1) & S2) {
            if (!(P & lo)) continue;  // (each split once: the part holding S2's lowest leaf)
            const double c = copt[P] + copt[S2 ^ P];
            if (c < bc) {
                bc = c;
                bp = P;
            }
        }
        copt[S2] = C_INNER * sa[S2] + bc;
        part[S2] = bp;
    }
    if (!(copt[full] < cost[N] * (1.0 - 1e-9))) return;
    // rebuild the treelet in that topology, reusing its internal nodes (N stays its root)
    int used = 0;
    struct Item {
        int S, id;
    };
    Item todo[TREELET], order[TREELET];
    int nt = 0, no = 0;
    todo[nt++] = {full, inner[used++]};
    auto node_of = [&](int S2) {
        if ((S2 & (S2 - 1)) == 0) return leaves[__builtin_ctz((unsigned)S2)];
        const int id = inner[used++];
        todo[nt++] = {S2, id};
        return id;
    };
    while (nt > 0) {
        const Item it = todo[--nt];
        order[no++] = it;
        const int l = node_of(part[it.S]), r = node_of(it.S ^ part[it.S]);
        T.left[it.id - T.n] = l;
        T.right[it.id - T.n] = r;
    }
    for (int k = no - 1; k >= 0; k--) {  // boxes and costs, children first
        const int id = order[k].id;
        const int l = T.left[id - T.n], r = T.right[id - T.n];
        T.box[id] = join(T.box[l], T.box[r]);
        cost[id] = C_INNER * area(T.box[id]) + cost[l] + cost[r];
    }
}

// One pass over every internal node; returns the tree's SAH cost after it (the root's subtree cost). threads > 1:
// disjoint subtrees in parallel (each in its own post order), then the nodes above them -- the same tree as one thread
// makes (a node's step touches its own subtree only, and every node still follows its children).
inline double optimize_pass(Tree& T, int threads = 1) {
    const std::vector<int> post = post_order(T);
    if (post.empty()) return C_LEAF * area(T.box[T.root]);
    std::vector<double> cost = subtree_costs(T, post);
    if (threads <= 1 || (int)post.size() < 4096) {
        TreeletScratch S;
        for (int N : post) optimize_node(T, cost, N, S);
        return cost[T.root];
    }
    // the subtrees: split the largest frontier node until there are 8 per thread (or they are small)
    std::vector<int> size(T.box.size(), 0);  // internal nodes per subtree
    for (int id : post) {
        const int l = T.left[id - T.n], r = T.right[id - T.n];
        size[id] = 1 + (l >= T.n ? size[l] : 0) + (r >= T.n ? size[r] : 0);
    }
    std::vector<char> top(T.box.size(), 0);
    std::vector<int> frontier{T.root};
    const size_t want = 8 * (size_t)threads;
    while (frontier.size() < want) {
        size_t bi = 0;
        for (size_t i = 1; i < frontier.size(); i++)
            if (size[frontier[i]] > size[frontier[bi]]) bi = i;
        const int id = frontier[bi];
        if (size[id] < 2048) break;
        top[id] = 1;
        frontier.erase(frontier.begin() + (long)bi);
        for (int c : {T.left[id - T.n], T.right[id - T.n]})
            if (c >= T.n) frontier.push_back(c);
    }
    std::sort(frontier.begin(), frontier.end(), [&](int a, int b) { return size[a] > size[b]; });  // big ones first
    std::atomic<size_t> next{0};
    auto work = [&]() {
        TreeletScratch S;
        for (size_t i; (i = next.fetch_add(1)) < frontier.size();) {
            Tree sub;  // (post_order needs only the root and the child arrays)
            std::vector<int> st{frontier[i]}, order;
            while (!st.empty()) {  // this subtree's post order, as post_order makes it
                const int id = st.back();
                st.pop_back();
                order.push_back(id);
                const int l = T.left[id - T.n], r = T.right[id - T.n];
                if (l >= T.n) st.push_back(l);
                if (r >= T.n) st.push_back(r);
            }
            for (auto it = order.rbegin(); it != order.rend(); ++it) optimize_node(T, cost, *it, S);
        }
    };
    std::vector<std::thread> pool;
    for (int k = 1; k < threads; k++) pool.emplace_back(work);
    work();
    for (std::thread& th : pool) th.join();
    TreeletScratch S;
    for (int N : post)  // the nodes above the subtrees, children first
        if (top[N]) optimize_node(T, cost, N, S);
    return cost[T.root];
}

inline double tree_cost(const Tree& T) {
    const std::vector<int> post = post_order(T);
    if (post.empty()) return C_LEAF * area(T.box[T.root]);
    return subtree_costs(T, post)[T.root];
}

}  // namespace rtt
