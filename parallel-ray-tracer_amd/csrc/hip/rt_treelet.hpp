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
#include <cstdint>
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

// One pass over every internal node; returns the tree's SAH cost after it (the root's subtree cost).
inline double optimize_pass(Tree& T) {
    const std::vector<int> post = post_order(T);
    if (post.empty()) return C_LEAF * area(T.box[T.root]);
    std::vector<double> cost = subtree_costs(T, post);
    const int FULL = (1 << TREELET) - 1;
    std::vector<double> sa(FULL + 1), copt(FULL + 1);
    std::vector<int> part(FULL + 1);
    std::vector<Box> sbox(FULL + 1);
    for (int N : post) {
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
        if (nl < 3) continue;
        const int full = (1 << nl) - 1;
        // least-cost topology over the treelet's leaves (subsets in increasing order: every proper subset first)
        for (int S = 1; S <= full; S++) {
            const int lo = S & -S;
            if (S == lo) {
                const int i = __builtin_ctz((unsigned)S);
                sbox[S] = T.box[leaves[i]];
                copt[S] = cost[leaves[i]];
                continue;
            }
            sbox[S] = join(sbox[S ^ lo], sbox[lo]);
            sa[S] = area(sbox[S]);
            double bc = 1e300;
            int bp = 0;
            for (int P = (S - 1) & S; P; P = (P - 1) & S) {
                if (!(P & lo)) continue;  // (each split once: the part holding S's lowest leaf)
                const double c = copt[P] + copt[S ^ P];
                if (c < bc) {
                    bc = c;
                    bp = P;
                }
            }
            copt[S] = C_INNER * sa[S] + bc;
            part[S] = bp;
        }
        if (!(copt[full] < cost[N] * (1.0 - 1e-9))) continue;
        // rebuild the treelet in that topology, reusing its internal nodes (N stays its root)
        int used = 0;
        struct Item {
            int S, id;
        };
        std::vector<Item> todo{{full, inner[used++]}};
        auto node_of = [&](int S) {
            if ((S & (S - 1)) == 0) return leaves[__builtin_ctz((unsigned)S)];
            const int id = inner[used++];
            todo.push_back({S, id});
            return id;
        };
        std::vector<Item> order;
        while (!todo.empty()) {
            const Item it = todo.back();
            todo.pop_back();
            order.push_back(it);
            const int l = node_of(part[it.S]), r = node_of(it.S ^ part[it.S]);
            T.left[it.id - T.n] = l;
            T.right[it.id - T.n] = r;
        }
        for (auto it = order.rbegin(); it != order.rend(); ++it) {  // boxes and costs, children first
            const int l = T.left[it->id - T.n], r = T.right[it->id - T.n];
            T.box[it->id] = join(T.box[l], T.box[r]);
            cost[it->id] = C_INNER * area(T.box[it->id]) + cost[l] + cost[r];
        }
    }
    return cost[T.root];
}

inline double tree_cost(const Tree& T) {
    const std::vector<int> post = post_order(T);
    if (post.empty()) return C_LEAF * area(T.box[T.root]);
    return subtree_costs(T, post)[T.root];
}

}  // namespace rtt
