// g++ test of rt_treelet.hpp (no GPU): a random binary tree over random boxes, restructured by treelets, stays a
// BVH of the same leaves -- every leaf once, every internal box the union of its children's, the root's box unchanged
// -- and its SAH cost does not rise; a second pass changes less than the first.
#include "rt_treelet.hpp"

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <cmath>
#include <random>

static int fails = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            fails++;                                                    \
        }                                                               \
    } while (0)

static bool same(const rtt::Box& a, const rtt::Box& b) {
    for (int k = 0; k < 3; k++)
        if (a.lo[k] != b.lo[k] || a.hi[k] != b.hi[k]) return false;
    return true;
}

static void check_tree(const rtt::Tree& T) {
    std::vector<int> seen(2 * T.n - 1, 0);
    std::vector<int> st{T.root};
    while (!st.empty()) {
        const int id = st.back();
        st.pop_back();
        CHECK(id >= 0 && id < 2 * T.n - 1);
        seen[id]++;
        if (id >= T.n) {
            const int l = T.left[id - T.n], r = T.right[id - T.n];
            CHECK(same(T.box[id], rtt::join(T.box[l], T.box[r])));
            st.push_back(l);
            st.push_back(r);
        }
    }
    for (int i = 0; i < 2 * T.n - 1; i++) CHECK(seen[i] == 1);
}

int main() {
    for (int trial = 0; trial < 6; trial++) {
        std::mt19937 rng(1234 + trial);
        std::uniform_real_distribution<float> U(0.0f, 100.0f), S(0.1f, 3.0f);
        const int n = trial < 3 ? 64 << trial : 5000;
        rtt::Tree T;
        T.n = n;
        T.box.resize(2 * n - 1);
        T.left.resize(n - 1);
        T.right.resize(n - 1);
        for (int i = 0; i < n; i++)
            for (int k = 0; k < 3; k++) {
                T.box[i].lo[k] = U(rng);
                T.box[i].hi[k] = T.box[i].lo[k] + S(rng);
            }
        // a poor tree: random merges
        std::vector<int> live(n);
        for (int i = 0; i < n; i++) live[i] = i;
        int next = n;
        while (live.size() > 1) {
            std::uniform_int_distribution<size_t> D(0, live.size() - 1);
            size_t a = D(rng), b = D(rng);
            if (a == b) continue;
            const int x = live[a], y = live[b];
            T.left[next - n] = x;
            T.right[next - n] = y;
            T.box[next] = rtt::join(T.box[x], T.box[y]);
            if (a < b) std::swap(a, b);
            live.erase(live.begin() + a);
            live.erase(live.begin() + b);
            live.push_back(next++);
        }
        T.root = live[0];
        const rtt::Box root_box = T.box[T.root];
        check_tree(T);
        const double c0 = rtt::tree_cost(T);
        const double c1 = rtt::optimize_pass(T);
        check_tree(T);
        CHECK(same(T.box[T.root], root_box));
        CHECK(c1 <= c0);
        CHECK(std::abs(c1 - rtt::tree_cost(T)) <= 1e-6 * c1);
        const double c2 = rtt::optimize_pass(T);
        check_tree(T);
        CHECK(c2 <= c1);
        CHECK(c0 - c1 >= c1 - c2);
        std::printf("n %d: SAH cost %.4g -> %.4g -> %.4g\n", n, c0, c1, c2);
    }
    // an already-good tree (median splits along the longest axis): few treelets are rebuilt, so most ancestors keep
    // the costs the pass computed at its start -- the returned cost must still be the tree's, and never above it
    for (int trial = 0; trial < 3; trial++) {
        std::mt19937 rng(99 + trial);
        std::uniform_real_distribution<float> U(0.0f, 100.0f), S(0.1f, 3.0f);
        const int n = 3000 << trial;
        rtt::Tree T;
        T.n = n;
        T.box.resize(2 * n - 1);
        T.left.resize(n - 1);
        T.right.resize(n - 1);
        for (int i = 0; i < n; i++)
            for (int k = 0; k < 3; k++) {
                T.box[i].lo[k] = U(rng);
                T.box[i].hi[k] = T.box[i].lo[k] + S(rng);
            }
        std::vector<int> ids(n);
        for (int i = 0; i < n; i++) ids[i] = i;
        int next = n;
        // recursive median split -> node id; below 32 leaves random merges (poor subtrees under a good top: the
        // subtrees' treelets are rebuilt, their ancestors' mostly not)
        std::function<int(int, int)> build = [&](int b, int e) -> int {
            if (e - b == 1) return ids[b];
            if (e - b <= 32) {
                std::vector<int> live(ids.begin() + b, ids.begin() + e);
                while (live.size() > 1) {
                    std::uniform_int_distribution<size_t> D(0, live.size() - 1);
                    size_t x = D(rng), y = D(rng);
                    if (x == y) continue;
                    const int id = next++;
                    T.left[id - n] = live[x];
                    T.right[id - n] = live[y];
                    T.box[id] = rtt::join(T.box[live[x]], T.box[live[y]]);
                    if (x < y) std::swap(x, y);
                    live.erase(live.begin() + x);
                    live.erase(live.begin() + y);
                    live.push_back(id);
                }
                return live[0];
            }
            rtt::Box bb = T.box[ids[b]];
            for (int i = b + 1; i < e; i++) bb = rtt::join(bb, T.box[ids[i]]);
            int ax = 0;
            for (int k = 1; k < 3; k++)
                if (bb.hi[k] - bb.lo[k] > bb.hi[ax] - bb.lo[ax]) ax = k;
            const int m = (b + e) / 2;
            std::nth_element(ids.begin() + b, ids.begin() + m, ids.begin() + e, [&](int x, int y) {
                return T.box[x].lo[ax] + T.box[x].hi[ax] < T.box[y].lo[ax] + T.box[y].hi[ax];
            });
            const int l = build(b, m), r = build(m, e);
            const int id = next++;
            T.left[id - n] = l;
            T.right[id - n] = r;
            T.box[id] = rtt::join(T.box[l], T.box[r]);
            return id;
        };
        T.root = build(0, n);
        check_tree(T);
        {  // threads: disjoint subtrees in parallel, then the nodes above them -- the same tree as one thread makes
            rtt::Tree A = T, B = T;
            const double ca = rtt::optimize_pass(A, 1), cb = rtt::optimize_pass(B, 4);
            CHECK(ca == cb && A.left == B.left && A.right == B.right);
            for (size_t i = 0; i < A.box.size(); i++) CHECK(same(A.box[i], B.box[i]));
        }
        double prev = rtt::tree_cost(T);
        for (int pass = 0; pass < 3; pass++) {
            const double c = rtt::optimize_pass(T);
            check_tree(T);
            const double real = rtt::tree_cost(T);
            CHECK(std::abs(c - real) <= 1e-9 * real);
            CHECK(real <= prev * (1.0 + 1e-12));
            std::printf("median n %d pass %d: SAH cost %.6g -> %.6g\n", n, pass, prev, real);
            prev = real;
        }
    }
    if (fails) return 1;
    std::printf("treelet: ok\n");
    return 0;
}
