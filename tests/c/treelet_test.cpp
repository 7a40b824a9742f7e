// g++ test of rt_treelet.hpp (no GPU): a random binary tree over random boxes, restructured by treelets, stays a
// BVH of the same leaves -- every leaf once, every internal box the union of its children's, the root's box unchanged
// -- and its SAH cost does not rise; a second pass changes less than the first.
#include "rt_treelet.hpp"

#include <cstdio>
#include <cstdlib>
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
    if (fails) return 1;
    std::printf("treelet: ok\n");
    return 0;
}
