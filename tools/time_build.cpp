// Host timing of the acceleration build's CPU stages (no GPU): load an OBJ, build the binned-SAH binary BVH
// (librt_host.so), run the treelet passes (rt_treelet.hpp) on it and the 8-wide collapse (rth_wbvh_build_cost); prints
// milliseconds per stage and a checksum of the results, so that a parallel version can be compared with the
// sequential one. usage: tools/time_build <obj> <mtl> [threads]
//   g++ -O2 -std=c++17 -pthread -Iinclude -Iparallel-ray-tracer_amd/csrc/hip tools/time_build.cpp \
//       -Lparallel-ray-tracer_amd/lib -lrt_host -Wl,-rpath,$PWD/parallel-ray-tracer_amd/lib -o /tmp/time_build
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rt_host.h"
#include "rt_treelet.hpp"

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const int threads = argc > 3 ? std::atoi(argv[3]) : 1;
    rt_triangle* T = nullptr;
    size_t n = 0;
    auto t0 = std::chrono::steady_clock::now();
    if (rth_triangles_load(argv[1], argv[2], &T, &n)) return 1;
    std::printf("load %.1f ms, %zu triangles\n", ms_since(t0), n);
    rt_bvh_node* nodes = nullptr;
    int nlen = 0;
    int* idx = nullptr;
    t0 = std::chrono::steady_clock::now();
    if (rth_bvh_build(T, n, RTH_BVH_BINNED_SAH, nullptr, &nodes, &nlen, &idx, nullptr)) return 1;
    std::printf("binned SAH %.1f ms, %d nodes\n", ms_since(t0), nlen);
    // the binary tree as rtt::Tree: the BVH's leaves as its leaves
    rtt::Tree tr;
    std::vector<int> leaf_of(nlen, -1), inner_of(nlen, -1);
    int nl = 0;
    for (int i = 0; i < nlen; i++)
        if (nodes[i].tr_len > 0) leaf_of[i] = nl++;
    tr.n = nl;
    tr.box.resize(2 * (size_t)nl - 1);
    tr.left.resize(nl - 1);
    tr.right.resize(nl - 1);
    int ni = nl;
    for (int i = 0; i < nlen; i++)
        if (nodes[i].tr_len == 0 && nodes[i].child > 0) inner_of[i] = ni++;
    auto id = [&](int i) { return leaf_of[i] >= 0 ? leaf_of[i] : inner_of[i]; };
    for (int i = 0; i < nlen; i++) {
        const int k = id(i);
        if (k < 0) continue;
        tr.box[k] = rtt::Box{{nodes[i].min.x, nodes[i].min.y, nodes[i].min.z}, {nodes[i].max.x, nodes[i].max.y, nodes[i].max.z}};
        if (inner_of[i] >= 0) {
            tr.left[k - nl] = id(nodes[i].child);
            tr.right[k - nl] = id(nodes[i].child + 1);
        }
    }
    tr.root = id(0);
    const double c0 = rtt::tree_cost(tr);
    t0 = std::chrono::steady_clock::now();
    for (int p = 0; p < 2; p++) rtt::optimize_pass(tr, threads);
    const double c2 = rtt::tree_cost(tr);
    long long sum = 0;
    for (size_t i = 0; i < tr.left.size(); i++) sum = sum * 31 + tr.left[i] * 7 + tr.right[i];
    std::printf("treelet x2 %.1f ms (threads %d), SAH %.6g -> %.6g, topology checksum %lld\n", ms_since(t0), threads, c0, c2,
                sum);
    uint32_t* words = nullptr;
    int* order = nullptr;
    rth_wbvh_info wi{};
    t0 = std::chrono::steady_clock::now();
    if (rth_wbvh_build_cost(nodes, nlen, idx, T, (int)n, 1e-3f, 2.0f, &words, &order, &wi)) return 1;
    unsigned long long h = 1469598103934665603ull;
    for (int i = 0; i < 20 * wi.n_nodes; i++) h = (h ^ words[i]) * 1099511628211ull;
    std::printf("wide collapse %.1f ms, %d wide nodes, depth %d, words hash %016llx\n", ms_since(t0), wi.n_nodes, wi.depth, h);
    return 0;
}
