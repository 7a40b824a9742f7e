// Stand-alone timing of the feedback list builder (rt_feedback.hpp: k_fb_max, k_fb_count, k_fb_place) on synthetic tile costs, away from the
// frame's kernels: 1080p's 8x8 tile grid, costs log-normal around ~5 us of s_memrealtime ticks, region layout 3.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude -Iparallel-ray-tracer_amd/csrc/hip tools/fb_bench.hip -o /tmp/fb_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "rt_feedback.hpp"

#define CK(x)                                                                      \
    do {                                                                           \
        if ((x) != hipSuccess) {                                                   \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, #x);            \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main(int argc, char** argv) {
    const int W = 1920, H = 1080, tx = (W + 7) / 8, ty = (H + 7) / 8, nt = tx * ty;
    const int pct = argc > 1 ? std::atoi(argv[1]) : 0;
    const double flat = argc > 2 ? std::atof(argv[2]) : 0.0;  // this share of the tiles (a band of rows): one cost
    std::mt19937 rng(7);
    std::lognormal_distribution<double> L(std::log(500.0), 0.8);
    std::vector<unsigned> cost(nt);
    std::vector<unsigned char> info(nt);
    for (int t = 0; t < nt; t++) {
        cost[t] = t < flat * nt ? 120u : (unsigned)L(rng);
        info[t] = rtd::fb_tile_info(t, tx, ty, 3, W, H);
    }
    unsigned *d_cost, *d_table;
    unsigned char* d_info;
    int *d_hot, *d_cold, *d_counts;
    CK(hipMalloc(&d_cost, (nt + 1) * 4));
    CK(hipMalloc(&d_table, rtd::FB_G * (rtd::FB_TK + 3) * 4));
    unsigned* d_next;
    CK(hipMalloc(&d_next, (nt + 1) * 4));
    cost.push_back(0u);
    CK(hipMalloc(&d_info, nt));
    CK(hipMalloc(&d_hot, 4 * nt * 4));
    CK(hipMalloc(&d_cold, (9 + nt) * 4));
    CK(hipMalloc(&d_counts, 16));
    CK(hipMemcpy(d_cost, cost.data(), (nt + 1) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_info, info.data(), nt, hipMemcpyHostToDevice));
    rtd::FbArgs F{d_cost, nt, tx, ty, pct, nt, 4, 4, (W + 3) / 4, (H + 3) / 4, 3, d_info, d_hot, d_cold, d_counts, d_table, d_table + rtd::FB_G * rtd::FB_TK, 0, d_next, nullptr, 0, nullptr, 0};
    auto run = [&]() {
        rtd::k_fb_max<<<rtd::FB_G, rtd::FB_THREADS>>>(F);
        rtd::k_fb_count<<<rtd::FB_G, rtd::FB_THREADS>>>(F);
        rtd::k_fb_place<<<rtd::FB_G, rtd::FB_THREADS>>>(F);
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 5; i++) run();
    CK(hipDeviceSynchronize());
    const int reps = 50;
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; i++) run();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<int> cold(9 + nt), counts(4);
    CK(hipMemcpy(cold.data(), d_cold, (9 + nt) * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(counts.data(), d_counts, 16, hipMemcpyDeviceToHost));
    // check: every cold tile once, regions in order, costliest bucket first within a region
    std::vector<int> seen(nt, 0);
    for (int i = 0; i < cold[8]; i++) seen[cold[9 + i]]++;
    int bad = 0;
    for (int t = 0; t < nt; t++) bad += seen[t] > 1 || (!pct && seen[t] != 1);
    std::vector<int> hot(4 * nt);  // with a hot set: every tile once, in one list or the other
    CK(hipMemcpy(hot.data(), d_hot, 4 * nt * 4, hipMemcpyDeviceToHost));
    std::vector<int> hs(nt, 0);
    const int ctw = (W + 3) / 4;
    for (int i = 0; i < counts[0]; i++) hs[(hot[i] / ctw / 2) * tx + (hot[i] % ctw) / 2]++;
    for (int t = 0; t < nt; t++) bad += (hs[t] > 0) + seen[t] != 1;
    const unsigned cmax = *std::max_element(cost.begin(), cost.end());
    auto bk = [&](unsigned c) { return c ? std::min(63, rtd::fb_log8(cmax) - rtd::fb_log8(c)) : 63; };
    for (int r = 0; r < 8; r++) {  // within a region: costliest bucket first
        const int b = cold[r], e = r < 7 ? cold[r + 1] : cold[8];
        for (int i = b + 1; i < e; i++) {  // (buckets as the kernel's: costliest first)
            const unsigned u = cost[cold[9 + i - 1]], v = cost[cold[9 + i]];
            bad += bk(v) < bk(u);
        }
    }
    std::printf("fb lists: %.2f us per launch (%d tiles, pct %d, flat %.2f): hot %d cold %d, region starts %d %d %d %d %d %d %d %d, bad %d\n",
                1000.f * ms / reps, nt, pct, flat, counts[0], cold[8], cold[0], cold[1], cold[2], cold[3], cold[4], cold[5], cold[6],
                cold[7], bad);
    return bad != 0;
}
