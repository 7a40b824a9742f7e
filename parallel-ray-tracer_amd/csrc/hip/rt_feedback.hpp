// rt_feedback.hpp — per-frame cost feedback for the drop-in's frame loop (single 1-spp frames, RT_VARIANT_HYBRID).
//
// The reference renders and waits frame by frame (cpu/src/main.c:171-185; gpu/src/main.cu:111-114 -> gpu.cu:98-127), so
// a single frame is as long as its slowest tile, and the order in which the persistent waves take the tiles decides
// how much of the chip that tail leaves idle. Once the default rule has chosen a configuration for the frame shape,
// every frame's kernels record each 8x8 tile's duration (one s_memrealtime pair per tile, KArgs::tile_cost), and the
// next frame's tile lists are built from them on the device, before its kernels, on the same stream: the tiles over
// pct % of the costliest go to k_coop (the chosen candidate's hot tiles, hottest first), the others to the cold kernel
// costliest first within each XCD region (longest processing time first). No measuring frame, no host round trip: a
// moving camera's lists are one frame old instead of up to 64 (the periodic refresh they replace).
//
// The order of the tiles changes which wave renders a pixel and when, never what it computes: every frame is bit-exact
// whatever the lists hold (tests/test_gpu_seam.py).
#pragma once
#include "rt_device.hpp"

namespace rtd {

struct FbArgs {
    const unsigned* cost;  // [n_tiles]: the last frame's 8x8 tile durations (KArgs::tile_cost)
    int n_tiles, tx, ty;   // the 8x8 tile grid of the frame's compact rows
    int pct;               // hot tiles: cost > pct % of the costliest (0: none)
    int hot_cap;           // at most this many hot-kernel tiles (the hottest; k_coop spends ~2x the wave time per ray)
    int tw, th, ctw, cth;  // the hot kernel's pixel tile (rt_coop.hpp GTile) and its tile grid
    int xcd_mode;          // region layout of the cold tiles (rt_hip.hip region_layout): 1 rows, 2 columns, 3 blocks,
                           // 0 one region
    const unsigned char* info;  // per 8x8 tile, fixed for the shape: region (bits 0-2), its k_coop<4> tiles (bits 3-5),
                                // its k_coop<2> tiles (bits 6-7) -- no division per tile in the kernel (fb_tile_info)
    int* hot;              // the hot kernel's tiles, hottest first
    int* cold;             // [9 region offsets into the tile part][the cold 8x8 tiles, region by region, costliest first]
    int* counts;           // [0]: the hot kernel's tiles
};

constexpr int FB_NB = 64;  // cost buckets: 8 per octave below the costliest tile, 8 octaves (cheaper: the last)
constexpr int FB_THREADS = 1024;
constexpr int FB_WAVES = FB_THREADS / 64;
constexpr int FB_GROUPS = 9;  // hot, then the 8 regions' cold tiles
constexpr int FB_KEYS = FB_GROUPS * FB_NB;

// log2(c) in 1/8 octaves (exponent and the mantissa's top 3 bits)
__device__ __forceinline__ int fb_log8(unsigned c) {
    if (c == 0u) return 0;
    const int e = 31 - __builtin_clz(c);
    const unsigned frac = e >= 3 ? (c >> (e - 3)) & 7u : (c << (3 - e)) & 7u;
    return e * 8 + (int)frac;
}
// the per-tile info byte (host: rt_hip.hip fb_info): region | k_coop<4> tiles << 3 | k_coop<2> tiles << 6, each
// hot-kernel count clipped at the frame's edge
__host__ __device__ inline unsigned char fb_tile_info(int t, int tx, int ty, int mode, int W, int rows) {
    const int x = t % tx, y = t / tx;
    const int reg = mode == 1 ? y * 8 / ty : mode == 2 ? x * 8 / tx : mode == 3 ? x * 4 / tx + 4 * (y * 2 / ty) : 0;
    auto nsub = [&](int tw, int th) {
        const int ctw = (W + tw - 1) / tw, cth = (rows + th - 1) / th, sx = 8 / tw, sy = 8 / th;
        const int x0 = x * sx, y0 = y * sy;
        return (ctw - x0 < sx ? ctw - x0 : sx) * (cth - y0 < sy ? cth - y0 : sy);
    };
    return (unsigned char)(reg | nsub(4, 4) << 3 | nsub(8, 4) << 6);
}

// One workgroup of 16 waves, wave w owning a contiguous 1/16 of the tiles: the costliest tile (reduction), the hot set
// (capped at hot_cap, costliest buckets first), then a counting sort by (group, bucket) -- per-wave counts in LDS (no
// wave contends with another), one exclusive scan in (group, bucket, wave) order, a scatter through the per-wave
// cursors. The order is costliest bucket first, then tile order within a bucket. The durations come from the other
// XCDs' kernels (memory, not this L2): each pass loads FB_PER of a lane's tiles at once, so that their latencies overlap
// (one load at a time made this kernel ~45 us of a 0.95-ms frame).
constexpr int FB_PER = 32;
__global__ __launch_bounds__(FB_THREADS) void k_fb_lists(FbArgs F) {
    __shared__ unsigned cnt[FB_KEYS * FB_WAVES];  // [key][wave]
    __shared__ unsigned part[FB_WAVES];
    __shared__ unsigned s_max, s_nhot, s_cut;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nt = F.n_tiles, chunk = (nt + FB_WAVES - 1) / FB_WAVES;
    const int t0 = wave * chunk, t1 = min(nt, t0 + chunk);
    for (int i = tid; i < FB_KEYS * FB_WAVES; i += FB_THREADS) cnt[i] = 0u;
    // the lane's tiles t0 + lane + 64 i, FB_PER at a time: cost (0 past the wave's tiles) and info
    unsigned c[FB_PER];
    unsigned char inf[FB_PER];
    auto load = [&](int base) {
#pragma unroll
        for (int i = 0; i < FB_PER; i++) {
            const int t = t0 + lane + 64 * (base + i);
            c[i] = t < t1 ? F.cost[t] : 0u;
            inf[i] = t < t1 ? F.info[t] : (unsigned char)0;
        }
    };
    const int iters = (chunk + 63) / 64;
    unsigned m = 0u;
    for (int base = 0; base < iters; base += FB_PER) {
        load(base);
#pragma unroll
        for (int i = 0; i < FB_PER; i++) m = max(m, c[i]);
    }
    for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, 64));
    if (lane == 0) part[wave] = m;
    if (tid == 0) {
        s_nhot = 0u;
        s_cut = FB_NB;
    }
    __syncthreads();
    if (tid == 0) {
        unsigned mm = 1u;
        for (int w = 0; w < FB_WAVES; w++) mm = max(mm, part[w]);
        s_max = mm;
    }
    __syncthreads();
    const unsigned cmax = s_max;
    const int lmax = fb_log8(cmax);
    const unsigned long long thr = (unsigned long long)F.pct * cmax;
    auto is_hot = [&](unsigned v) { return F.pct > 0 && (unsigned long long)v * 100ull > thr; };
    auto bucket = [&](unsigned v) { return v == 0u ? FB_NB - 1 : min(FB_NB - 1, lmax - fb_log8(v)); };
    int cut = FB_NB;
    auto key_of = [&](int i, unsigned& w) -> int {  // group * FB_NB + bucket; w: hot-kernel tiles (hot) or 1
        const int b = bucket(c[i]);
        if (is_hot(c[i]) && b < cut) {
            w = (unsigned)(F.tw == 4 ? (inf[i] >> 3) & 7 : inf[i] >> 6);
            return b;
        }
        w = 1u;
        return (1 + (inf[i] & 7)) * FB_NB + b;
    };
    for (int pass = 0; pass < 2; pass++) {  // the histogram; again with a cut when the hot set exceeds hot_cap (rare)
        unsigned nh = 0u;
        for (int base = 0; base < iters; base += FB_PER) {
            load(base);
#pragma unroll
            for (int i = 0; i < FB_PER; i++) {
                const int t = t0 + lane + 64 * (base + i);
                if (t >= t1) continue;
                unsigned w;
                const int k = key_of(i, w);
                if (k < FB_NB) nh += w;
                atomicAdd(&cnt[k * FB_WAVES + wave], w);
            }
        }
        for (int o = 32; o > 0; o >>= 1) nh += (unsigned)__shfl_xor((int)nh, o, 64);
        if (lane == 0 && nh) atomicAdd(&s_nhot, nh);
        __syncthreads();
        if (pass == 1 || s_nhot <= (unsigned)F.hot_cap) break;
        if (wave == 0) {  // the hot buckets, costliest first, while they fit hot_cap (64 buckets: one per lane)
            unsigned v = 0u;
            for (int w = 0; w < FB_WAVES; w++) v += cnt[lane * FB_WAVES + w];  // (hot tiles' k_coop tiles: >= 1 each)
            unsigned inc = v;
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned u = (unsigned)__shfl_up((int)inc, o, 64);
                if (lane >= o) inc += u;
            }
            const unsigned long long over = __ballot(inc > (unsigned)F.hot_cap);
            if (lane == 0) s_cut = over ? (unsigned)__builtin_ctzll(over) : (unsigned)FB_NB;
        }
        __syncthreads();
        cut = (int)s_cut;
        for (int i = tid; i < FB_KEYS * FB_WAVES; i += FB_THREADS) cnt[i] = 0u;
        __syncthreads();
    }
    // exclusive scan of the [key][wave] counts in place: PER consecutive counts per thread, then the threads' sums
    constexpr int PER = FB_KEYS * FB_WAVES / FB_THREADS;
    static_assert(PER * FB_THREADS == FB_KEYS * FB_WAVES, "scan layout");
    unsigned loc[PER], sum = 0u;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        loc[k] = cnt[tid * PER + k];
        sum += loc[k];
    }
    unsigned inc = sum;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned v = (unsigned)__shfl_up((int)inc, o, 64);
        if (lane >= o) inc += v;
    }
    if (lane == 63) part[wave] = inc;
    __syncthreads();
    if (tid == 0) {
        unsigned run = 0u;
        for (int w = 0; w < FB_WAVES; w++) {
            const unsigned v = part[w];
            part[w] = run;
            run += v;
        }
    }
    __syncthreads();
    unsigned at = part[wave] + inc - sum;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        cnt[tid * PER + k] = at;
        at += loc[k];
    }
    __syncthreads();
    const unsigned nhot = cnt[FB_NB * FB_WAVES];  // the hot group's total (the first cold key's start)
    if (tid == 0) F.counts[0] = (int)nhot;
    if (tid < 8) F.cold[tid] = (int)(cnt[(1 + tid) * FB_NB * FB_WAVES] - nhot);  // region r's start in the tile part
    __syncthreads();  // (the region starts read before the scatter moves the cursors)
    for (int base = 0; base < iters; base += FB_PER) {  // scatter through the wave's cursors
        load(base);
#pragma unroll
        for (int i = 0; i < FB_PER; i++) {
            const int t = t0 + lane + 64 * (base + i);
            if (t >= t1) continue;
            unsigned w;
            const int k = key_of(i, w);
            const unsigned pos = atomicAdd(&cnt[k * FB_WAVES + wave], w);
            if (k < FB_NB) {  // a hot tile: its hot-kernel tiles
                const int sx = 8 / F.tw, sy = 8 / F.th, x0 = (t % F.tx) * sx, y0 = (t / F.tx) * sy;
                int p = (int)pos;
                for (int qy = 0; qy < sy; qy++)
                    for (int qx = 0; qx < sx; qx++)
                        if (x0 + qx < F.ctw && y0 + qy < F.cth) F.hot[p++] = (y0 + qy) * F.ctw + x0 + qx;
            } else {
                F.cold[9 + (int)(pos - nhot)] = t;
            }
        }
    }
    __syncthreads();
    if (tid == 0) F.cold[8] = (int)(cnt[FB_KEYS * FB_WAVES - 1] - nhot);  // the last cursor: the cold total
}

}  // namespace rtd
