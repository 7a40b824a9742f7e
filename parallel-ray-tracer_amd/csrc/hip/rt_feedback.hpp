// rt_feedback.hpp — per-frame cost feedback for the drop-in's frame loop (single 1-spp frames, RT_VARIANT_HYBRID).
//
// The reference renders and waits frame by frame (cpu/src/main.c:171-185; gpu/src/main.cu:111-114 -> gpu.cu:98-127), so
// a single frame is as long as its slowest tile, and the order in which the persistent waves take the tiles decides
// how much of the chip that tail leaves idle. Every frame's kernels record each 8x8 tile's duration (one s_memrealtime
// pair per tile, KArgs::tile_cost), and a hybrid candidate's frame -- tried or chosen by the default rule -- builds its
// tile lists from the previous frame's on the device, before its kernels, on the same stream: the tiles over pct % of
// the costliest (and over twice the mean) go to k_coop (hottest first), the others to the cold kernel costliest first
// within each XCD region (longest processing time first). No measuring frame after the first, no host round trip: a
// moving camera's lists are one frame old instead of up to 64 (the periodic refresh they replace), priced by each
// tile's neighbourhood when the camera moved (FbArgs::moved).
//
// The order of the tiles changes which wave renders a pixel and when, never what it computes: every frame is bit-exact
// whatever the lists hold (tests/test_gpu_seam.py).
#pragma once
#include "rt_device.hpp"

namespace rtd {

struct FbArgs {
    unsigned* cost;        // [n_tiles]: the last frame's 8x8 tile durations (KArgs::tile_cost)
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
    unsigned* table;       // [FB_G][FB_TK]: each workgroup's key counts (k_fb_count -> k_fb_place)
    unsigned* part;        // [3 FB_G]: k_fb_max's per-workgroup maxima and totals (fb_frame)
    int moved;             // the camera differs from the last frame's: the costs have moved with the image by up to
                           // about a tile, so each tile is priced as the costliest of itself and its 4 neighbours (a
                           // car_boxed walkthrough -7 %; kept off for a fixed camera, where it costs +5 %)
    unsigned* cost_next;   // [n_tiles + 1]: this frame's durations, cleared by k_fb_max (not read by the builder)
    unsigned long long* zero64;  // nullable: the frame's ray counters, n64 of them, cleared by k_fb_max
    int n64;
    unsigned* zero32;      // the persistent kernels' work counters, n32 words, cleared by k_fb_max
    int n32;
};

constexpr int FB_NB = 64;  // cost buckets: 8 per octave below the costliest tile, 8 octaves (cheaper: the last)
constexpr int FB_THREADS = 1024;
constexpr int FB_G = 16;      // workgroups (CUs) of each builder kernel: LDS atomics run ~1 lane per clock per CU, and
                              // one CU for a 1080p frame's 32400 tiles took ~35 us
constexpr int FB_KEYS = 9 * FB_NB;          // list keys: hot bucket b; cold (region r, bucket b): FB_NB (1 + r) + b
constexpr int FB_TK = FB_KEYS + 8 * FB_NB;  // + the hot tiles again as cold keys (region r, bucket b): a hot set over
                                            // hot_cap drops its cheapest buckets to the cold lists (k_fb_place)

// log2(c) in 1/8 octaves (exponent and the mantissa's top 3 bits)
__host__ __device__ inline int fb_log8(unsigned c) {
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

// The three kernels (FB_G workgroups of FB_THREADS each, workgroup g owning a contiguous 1/FB_G of the tiles, tile
// t = t0 + thread + FB_THREADS j) form a counting sort by (group, bucket) -- hot tiles by bucket, costliest first, then
// each region's cold tiles by bucket; tile order within a bucket does not matter (any order renders the same frame):
//   k_fb_max   the costliest tile (the buckets are relative to it) and the tiles' total, per workgroup
//   k_fb_count each workgroup's key counts, in its LDS, to table
//   k_fb_place every workgroup sums the table (its cursors: the keys before, the workgroups before it), caps the hot
//              set at hot_cap (cheapest hot buckets to the cold lists), and scatters its tiles through LDS cursors.
struct FbTile {  // a tile's key and weight under the frame's costliest tile
    int b, grp;  // bucket; group: -1 past the tiles, 0 hot, 1 + region cold
    unsigned w;  // hot: its hot-kernel tiles
};
// The frame's costliest tile and its tiles' total, from k_fb_max's per-workgroup partials (part: [FB_G] maxima, then
// [FB_G] totals as lo, hi word pairs), read once per workgroup into LDS by its first thread
struct FbFrame {
    unsigned cmax;
    unsigned long long sum;
};
__device__ __forceinline__ FbFrame fb_frame(const FbArgs& F) {
    __shared__ FbFrame s;
    if (threadIdx.x == 0) {
        FbFrame f{1u, 0ull};
        for (int g = 0; g < FB_G; g++) {
            f.cmax = max(f.cmax, F.part[g]);
            f.sum += (unsigned long long)F.part[FB_G + 2 * g] | (unsigned long long)F.part[FB_G + 2 * g + 1] << 32;
        }
        s = f;
    }
    __syncthreads();
    return s;
}
// hot: over pct % of the costliest tile AND over twice the mean tile -- a frame of even cost (a camera that looks
// past the model) has no hot tiles at all; by the first test alone half its tiles went to k_coop (a dragon871k
// walkthrough's frames 0.33 -> 2-4 ms when the model left the view under a choice made while it was in it)
__device__ __forceinline__ FbTile fb_tile(const FbArgs& F, int t, const FbFrame& fr) {
    const unsigned cmax = fr.cmax;
    FbTile r{0, -1, 1u};
    if (t >= F.n_tiles) return r;
    unsigned v = F.cost[t];
    if (F.moved) {  // the camera moved: a tile priced as the costliest of itself and its 4 neighbours
        const int x = t % F.tx;
        if (x > 0) v = max(v, F.cost[t - 1]);
        if (x + 1 < F.tx) v = max(v, F.cost[t + 1]);
        if (t >= F.tx) v = max(v, F.cost[t - F.tx]);
        if (t + F.tx < F.n_tiles) v = max(v, F.cost[t + F.tx]);
    }
    const int inf = F.info[t];
    r.b = v == 0u ? FB_NB - 1 : min(FB_NB - 1, fb_log8(cmax) - fb_log8(v));
    if (F.pct > 0 && (unsigned long long)v * 100ull > (unsigned long long)F.pct * cmax &&
        (unsigned long long)v * (unsigned long long)F.n_tiles > 2ull * fr.sum) {
        r.grp = 0;
        r.w = (unsigned)(F.tw == 4 ? (inf >> 3) & 7 : inf >> 6);
    } else {
        r.grp = 1 + (inf & 7);
    }
    return r;
}
__device__ __forceinline__ int fb_t0(const FbArgs& F) { return blockIdx.x * ((F.n_tiles + FB_G - 1) / FB_G); }
__device__ __forceinline__ int fb_t1(const FbArgs& F) { return min(F.n_tiles, fb_t0(F) + (F.n_tiles + FB_G - 1) / FB_G); }

__global__ __launch_bounds__(FB_THREADS) void k_fb_max(FbArgs F) {
    __shared__ unsigned part[FB_THREADS / 64];
    __shared__ unsigned long long s_sum;
    if (threadIdx.x == 0) s_sum = 0ull;
    __syncthreads();
    const int t1 = fb_t1(F);
    unsigned m = 0u;
    unsigned long long sum = 0ull;
    for (int t = fb_t0(F) + (int)threadIdx.x; t < t1; t += FB_THREADS) {
        const unsigned v = F.cost[t];
        m = max(m, v);
        sum += v;
        F.cost_next[t] = 0u;  // (this frame's buffer: the three memsets a frame launched before, folded in here)
    }
    if (sum) atomicAdd(&s_sum, sum);
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) F.cost_next[F.n_tiles] = 0u;
        if (F.zero64)
            for (int i = threadIdx.x; i < F.n64; i += FB_THREADS) F.zero64[i] = 0ull;
        for (int i = threadIdx.x; i < F.n32; i += FB_THREADS) F.zero32[i] = 0u;
    }
    for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, 64));
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x < 64) {
        m = threadIdx.x < FB_THREADS / 64 ? part[threadIdx.x] : 0u;
        for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, 64));
        if (threadIdx.x == 0) {  // this workgroup's partials (no atomics, nothing to clear between frames)
            F.part[blockIdx.x] = m;
            F.part[FB_G + 2 * blockIdx.x] = (unsigned)s_sum;
            F.part[FB_G + 2 * blockIdx.x + 1] = (unsigned)(s_sum >> 32);
        }
    }
}

__global__ __launch_bounds__(FB_THREADS) void k_fb_count(FbArgs F) {
    __shared__ unsigned h[FB_TK];
    for (int k = threadIdx.x; k < FB_TK; k += FB_THREADS) h[k] = 0u;
    const FbFrame fr = fb_frame(F);  // (its barrier also orders the clearing above)
    const int t1 = fb_t1(F);
    for (int t = fb_t0(F) + (int)threadIdx.x; t < t1; t += FB_THREADS) {
        const FbTile q = fb_tile(F, t, fr);
        if (q.grp == 0) {
            atomicAdd(&h[q.b], q.w);
            atomicAdd(&h[FB_KEYS + (F.info[t] & 7) * FB_NB + q.b], 1u);
        } else {
            atomicAdd(&h[q.grp * FB_NB + q.b], 1u);
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < FB_TK; k += FB_THREADS) F.table[blockIdx.x * FB_TK + k] = h[k];
}

__global__ __launch_bounds__(FB_THREADS) void k_fb_place(FbArgs F) {
    __shared__ unsigned tot[FB_TK], mine[FB_TK], cur[FB_KEYS];
    __shared__ unsigned part[FB_THREADS / 64];
    __shared__ int s_cut;
    __shared__ unsigned s_nhot;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = blockIdx.x;
    for (int k = tid; k < FB_TK; k += FB_THREADS) {  // the key's total, and its count in the workgroups before this one
        unsigned a = 0u, b = 0u;
#pragma unroll
        for (int q = 0; q < FB_G; q++) {
            const unsigned v = F.table[q * FB_TK + k];
            a += v;
            b += q < g ? v : 0u;
        }
        tot[k] = a;
        mine[k] = b;
    }
    __syncthreads();
    if (wave == 0) {  // the hot buckets, costliest first, while they fit hot_cap (one per lane)
        unsigned inc = tot[lane];
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned u = (unsigned)__shfl_up((int)inc, o, 64);
            if (lane >= o) inc += u;
        }
        const unsigned long long over = __ballot(inc > (unsigned)F.hot_cap);
        if (lane == 0) s_cut = over ? __builtin_ctzll(over) : FB_NB;
    }
    __syncthreads();
    const int cut = s_cut;
    // the list keys' counts under the cut, exclusive scan over the keys (FB_KEYS <= FB_THREADS: one per thread)
    unsigned e = 0u, em = 0u;
    if (tid < FB_KEYS) {
        const int b = tid % FB_NB;
        if (tid < FB_NB) {
            e = b < cut ? tot[tid] : 0u;
            em = b < cut ? mine[tid] : 0u;
        } else {
            const int dk = FB_KEYS + tid - FB_NB;  // the same (region, bucket) among the hot tiles
            e = tot[tid] + (b >= cut ? tot[dk] : 0u);
            em = mine[tid] + (b >= cut ? mine[dk] : 0u);
        }
    }
    unsigned inc = e;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned u = (unsigned)__shfl_up((int)inc, o, 64);
        if (lane >= o) inc += u;
    }
    if (lane == 63) part[wave] = inc;
    __syncthreads();
    unsigned before = 0u;
    for (int w = 0; w < wave; w++) before += part[w];
    const unsigned start = before + inc - e;  // the key's first slot in the lists (hot part, then cold part)
    if (tid < FB_KEYS) cur[tid] = start + em;
    if (tid == FB_NB) s_nhot = start;  // (the first cold key's start: the hot total)
    __syncthreads();
    const unsigned nhot = s_nhot;
    if (g == 0) {  // (thread FB_KEYS: e = 0, start = the lists' total)
        if (tid == 0) F.counts[0] = (int)nhot;
        if (tid >= FB_NB && tid < FB_KEYS && tid % FB_NB == 0) F.cold[tid / FB_NB - 1] = (int)(start - nhot);
        if (tid == FB_KEYS) F.cold[8] = (int)(start - nhot);
    }
    const FbFrame fr = fb_frame(F);
    const int t1 = fb_t1(F);
    for (int t = fb_t0(F) + tid; t < t1; t += FB_THREADS) {
        const FbTile q = fb_tile(F, t, fr);
        if (q.grp == 0 && q.b < cut) {  // a hot tile: its hot-kernel tiles
            int p = (int)atomicAdd(&cur[q.b], q.w);
            const int sx = 8 / F.tw, sy = 8 / F.th, x0 = (t % F.tx) * sx, y0 = (t / F.tx) * sy;
            for (int qy = 0; qy < sy; qy++)
                for (int qx = 0; qx < sx; qx++)
                    if (x0 + qx < F.ctw && y0 + qy < F.cth) F.hot[p++] = (y0 + qy) * F.ctw + x0 + qx;
        } else {
            const int k = (q.grp == 0 ? 1 + (F.info[t] & 7) : q.grp) * FB_NB + q.b;
            F.cold[9 + (int)(atomicAdd(&cur[k], 1u) - nhot)] = t;
        }
    }
}

}  // namespace rtd
