// rt_coop.hpp — group-cooperative wide walk: G lanes (2, 4 or 8) trace ONE ray together.
//
// Why: a frame ends when its slowest tile does, and a tile's cost is a chain of dependent wide-node
// visits (PRT_TILE_TRACE, bench frame: the slowest 8x8 tile takes ~710 wave steps at ~2.1 us each,
// ~1.4 ms, whether the chip is full or 87 % idle — it is latency, not throughput: one lane tests 8
// child boxes (~250 instructions) and then the hit leaves' triangles one after another, each behind a
// dependent load). With the frame split over 8 GPUs the chip runs 1.3 tiles per wave and the frame is
// that chain: 1.7x at 8 GPUs. Here the G lanes of a group split each visit: lane q tests child slots
// q, q + G, ... (8 / G of them) and the group ORs its hit bits with DPP (quad_perm / row_half_mirror,
// no LDS); the hit leaves' triangles are dealt round-robin, G per round; the best hit is merged with
// DPP min. A wave traces 64 / G rays (a TW x TH pixel tile), each visit is ~G x shorter, and fewer rays
// per wave means less divergence.
//
// Control flow is uniform within a group (every branch depends on merged values), so the group's lanes
// are always all active or all inactive and DPP inside a quad / half-row only reads active lanes.
// Each lane keeps its own copy of the traversal stack (its LDS column) and of the ray state; shading
// and the strict fallback walk run redundantly in every lane of the group (same values, same bits).
//
// Result semantics equal closest_wide / visible_wide (rt_kernels.hpp), which equal the reference's:
//   closest: min t over all triangles; an exact tie of the final t (reference: first found wins,
//            bvh.c:331) is reported and re-walked strictly. Merge rule: the group best is the lanes'
//            min; tie = a lane at that min saw a tie, or two lanes at the min hold different triangles.
//   visible: occluded iff some triangle nearer than the light (bvh.c:283-290): the group ORs its lanes'
//            occlusion flags after each round.
#pragma once
#include "rt_kernels.hpp"

namespace rtd {

// DPP lane exchange within a quad / half-row (all lanes of the group active)
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u(unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
constexpr int DPP_QUAD_1032 = 0xB1;  // quad_perm [1,0,3,2]: lane ^ 1
constexpr int DPP_QUAD_2301 = 0x4E;  // quad_perm [2,3,0,1]: lane ^ 2
constexpr int DPP_HALF_MIRROR = 0x141;  // row_half_mirror: lane i <-> 7 - i within 8 lanes

template <int G>
__device__ __forceinline__ unsigned g_or(unsigned v) {
    if (G >= 2) v |= dpp_u<DPP_QUAD_1032>(v);
    if (G >= 4) v |= dpp_u<DPP_QUAD_2301>(v);
    if (G >= 8) v |= dpp_u<DPP_HALF_MIRROR>(v);
    return v;
}
template <int G>
__device__ __forceinline__ float g_minf(float v) {
    if (G >= 2) v = fminf(v, dpp_f<DPP_QUAD_1032>(v));
    if (G >= 4) v = fminf(v, dpp_f<DPP_QUAD_2301>(v));
    if (G >= 8) v = fminf(v, dpp_f<DPP_HALF_MIRROR>(v));
    return v;
}
template <int G>
__device__ __forceinline__ int g_mini(int v) {
    if (G >= 2) v = min(v, (int)dpp_u<DPP_QUAD_1032>((unsigned)v));
    if (G >= 4) v = min(v, (int)dpp_u<DPP_QUAD_2301>((unsigned)v));
    if (G >= 8) v = min(v, (int)dpp_u<DPP_HALF_MIRROR>((unsigned)v));
    return v;
}
template <int G>
__device__ __forceinline__ int g_maxi(int v) {
    if (G >= 2) v = max(v, (int)dpp_u<DPP_QUAD_1032>((unsigned)v));
    if (G >= 4) v = max(v, (int)dpp_u<DPP_QUAD_2301>((unsigned)v));
    if (G >= 8) v = max(v, (int)dpp_u<DPP_HALF_MIRROR>((unsigned)v));
    return v;
}

// The group's share of one wide-node visit: lane q tests slots q, q + G, ...; outputs as wide_node's
// (identical in every lane of the group).
template <int G, bool COUNT>
__device__ __forceinline__ void wide_node_g(const WNode& nd, const RayPre& p, unsigned oct, float lim, unsigned q,
                                            unsigned& nh, unsigned& th, int& cbase, int& tbase, unsigned& imask,
                                            unsigned& nleaf) {
    const float4 f0 = nd.f0, f1 = nd.f1, f2 = nd.f2, f3 = nd.f3, f4 = nd.f4;
    const unsigned e = __float_as_uint(f0.w);  // exponents (signed bytes) | interior mask
    imask = e >> 24;
    cbase = __float_as_int(f1.x);
    tbase = __float_as_int(f1.y);
    // the node's grid, as in wide_node (same FMAs, same roundings)
    const float ax = __builtin_fmaf(f0.x, p.ix, -p.ox), ay = __builtin_fmaf(f0.y, p.iy, -p.oy),
                az = __builtin_fmaf(f0.z, p.iz, -p.oz);
    const float kx = __builtin_ldexpf(p.ix, (int)(signed char)(e & 0xFFu)),
                ky = __builtin_ldexpf(p.iy, (int)(signed char)((e >> 8) & 0xFFu)),
                kz = __builtin_ldexpf(p.iz, (int)(signed char)((e >> 16) & 0xFFu));
    const bool bx = (oct & 1u) != 0, by = (oct & 2u) != 0, bz = (oct & 4u) != 0;
    // the slot pairs' plane words per axis (rt_device.hpp: word j = qlo[2j], qhi[2j], qlo[2j+1], qhi[2j+1])
    const unsigned xw[4] = {__float_as_uint(f2.x), __float_as_uint(f2.y), __float_as_uint(f2.z), __float_as_uint(f2.w)},
                   yw[4] = {__float_as_uint(f3.x), __float_as_uint(f3.y), __float_as_uint(f3.z), __float_as_uint(f3.w)},
                   zw[4] = {__float_as_uint(f4.x), __float_as_uint(f4.y), __float_as_uint(f4.z), __float_as_uint(f4.w)};
    // near / far byte of a slot's planes by the octant: lo at bit 16 (s & 1), hi 8 bits above
    const unsigned nxs = bx ? 8u : 0u, fxs = 8u - nxs, nys = by ? 8u : 0u, fys = 8u - nys, nzs = bz ? 8u : 0u,
                   fzs = 8u - nzs;
    unsigned hit = 0;
#pragma unroll
    for (int j = 0; j < 8 / G; j++) {
        const unsigned s = q + (unsigned)(j * G);
        // the pair's word: j * G / 2 + (q >> 1) (G = 2: q >> 1 == 0; G = 4: one of two words, selected)
        const int w0 = j * G / 2;
        const bool w1 = G > 2 && (q >> 1) != 0u;
        const unsigned xs = w1 ? xw[w0 + (G > 2 ? 1 : 0)] : xw[w0], ys = w1 ? yw[w0 + (G > 2 ? 1 : 0)] : yw[w0],
                       zs = w1 ? zw[w0 + (G > 2 ? 1 : 0)] : zw[w0];
        const unsigned sh = 16u * (s & 1u);
        // (plane = 2^e * (QBIAS + q) + p: QBIAS + q is exact in float, the FMA rounds once, as wide_node's fma_mix)
        const float tnx = __builtin_fmaf((float)(QBIAS + ((xs >> (sh + nxs)) & 0xFFu)), kx, ax);
        const float tfx = __builtin_fmaf((float)(QBIAS + ((xs >> (sh + fxs)) & 0xFFu)), kx, ax);
        const float tny = __builtin_fmaf((float)(QBIAS + ((ys >> (sh + nys)) & 0xFFu)), ky, ay);
        const float tfy = __builtin_fmaf((float)(QBIAS + ((ys >> (sh + fys)) & 0xFFu)), ky, ay);
        const float tnz = __builtin_fmaf((float)(QBIAS + ((zs >> (sh + nzs)) & 0xFFu)), kz, az);
        const float tfz = __builtin_fmaf((float)(QBIAS + ((zs >> (sh + fzs)) & 0xFFu)), kz, az);
        const float lo = fmaxf(fmaxf(tnx, tny), fmaxf(tnz, BOX_TMIN));
        const float hi = fminf(fminf(tfx, tfy), fminf(tfz, lim));
        hit |= lo <= hi ? (1u << s) : 0u;
    }
    const unsigned hit8 = g_or<G>(hit);
    unsigned x = hit8 & imask;  // interior hits in visiting order (bit k = slot k ^ oct), as wide_node
    x = (oct & 1u) ? (((x & 0x55u) << 1) | ((x >> 1) & 0x55u)) : x;
    x = (oct & 2u) ? (((x & 0x33u) << 2) | ((x >> 2) & 0x33u)) : x;
    x = (oct & 4u) ? (((x & 0x0Fu) << 4) | ((x >> 4) & 0x0Fu)) : x;
    nh = x;
    const unsigned m[2] = {__float_as_uint(f1.z), __float_as_uint(f1.w)};
    unsigned lh = hit8 & ~imask;
    th = 0;
    nleaf = 0;
    while (lh) {
        const unsigned sl = (unsigned)__builtin_ctz(lh);
        lh &= lh - 1u;
        const unsigned meta = (m[sl >> 2] >> (8u * (sl & 3u))) & 0xFFu;
        th |= ((1u << (meta >> 5)) - 1u) << (meta & 31u);
        if (COUNT) nleaf += meta ? 1u : 0u;
    }
}

// One round of the triangle deal: lane q's triangle bit among the G lowest set bits of `rem` (0: none),
// and `rem` without those G bits.
template <int G>
__device__ __forceinline__ unsigned deal(unsigned& rem, unsigned q) {
    unsigned r = rem, mine = 0;
#pragma unroll
    for (int j = 0; j < G; j++) {
        const unsigned low = r & (0u - r);
        mine = (unsigned)j == q ? low : mine;
        r &= r - 1u;
    }
    rem = r;
    return mine;
}

template <int G, bool COUNT>
__device__ __forceinline__ void closest_wide_g(const DWide& W, v3 o, v3 d, float& best, int& hp, int& nd, bool& tie,
                                               int* __restrict__ stk, Ctr& c, unsigned q) {
    const RayPre p = ray_pre(o, d);
    const unsigned oct = (p.ix < 0.0f ? 1u : 0u) | (p.iy < 0.0f ? 2u : 0u) | (p.iz < 0.0f ? 4u : 0u);
    int sp = 0;
    WNode N = wload(W, 0);
    for (;;) {
        unsigned nh, th, imask, nl;
        int cb, tb;
        wide_node_g<G, COUNT>(N, p, oct, best * PRUNE_SLACK, q, nh, th, cb, tb, imask, nl);
        if (COUNT) {
            c.chi++;
            c.chl += nl;
            c.nb += 10;
            c.ws += first_active_lane();
        }
        const int next = wide_next(nh, cb, imask, oct, sp, stk);
        N = wload(W, next >= 0 ? next : 0);  // unconditional (rt_kernels.hpp closest_wide)
        if (th) {  // uniform in the group
            float lb = best;
            int lhp = hp, lnd = nd;
            bool ltie = tie;
            while (th) {
                const unsigned mine = deal<G>(th, q);
                if (mine) {
                    const int i = tb + __builtin_ctz(mine);
                    int k;
                    const float tt = hit_triangle(o, d, W.tris + 3 * i, k);
                    if (COUNT) c.cht++;
                    if (tt < lb) {
                        lb = tt;
                        lnd = k;
                        lhp = i;
                        ltie = false;
                    } else if (tt == lb && tt != FMAX) {
                        ltie = true;
                    }
                }
            }
            // merge: min t; tie if a lane at the min saw one or the lanes at the min disagree on the triangle
            const float m = g_minf<G>(lb);
            const bool at = lb == m;
            const int hlo = g_mini<G>(at ? lhp : 0x7FFFFFFF), hhi = g_maxi<G>(at ? lhp : (int)0x80000000);
            tie = g_or<G>(at && ltie ? 1u : 0u) != 0u || hlo != hhi;
            nd = (int)g_or<G>(at && lhp == hlo ? (unsigned)lnd : 0u);
            best = m;
            hp = hlo;
        }
        if (next < 0) {
            if (next == -2) CTR_INC(c, err, C_ERR);
            break;
        }
    }
}

template <int G, bool COUNT>
__device__ __forceinline__ bool visible_wide_g(const DWide& W, v3 o, v3 d, float ld2, int* __restrict__ stk, Ctr& c,
                                               unsigned q) {
    const RayPre p = ray_pre(o, d);
    const unsigned oct = (p.ix < 0.0f ? 1u : 0u) | (p.iy < 0.0f ? 2u : 0u) | (p.iz < 0.0f ? 4u : 0u);
    float best = FMAX;
    const float reach = shadow_reach(o, ld2);
    int sp = 0;
    WNode N = wload(W, 0);
    for (;;) {
        unsigned nh, th, imask, nl;
        int cb, tb;
        wide_node_g<G, COUNT>(N, p, oct, fminf(best * PRUNE_SLACK, reach), q, nh, th, cb, tb, imask, nl);
        if (COUNT) {
            c.shi++;
            c.shl += nl;
            c.nb += 10;
            c.ws += first_active_lane();
        }
        const int next = wide_next(nh, cb, imask, oct, sp, stk);
        N = wload(W, next >= 0 ? next : 0);  // unconditional (rt_kernels.hpp closest_wide)
        if (th) {
            float lb = best;
            unsigned occ = 0;
            while (th) {
                const unsigned mine = deal<G>(th, q);
                if (mine && !occ) {
                    const int i = tb + __builtin_ctz(mine);
                    int k;
                    const float tt = hit_triangle(o, d, W.tris + 3 * i, k);
                    if (COUNT) c.sht++;
                    if (tt < lb) {
                        lb = tt;
                        const v3 ip = add(o, mul(d, lb));
                        const v3 oi = sub(o, ip);
                        if (ld2 > dot(oi, oi)) occ = 1;
                    }
                }
            }
            if (g_or<G>(occ)) return false;
            best = g_minf<G>(lb);
        }
        if (next < 0) {
            if (next == -2) CTR_INC(c, err, C_ERR);
            break;
        }
    }
    return true;
}

template <int G, bool COUNT>
__device__ __forceinline__ int closest_g(const DScene& s, v3 o, v3 d, float& best, int& nd, int* __restrict__ stk,
                                         Ctr& c, unsigned q, bool unit) {
    int hp = -1;
    bool tie = false;
    best = FMAX;
    nd = 0;
    if (!degenerate(d) || degenerate_ok(s, o, d)) {  // (as closest)
        const DWide& W = wide_for(s, unit);
        closest_wide_g<G, COUNT>(W, o, d, best, hp, nd, tie, stk, c, q);
        if (!tie) return hp >= 0 ? W.tri_orig[hp] : -1;
        CTR_INC(c, fb, C_FALLBACK);  // strict re-walk, redundantly in every lane of the group
        if (TIE_BOUNDED) {  // (bounded just past the tie: closest)
            const float tb = tie_bound(o, best), cut = best - (tb - best);
            hp = -1;
            nd = 0;
            best = tb;
            closest_walk<true, COUNT, true, TIE_CUT>(s.ref, o, d, best, hp, nd, tie, stk, c, cut);
            if (hp >= 0) return s.ref.tri_orig[hp];
        }
        hp = -1;
        best = FMAX;
        nd = 0;
    } else {
        CTR_INC(c, fb, C_FALLBACK);
    }
    closest_walk<true, COUNT, true>(s.ref, o, d, best, hp, nd, tie, stk, c);
    return hp >= 0 ? s.ref.tri_orig[hp] : -1;
}

template <int G, bool COUNT>
__device__ __forceinline__ bool visible_g(const DScene& s, v3 o, v3 d, float ld2, int* __restrict__ stk, Ctr& c,
                                          unsigned q) {
    if (!degenerate(d) || degenerate_ok(s, o, d))  // |d| = 1
        return visible_wide_g<G, COUNT>(wide_for(s, true), o, d, ld2, stk, c, q);
    CTR_INC(c, fb, C_FALLBACK);
    return visible_walk<true, COUNT, true>(s.ref, o, d, ld2, stk, c);
}

// Counters of a group: every lane counts the ray work redundantly except triangle tests (each lane
// counts its own) and wave steps (the wave's first active lane, q == 0): lanes q != 0 report only those.
template <bool COUNT, int G>
__device__ __forceinline__ void flush_g(Ctr c, unsigned long long* g, unsigned q) {
    if (q != 0) {
        const unsigned cht = c.cht, sht = c.sht, ws = c.ws;
        c = Ctr{};
        c.cht = cht;
        c.sht = sht;
        c.ws = ws;
    }
    flush<COUNT>(c, g);
}

// The single-frame feedback (rt_feedback.hpp) ranks 8x8 tiles by the time their last render took; a tile rendered by
// k_coop is priced as k_persist would have taken for it, so that hot and cold tiles compare: k_coop spends about twice
// k_persist's wave time per ray, and its tile holds 64 / G of the 8x8 tile's 64 rays, so a group tile's time t is
// ~2 T / G of the 8x8 tile's T -- priced at t G / 2 (the longest of the tile's G group tiles). A biased price makes the
// hot set sticky: priced 2x (G = 2 at a fixed 2x), last frame's hot tiles stayed over the cut and no other tile could
// reach it, so a moving camera's hot set froze where it had been (a car_boxed walkthrough ~20 % slower than persist).
template <int G> constexpr unsigned fb_coop_scale() { return G / 2; }

// Pixel tile of one wave: 64 / G pixels.
template <int G> struct GTile;
template <> struct GTile<2> { static constexpr int TW = 8, TH = 4; };
template <> struct GTile<4> { static constexpr int TW = 4, TH = 4; };
template <> struct GTile<8> { static constexpr int TW = 4, TH = 2; };

// Persistent waves pulling TW x TH pixel tiles (k_persist's dealing: one atomic per wave per tile,
// optional centre-out order); lane = (pixel lane / G, group member lane % G).
template <int MAXB, bool COUNT, int G, int OCC = 3, bool TRACE = false, bool BATCH = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, BLOCK), amdgpu_waves_per_eu(OCC))) void k_coop(KArgs A) {
    __shared__ int lds[STACK * BLOCK];
    int* stk = lds + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const unsigned q = (unsigned)lane % G;
    const int pi = lane / G;
    constexpr int TW = GTile<G>::TW;
    Ctr c = {};
    // frame batches: as k_persist; a list built on the device (the single-frame feedback) has its length there
    const unsigned items =
        (unsigned)(A.n_tiles_dev ? __builtin_amdgcn_readfirstlane(*A.n_tiles_dev) : A.n_tiles) * (unsigned)A.n_frames;
    for (;;) {
        unsigned t = 0;
        if (lane == 0) t = atomicAdd(A.work, 1u);
        t = __builtin_amdgcn_readfirstlane(__shfl(t, 0, 64));
        if (t >= items) break;
        const int frame = (int)(t % (unsigned)A.n_frames);
        unsigned tile = t / (unsigned)A.n_frames;
        if (A.tile_order) tile = (unsigned)A.tile_order[tile];
        const int tx = (int)(tile % (unsigned)A.tiles_x), ty = (int)(tile / (unsigned)A.tiles_x);
        const int x = tx * TW + pi % TW, k = ty * GTile<G>::TH + pi / TW;
        unsigned long long t0 = 0;
        const unsigned fb0 = c.fb, ws0 = c.ws, nd0 = c.chi + c.shi;
        if (TRACE || A.tile_cost) t0 = __builtin_amdgcn_s_memrealtime();
        if (x < A.W && k < A.n_rows) render_pixel<MAXB, false, COUNT, true, G>(A, cam_of<BATCH>(A, frame), frame, x, k, stk, c, q);
        if (A.tile_cost && lane == 0)  // the feedback's cost of the 8x8 tile this tile lies in (rt_feedback.hpp)
            atomicMax(A.tile_cost + (ty * GTile<G>::TH / 8) * A.tiles_x8 + tx * TW / 8,
                      (unsigned)(__builtin_amdgcn_s_memrealtime() - t0) * fb_coop_scale<G>());
        if (TRACE) {  // as k_persist's: {begin, end, wave | fallbacks << 32, wave steps | ray node visits << 32}
            const unsigned fb = wave_sum(q == 0 ? c.fb - fb0 : 0u), ws = wave_sum(c.ws - ws0),
                           nv = wave_sum(q == 0 ? c.chi + c.shi - nd0 : 0u);
            if (lane == 0) {
                A.tile_trace[4 * tile] = t0;
                A.tile_trace[4 * tile + 1] = __builtin_amdgcn_s_memrealtime();
                A.tile_trace[4 * tile + 2] = (blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6)) | ((unsigned long long)fb << 32);
                A.tile_trace[4 * tile + 3] = ws | ((unsigned long long)nv << 32);
            }
        }
    }
    flush_g<COUNT, G>(c, A.counters, q);
}

}  // namespace rtd
