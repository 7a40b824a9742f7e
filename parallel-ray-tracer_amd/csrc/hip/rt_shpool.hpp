// rt_shpool.hpp — k_persist's per-wave shadow pool (RT_VARIANT_SHPOOL).
//
// k_persist walks a bounce level's shadow rays light by light (path_step, raytracer.c:149-160): every light's
// walk lasts as long as its slowest lane, and a lane whose path has ended — or whose pixel is a miss, or whose
// light failed the back-face test — idles through all of them. Here the wave's shadow rays of one level are ONE
// pool of (pixel lane, light) pairs that every lane of the wave walks: a lane whose walk ends takes the next
// unassigned pair (any pixel's, any light's), so a level costs about (its shadow work / 64 lanes) plus one
// walk's tail instead of one tail per light, and the lanes of ended paths work too. No workgroup barrier: the
// pool, its cursor and the hand-over are wave-level (ballots, scalar registers, lane reads).
//
// The results are bit-identical: a pair's ray is the reference's (light_v, raytracer.c:62-99: o = the owner's hit
// point, d = the normalised direction to the light, ld2 from the same expressions), its visibility does not
// depend on which lane walks it or when, and the owner folds the lights' Lambert/Blinn terms in the reference's
// order once all of its level's rays have returned (trace_path_shp).
#pragma once
#include <type_traits>

#include "rt_kernels.hpp"

namespace rtd {

// a wave-uniform 64-bit value (a ballot, the pool's cursor) pinned to scalar registers: without it the compiler
// keeps the cursor in vector registers and runs its scalar loop lane-masked (measured: +34 % per step)
__device__ __forceinline__ unsigned long long uni64(unsigned long long v) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// position of the k-th (0-based) set bit of m (k < popcount(m)): a binary search over popcounts, on scalar registers
// for a wave-uniform (m, k), per lane otherwise
__device__ __forceinline__ int kth_bit(unsigned long long m, unsigned k) {
    int pos = 0;
    unsigned c = (unsigned)__builtin_popcount((unsigned)m);
    if (k >= c) {
        k -= c;
        m >>= 32;
        pos = 32;
    }
    unsigned w = (unsigned)m;
#pragma unroll
    for (int b = 16; b >= 2; b >>= 1) {
        c = (unsigned)__builtin_popcount(w & ((1u << b) - 1u));
        if (k >= c) {
            k -= c;
            w >>= b;
            pos += b;
        }
    }
    return pos + (k >= (w & 1u) ? 1 : 0);
}
// m without its lowest n set bits (n <= popcount(m))
__device__ __forceinline__ unsigned long long drop_low(unsigned long long m, unsigned n) {
    if (n == 0) return m;
    const int p = kth_bit(m, n - 1u);
    return p >= 63 ? 0ull : m & ~((2ull << p) - 1ull);
}

// Wave-uniform ray counts of the shadow-pool kernels. Their path loop runs in step over the wave (every lane takes
// part, lanes outside the frame as walkers only), so each count is a popcount of a ballot and lives in a scalar
// register, instead of one vector register per counter and lane held across every walk (the register budget of the
// 4-wave kernel is 128 VGPRs; what does not fit spills).
struct UCtr {
    unsigned prim, refl, shad, skip, hits, pix;
};
__device__ __forceinline__ unsigned popc_wave(bool v) { return (unsigned)__builtin_popcountll(uni64(__ballot(v))); }
__device__ __forceinline__ void flush_u(const UCtr& u, unsigned long long* g) {
    if ((threadIdx.x & 63u) != 0u) return;
    const unsigned v[6] = {u.prim, u.refl, u.shad, u.skip, u.hits, u.pix};
    const int at[6] = {C_PRIM, C_REFL, C_SHAD, C_SKIP, C_HITS, C_PIX};
#pragma unroll
    for (int i = 0; i < 6; i++)
        if (v[i]) atomicAdd(g + at[i], (unsigned long long)v[i]);
}

// Packed triangle tests (TQ, the all-levels pool): a wave step's hit leaf slots hold few triangles per lane and the
// per-lane loop over them runs as long as the lane with the most (dragon: 2.7 loop rounds per pool step at 10 % of the
// lanes, PRT_DIAG_TRI). When some lane holds 3 or more, the step's (owner lane, triangle) pairs are written to the
// wave's LDS queue (TQ_*, rt_kernels.hpp) instead and tested 64 at a time, each by the lane that reads it, with the
// owner's ray fetched by `ds_bpermute`; occlusion (the reference's per-triangle test, bvh.c:283-290) and the nearest
// hit (for the walk's box pruning) go back to the owner's LDS slots.

// The shadow rays of LV bounce levels of the wave's paths, walked as ONE wave-level pool.
// okm(l): bit j = this lane's path hit a surface at level l and light j passed the back-face test (dot(L - ip, n)
// >= 0, the reference's early-out, raytracer.c:66-67; failing lights are not walked). lvl: the wave's path-buffer
// slots of those levels (LDS, [level][lane]); the owner lane p has stored its level-l hit point in lvl[64 l + p].xyz
// and 0 in its .w, and the walkers set bit j of that .w (as an unsigned) when light j is visible from it along the
// reference's shadow ray. regroup: idle lanes that trigger a refill (all lanes idle always do). Called by every lane
// of the wave.
template <bool COUNT, int LV, bool TQ = false, class OKM>
__device__ __forceinline__ void shadow_pool(const DScene& s, OKM okm, float4* lvl, int* __restrict__ stk,
                                            int* __restrict__ sstk, int wcap, int regroup, Ctr& c, UCtr& u,
                                            int* tq = nullptr) {
    const unsigned lane = threadIdx.x & 63u;
    // (TQ: the queue's result slots are clear, tq_clear)
    const unsigned long long all = uni64(__ballot(1));
    const int nl = s.n_lights;
    const DWide& W = wide_for(s, true);  // |d| = 1: the unit-direction view
    const gnodes nbase = walk_base(W.nodes);
    // the cursor (wave-uniform): level cl, light cj, and the owner lanes whose ray toward it is still unassigned
    int cl = 0, cj = -1;
    unsigned long long cm = 0;
    auto advance = [&]() {  // the next (level, light) with owners past the back-face test
        while (cm == 0 && (cl + 1 < LV || cj + 1 < nl)) {
            if (cj + 1 < nl) {
                cj = uni(cj + 1);
            } else {
                cj = 0;
                cl = uni(cl + 1);
            }
            cm = uni64(__ballot((okm(cl) >> cj) & 1u));
            u.shad += (unsigned)__builtin_popcountll(cm);
        }
    };
    // this lane's ray (owner lane | level << 6 | light << 9) and its walk state (visible_wide's)
    bool busy = false;
    int wo = 0;
    v3 o = mk(0.0f, 0.0f, 0.0f), d = o;
    RayPre p = {};
    unsigned oct = 0;
    float ld2 = 0.0f, reach = 0.0f, best = FMAX;
    int sp = 0;
    TopC tc;
    WNode N = {};
    for (;;) {
        advance();
        const unsigned long long idle = uni64(__ballot(!busy));
        if (idle == all && cm == 0) break;
        if (cm != 0) {  // refill every idle lane while there is work
            // every idle lane at once: the k-th requester takes the k-th unassigned owner of light cj, the rest
            // move on to the next light (one round per light, no per-ray scalar loop)
            unsigned long long req = idle;
            bool got = false;
            while (req != 0ull && cm != 0ull) {
                const unsigned nreq = (unsigned)__builtin_popcountll(req), nav = (unsigned)__builtin_popcountll(cm);
                const unsigned k = __builtin_amdgcn_mbcnt_hi((unsigned)(req >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((unsigned)req, 0u));
                if (((req >> lane) & 1ull) && k < nav) {
                    wo = kth_bit(cm, k) | (cl << 6) | (cj << 9);
                    got = true;
                }
                if (nreq >= nav) {
                    req = uni64(drop_low(req, nav));
                    cm = 0ull;
                    advance();
                } else {
                    cm = uni64(drop_low(cm, nreq));
                    req = 0ull;
                }
            }
            if (got) {
                // the reference's shadow ray, light_v (raytracer.c:62-99) as path_step forms it, from the owner's hit
                // point (its path-buffer slot)
                const v3 ipo = xyz(lvl[wo & 511]);  // (64 level + owner)
                const v3 Lp = xyz(s.lights[2 * (wo >> 9)]);
                v3 l = sub(Lp, ipo);
                const float mg = mag(l);
                l = dvs(l, mg);
                const v3 tmp = sub(ipo, Lp);
                ld2 = dot(tmp, tmp);
                o = ipo;
                d = l;
                if (degenerate(d) && !degenerate_ok(s, o, d)) {  // a 0 / 0 in the reference's slabs: walked strictly
                    CTR_INC(c, fb, C_FALLBACK);
                    if (visible_walk<true, COUNT, true>(s.ref, o, d, ld2, sstk ? sstk : stk, c))
                        atomicOr(reinterpret_cast<unsigned*>(lvl + (wo & 511)) + 3, 1u << ((wo >> 9) & 31));
                } else {
                    reach = shadow_reach(o, ld2);
                    p = ray_pre_shadow(o, d, reach);
                    oct = (p.ix < 0.0f ? 1u : 0u) | (p.iy < 0.0f ? 2u : 0u) | (p.iz < 0.0f ? 4u : 0u);
                    best = FMAX;
                    sp = 0;
                    N = wload_at(nbase, 0, c.top[1]);
                    busy = true;
                }
            }
        }
        // walk until the wave is idle, or enough of it to refill while work is left: visible_wide's loop, one
        // ballot per step
        const bool more = cm != 0 || cj + 1 < nl || cl + 1 < LV;
        for (;;) {
            unsigned th = 0u;
            int tb = 0, next = -1;
            if (busy) {  // one step of visible_wide
                unsigned nh, imask, nlf;
                int cb;
                pin_node(N);
                wide_node<COUNT, LATE_TRIS, SHADOW_CLAMP ? 1 : 0>(N, p, oct, fminf(best * PRUNE_SLACK, reach), nh, th, cb, tb,
                                                          imask, nlf, SHADOW_ORDER_XOR);
                const unsigned m0 = __float_as_uint(N.f1.z), m1 = __float_as_uint(N.f1.w);
                next = wide_step_next<true>(nh, cb, imask, oct ^ SHADOW_ORDER_XOR, sp, tc, stk, wcap);
                N = wload_at(nbase, next >= 0 ? next : 0, c.top[1]);  // unconditional (closest_wide)
                top_reload<true>(sp, tc, stk, wcap);
                if constexpr (LATE_TRIS) th = leaf_tris<COUNT>(th, m0, m1, nlf);
                if (COUNT) {
                    c.shi++;
                    c.shl += nlf;
                    c.nb += 10;
                    count_step(c, true);
                }
            }
            bool occ = false, seq = true;
            if constexpr (TQ) {
                const unsigned nt = (unsigned)__builtin_popcount(th);
                if (uni64(__ballot(nt >= TQ_MIN)) != 0ull) {
                    unsigned* cnt = reinterpret_cast<unsigned*>(tq + TQ_CNT);
                    unsigned pos = 0u;
                    if (nt) pos = atomicAdd(cnt, nt);
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    const unsigned T = (unsigned)uni((int)atomicAdd(cnt, 0u));
                    if (T <= (unsigned)TQ_CAP) {
                        seq = false;
                        for (unsigned m = th; m; m &= m - 1u) tq[pos++] = (int)((lane << 26) | (unsigned)(tb + __builtin_ctz(m)));
                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                        for (unsigned base = 0u; base < T; base += 64u) {
                            const unsigned j = base + lane;
                            const unsigned job = j < T ? (unsigned)tq[j] : lane << 26;
                            const int ow = (int)(job >> 26);
                            const v3 oo = mk(__shfl(o.x, ow, 64), __shfl(o.y, ow, 64), __shfl(o.z, ow, 64));
                            const v3 dd = mk(__shfl(d.x, ow, 64), __shfl(d.y, ow, 64), __shfl(d.z, ow, 64));
                            const float l2 = __shfl(ld2, ow, 64);
                            if (j < T) {
                                PRT_TRI_ITER(c, q2);
                                int k;
                                const float tt = hit_triangle<SHADOW_RCP>(oo, dd, W.tris + 3 * (int)(job & 0x3FFFFFFu), k);
                                if (COUNT) c.sht++;
                                if (tt < FMAX) {
                                    const v3 q = add(oo, mul(dd, tt));
                                    const v3 oi = sub(oo, q);
                                    if (l2 > dot(oi, oi)) tq[TQ_OCC + ow] = 1;
                                    atomicMax(reinterpret_cast<unsigned*>(tq + TQ_T + ow), ~__float_as_uint(tt));
                                }
                            }
                        }
                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                        if (nt) {
                            occ = tq[TQ_OCC + lane] != 0;
                            const unsigned tc = (unsigned)tq[TQ_T + lane];
                            if (tc) best = fminf(best, __uint_as_float(~tc));
                            tq[TQ_OCC + lane] = 0;
                            tq[TQ_T + lane] = 0;
                        }
                    }
                    if (lane == 0u) *cnt = 0u;
                }
            }
            if (busy) {
                while (seq && th) {
                    PRT_TRI_ITER(c, q2);
                    const int i = tb + __builtin_ctz(th);
                    th &= th - 1u;
                    int k;
                    const float tt = hit_triangle<SHADOW_RCP>(o, d, W.tris + 3 * i, k);
                    if (COUNT) c.sht++;
                    if (tt < best) {
                        best = tt;
                        const v3 q = add(o, mul(d, best));
                        const v3 oi = sub(o, q);
                        if (ld2 > dot(oi, oi)) {
                            occ = true;
                            break;
                        }
                    }
                }
                if (occ || next < 0) {
                    if (!occ && next == -2) CTR_INC(c, err, C_ERR);
                    if (!occ)  // the owner's visibility bit
                        atomicOr(reinterpret_cast<unsigned*>(lvl + (wo & 511)) + 3, 1u << ((wo >> 9) & 31));
                    busy = false;
                }
            }
            const unsigned long long id2 = uni64(__ballot(!busy));
            if (id2 == all || (more && __builtin_popcountll(id2) >= regroup)) break;
        }
    }
    if constexpr (TQ) tq_clear(tq);  // (the pool's jobs 64..127 overwrote the closest walk's flag words)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// trace_path (rt_kernels.hpp) with each level's shadow rays walked by shadow_pool: the path loop runs in step over
// the wave (a lane whose path has ended, or that holds no pixel, stays in it as a shadow worker) and a level's
// colour is formed after the pool with path_step's expressions in the reference's order. Path levels in the LDS
// path buffer (PB = 2): a level's slot holds the hit point and the visibility word while the pool runs, and the
// level's colour and material afterwards. Across the pool a lane keeps only its direction, the hit triangle and the
// lights' back-face mask; the hit point comes back from the slot, the normal and material from the shading record.
// hpix >= 0: the pixel's output index, for hit / t (level 0) and bounce_hit.
template <int MAXB, bool COUNT>
__device__ __forceinline__ v3 trace_path_shp(const KArgs& A, bool alive, v3 o, v3 d, int* __restrict__ stk, Ctr& c,
                                             UCtr& u, int hpix, int* __restrict__ sstk, int wcap) {
    extern __shared__ int lds_dyn[];
    float4* pb0 = (float4*)(lds_dyn + wstack_words(wcap, true) * BLOCK);
    float4* pb = pb0 + (size_t)((threadIdx.x >> 6) * MAXB) * 64 + (threadIdx.x & 63);
    float4* pbw = pb - (threadIdx.x & 63);  // the wave's slots of level 0
    // the wave's packed-triangle queue (TQ_*) after the path buffer, clear
    int* tq = (int*)(pb0 + (size_t)BLOCK * MAXB) + (threadIdx.x >> 6) * TQ_WORDS;
    tq_clear(tq);
    const DScene& s = A.s;
    const v3 amb = mk(s.amb_x, s.amb_y, s.amb_z);
    int L = 0;
    bool tail = false;
    for (int it = 0; it < A.bounces; ++it) {
        const unsigned na = popc_wave(alive);
        if (na == 0) break;
        if (COUNT) c.lvl = (unsigned)it;
        if (it == 0) u.prim += na;
        else u.refl += na;
        int hit = -1;  // the hit triangle (original index) | nd << 31 ... as two fields below
        bool nd_side = false;
        unsigned okm = 0;
        if (alive) {  // raytracer.c:101-147 as path_step
            float best;
            int nd;
            const int orig = closest<false, COUNT, true, false, true, true>(s, o, d, best, nd, stk, c, sstk, wcap, it > 0, tq);
            if (hpix >= 0) {
                const int h = opaque(hpix);  // (the outputs' addresses formed here, not hoisted and held: OPAQUE_OUT)
                if (it == 0) {
                    if (A.hit) A.hit[h] = orig;
                    if (A.t) A.t[h] = best;
                }
                if (A.bounce_hit) A.bounce_hit[(size_t)h * A.bounces + it] = orig;
            }
            if (orig < 0) {  // raytracer.c:132-135
                pb[it * 64] = make_float4(0.0f + amb.x, 0.0f + amb.y, 0.0f + amb.z, __int_as_float(0));
                L = it + 1;
                tail = false;
                alive = false;
            } else {
                hit = orig;
                nd_side = nd != 0;
                const v3 ip = add(o, mul(d, best));
                const float4 sh = s.shade[2 * orig + (nd ? 1 : 0)];
                const v3 n = xyz(sh);
                for (int j = 0; j < s.n_lights; ++j) {  // light_v's back-face test (raytracer.c:66-67)
                    const v3 tmp2 = sub(xyz(s.lights[2 * j]), ip);
                    okm |= dot(tmp2, n) < 0 ? 0u : (1u << j);
                }
                pb[it * 64] = make_float4(ip.x, ip.y, ip.z, __uint_as_float(0u));
            }
        }
        const unsigned nh = popc_wave(hit >= 0);
        u.hits += nh;
        if (nh) {
            u.skip += nh * (unsigned)s.n_lights;  // less the rays walked (shadow_pool counts those in u.shad)
            const unsigned sh0 = u.shad;
            shadow_pool<COUNT, 1, true>(s, [&](int) { return okm; }, pbw + it * 64, stk, sstk, wcap, A.regroup, c, u,
                                        tq);
            u.skip -= u.shad - sh0;
        }
        if (hit >= 0) {  // raytracer.c:144-172 as path_step, the lights' visibility from the pool
            const float4 e = pb[it * 64];
            const v3 ip = xyz(e);
            const unsigned vis = __float_as_uint(e.w) & okm;
            const float4 sh0 = s.shade[2 * hit], sh1 = s.shade[2 * hit + 1];
            const int m = __float_as_int(sh0.w);
            const v3 n = nd_side ? xyz(sh1) : xyz(sh0);
            const v3 kd0 = xyz(s.mats[3 * m + 1]);
            v3 col = mk(0.0f + kd0.x * amb.x, 0.0f + kd0.y * amb.y, 0.0f + kd0.z * amb.z);
            const v3 v = mul(d, -1.0f);
            for (int j = 0; j < s.n_lights; ++j) {
                const v3 Lp = xyz(s.lights[2 * j]);
                v3 l = sub(Lp, ip);
                float mg = mag(l);
                l = dvs(l, mg);
                mg *= mg;
                const int V = (int)((vis >> j) & 1u);  // 0 behind the surface (okm), else the shadow ray's answer
                const v3 kl = xyz(s.lights[2 * j + 1]);
                const v3 ks = xyz(s.mats[3 * m]), kd = xyz(s.mats[3 * m + 1]);
                const float ndl = dot(n, l);
                const v3 h = normalize(add(l, v));
                const float coeff = fmaxf(0.0f, dot(n, h));
                const v3 cr = mk(kd.x * fmaxf(0.0f, ndl) + ks.x * coeff, kd.y * fmaxf(0.0f, ndl) + ks.y * coeff,
                                 kd.z * fmaxf(0.0f, ndl) + ks.z * coeff);
                const float fV = (float)V;
                col.x = col.x + fV * kl.x * cr.x / mg;
                col.y = col.y + fV * kl.y * cr.y / mg;
                col.z = col.z + fV * kl.z * cr.z / mg;
            }
            const v3 dd = mul(v, -1.0f);
            const v3 ns = mul(n, 2.0f * __builtin_fabsf(dot(dd, n)));
            const v3 r = normalize(add(dd, ns));
            pb[it * 64] = make_float4(col.x, col.y, col.z, __int_as_float(m));
            const v3 kr = xyz(s.mats[3 * m + 2]);
            if (!(mag(kr) > 0.0f)) {  // raytracer.c:168
                L = it + 1;
                tail = false;
                alive = false;
            } else if (it + 1 == A.bounces) {  // raytrace(.., BOUNCES) returns {0,0,0}: col += kr * 0
                L = it + 1;
                tail = true;
                alive = false;
            } else {
                o = ip;
                d = r;
            }
        }
    }
    return fold_pb<MAXB>(s, pb, L, tail);
}

// trace_path_shp with ONE pool for every level's shadow rays (RT_VARIANT_SHDEFER): a path's closest hits are walked
// level by level first -- the reflection ray of level i needs level i's hit point and normal, never its shadow rays --
// and then the shadow rays of all its levels, every pixel's and every light's, form one pool, so a tile pays one
// pool tail instead of one per level and the few shadow rays of the deep levels fill the lanes together with the
// others. The levels' colours follow in the reference's order (path_step's expressions, level 0 first, each with its
// own direction: the primary one, then each level's reflection, recomputed), then the deepest-first fold. The path
// buffer holds a level's hit point and visibility word (then its colour and material), and a second [level][lane]
// array its hit triangle (orig | nd << 30, -1: a miss).
template <int MAXB, bool COUNT>
__device__ __forceinline__ v3 trace_path_dfr(const KArgs& A, bool alive, v3 o, v3 d, int* __restrict__ stk, Ctr& c,
                                             UCtr& u, int hpix, int* __restrict__ sstk, int wcap) {
    extern __shared__ int lds_dyn[];
    float4* pb0 = (float4*)(lds_dyn + wstack_words(wcap, true) * BLOCK);
    const size_t wl = (size_t)((threadIdx.x >> 6) * MAXB) * 64 + (threadIdx.x & 63);
    float4* pb = pb0 + wl;
    float4* pbw = pb - (threadIdx.x & 63);  // the wave's slots of level 0
    int* hid = (int*)(pb0 + (size_t)BLOCK * MAXB) + wl;
    // the wave's packed-triangle queue (TQ_*): the closest walks' result slots empty, its counter 0
    int* tq = (int*)(pb0 + (size_t)BLOCK * MAXB) + BLOCK * MAXB + (threadIdx.x >> 6) * TQ_WORDS;
    tq_clear(tq);
    const DScene& s = A.s;
    const v3 amb = mk(s.amb_x, s.amb_y, s.amb_z);
    const v3 d0 = d;
    // the levels' back-face masks, 8 bits per level (1..8 lights: the rule's shd_ok) in one or two registers
    using OkT = typename std::conditional<MAXB <= 4, unsigned, unsigned long long>::type;
    OkT okm = 0;
    int L = 0;
    bool tail = false;
    unsigned nhits = 0;
    for (int it = 0; it < A.bounces; ++it) {  // the closest hits of every level (raytracer.c:101-147, 163-172)
        const unsigned na = popc_wave(alive);
        if (na == 0) break;
        if (COUNT) c.lvl = (unsigned)it;
        if (it == 0) u.prim += na;
        else u.refl += na;
        bool hitl = false;
        if (alive) {
            float best;
            int nd;
            const int orig =
                closest<false, COUNT, true, false, true, true>(s, o, d, best, nd, stk, c, sstk, wcap, it > 0, tq);
            if (hpix >= 0) {
                const int h = opaque(hpix);  // (the outputs' addresses formed here, not hoisted and held: OPAQUE_OUT)
                if (it == 0) {
                    if (A.hit) A.hit[h] = orig;
                    if (A.t) A.t[h] = best;
                }
                if (A.bounce_hit) A.bounce_hit[(size_t)h * A.bounces + it] = orig;
            }
            if (orig < 0) {  // raytracer.c:132-135 (the colour is written by the shading loop below)
                hid[it * 64] = -1;
                L = it + 1;
                tail = false;
                alive = false;
            } else {
                hitl = true;
                const v3 ip = add(o, mul(d, best));
                const float4 sh0 = s.shade[2 * orig], sh1 = s.shade[2 * orig + 1];
                const int m = __float_as_int(sh0.w);
                const v3 n = nd ? xyz(sh1) : xyz(sh0);
                unsigned ok = 0;
                for (int j = 0; j < s.n_lights; ++j) {  // light_v's back-face test (raytracer.c:66-67)
                    const v3 tmp2 = sub(xyz(s.lights[2 * j]), ip);
                    ok |= dot(tmp2, n) < 0 ? 0u : (1u << j);
                }
                okm |= (OkT)ok << (8 * it);
                pb[it * 64] = make_float4(ip.x, ip.y, ip.z, __uint_as_float(0u));
                hid[it * 64] = orig | (nd ? (1 << 30) : 0);
                const v3 ns = mul(n, 2.0f * __builtin_fabsf(dot(d, n)));  // (dd = -(-d) = d exactly)
                const v3 r = normalize(add(d, ns));
                const v3 kr = xyz(s.mats[3 * m + 2]);
                if (!(mag(kr) > 0.0f)) {  // raytracer.c:168
                    L = it + 1;
                    tail = false;
                    alive = false;
                } else if (it + 1 == A.bounces) {  // raytrace(.., BOUNCES) returns {0,0,0}: col += kr * 0
                    L = it + 1;
                    tail = true;
                    alive = false;
                } else {
                    o = ip;
                    d = r;
                }
            }
        }
        const unsigned nh = popc_wave(hitl);
        u.hits += nh;
        nhits += nh;
    }
    if (nhits) {  // every level's shadow rays as one pool
        u.skip += nhits * (unsigned)s.n_lights;
        const unsigned sh0 = u.shad;
        shadow_pool<COUNT, MAXB, true>(s, [&](int l) { return (unsigned)(okm >> (8 * l)) & 0xFFu; }, pbw, stk, sstk, wcap,
                                       A.regroup, c, u, tq);
        u.skip -= u.shad - sh0;
    }
    v3 dl = d0;  // level i's direction: the primary one, then each level's reflection
    for (int it = 0; it < L; ++it) {  // the levels' colours (raytracer.c:144-160 as path_step), in order
        const int h = hid[it * 64];
        if (h < 0) {  // a miss (the path's last level): the background
            pb[it * 64] = make_float4(0.0f + amb.x, 0.0f + amb.y, 0.0f + amb.z, __int_as_float(0));
            break;
        }
        const float4 e = pb[it * 64];
        const v3 ip = xyz(e);
        const unsigned vis = __float_as_uint(e.w) & ((unsigned)(okm >> (8 * it)) & 0xFFu);
        const int orig = h & ((1 << 30) - 1);
        const float4 sh0 = s.shade[2 * orig], sh1 = s.shade[2 * orig + 1];
        const int m = __float_as_int(sh0.w);
        const v3 n = (h >> 30) ? xyz(sh1) : xyz(sh0);
        const v3 kd0 = xyz(s.mats[3 * m + 1]);
        v3 col = mk(0.0f + kd0.x * amb.x, 0.0f + kd0.y * amb.y, 0.0f + kd0.z * amb.z);
        const v3 v = mul(dl, -1.0f);
        for (int j = 0; j < s.n_lights; ++j) {
            const v3 Lp = xyz(s.lights[2 * j]);
            v3 l = sub(Lp, ip);
            float mg = mag(l);
            l = dvs(l, mg);
            mg *= mg;
            const int V = (int)((vis >> j) & 1u);
            const v3 kl = xyz(s.lights[2 * j + 1]);
            const v3 ks = xyz(s.mats[3 * m]), kd = xyz(s.mats[3 * m + 1]);
            const float ndl = dot(n, l);
            const v3 hv = normalize(add(l, v));
            const float coeff = fmaxf(0.0f, dot(n, hv));
            const v3 cr = mk(kd.x * fmaxf(0.0f, ndl) + ks.x * coeff, kd.y * fmaxf(0.0f, ndl) + ks.y * coeff,
                             kd.z * fmaxf(0.0f, ndl) + ks.z * coeff);
            const float fV = (float)V;
            col.x = col.x + fV * kl.x * cr.x / mg;
            col.y = col.y + fV * kl.y * cr.y / mg;
            col.z = col.z + fV * kl.z * cr.z / mg;
        }
        pb[it * 64] = make_float4(col.x, col.y, col.z, __int_as_float(m));
        const v3 dd = mul(v, -1.0f);
        dl = normalize(add(dd, mul(n, 2.0f * __builtin_fabsf(dot(dd, n)))));
    }
    return fold_pb<MAXB>(s, pb, L, tail);
}

// render_pixel (rt_kernels.hpp) for the shadow-pool kernels: called by EVERY lane of the wave (valid = the lane
// holds a pixel of the frame), so that the path loop and the pool run in uniform control flow
template <int MAXB, bool COUNT, bool SPP1, int SHP>
__device__ __forceinline__ void render_pixel_shp(const KArgs& A, const Cam& C, int frame, int x, int k, bool valid,
                                                 int* __restrict__ stk, Ctr& c, UCtr& u, int* __restrict__ sstk,
                                                 int wcap) {
    auto trace = [&](v3 d, int hp) {
        if constexpr (SHP == 2) return trace_path_dfr<MAXB, COUNT>(A, valid, C.pos, d, stk, c, u, hp, sstk, wcap);
        else return trace_path_shp<MAXB, COUNT>(A, valid, C.pos, d, stk, c, u, hp, sstk, wcap);
    };
    const int y = image_row(A, k, frame);
    valid = valid && y < A.H;  // frame_shift: a rotated rank's compact rows past the image
    u.pix += popc_wave(valid);
    if (A.bounce_hit && valid) {
        const size_t o = (size_t)frame * A.frame_px + (size_t)k * A.W + x;
        for (int i = 0; i < A.bounces; i++) A.bounce_hit[o * (size_t)A.bounces + i] = -2;
    }
    if constexpr (SPP1) {  // (the host runs the SPP1 builds for spp = 1, the others for spp > 1 only)
        const int o = (int)((size_t)frame * A.frame_px + (size_t)k * A.W + x);  // (< 2^31: rt_render's output bound)
        const v3 col = clamp01(trace(primary_dir(C, (float)x, (float)y), valid ? o : -1));
        if (valid) store_px(A.rgb, A.bgra, (size_t)opaque(o), col);
    } else {  // stratified g x g sub-pixel grid, mean of clamped samples; hit / t from the first sample
        // The lane's A.lanebuf slot carries the running sum and the pixel (x, compact row k) from sample to sample, so
        // that no register stays live across a sample's path (spp_slot; the host guarantees W, n_rows <= 65535)
        const int g = A.spp_grid;
        *lane_slot<true>(A) = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float((unsigned)x | ((unsigned)k << 16)));
        v3 acc = mk(0.0f, 0.0f, 0.0f);
        for (int s = 0; s < g * g; ++s) {
            __asm__ volatile("" ::: "memory");  // (read the slot back: no value forwarded in registers across the path)
            float4* lb = lane_slot<true>(A);
            const float4 e = *lb;
            const unsigned px = __float_as_uint(e.w);
            const int xs = (int)(px & 0xFFFFu), ks = (int)(px >> 16), ys = image_row(A, ks, frame);
            const int sj = s / g, si = s - sj * g;
            const float fx = (float)xs + ((float)si + 0.5f) / (float)g;
            const float fy = (float)ys + ((float)sj + 0.5f) / (float)g;
            const int hp = s == 0 && valid ? (int)((size_t)frame * A.frame_px + (size_t)ks * A.W + xs) : -1;
            const v3 cs = clamp01(trace(primary_dir_sample(C, fx, fy), hp));
            __asm__ volatile("" ::: "memory");
            lb = lane_slot<true>(A);
            const float4 a = *lb;
            acc = add(mk(a.x, a.y, a.z), cs);
            *lb = make_float4(acc.x, acc.y, acc.z, a.w);
        }
        const float nn = (float)(g * g);
        __asm__ volatile("" ::: "memory");
        const unsigned px = __float_as_uint(lane_slot<true>(A)->w);  // (the pixel from the slot: nothing of it live across the loop)
        const size_t o = (size_t)frame * A.frame_px + (size_t)(px >> 16) * A.W + (px & 0xFFFFu);
        if (valid) store_px(A.rgb, A.bgra, o, mk(acc.x / nn, acc.y / nn, acc.z / nn));
    }
}

}  // namespace rtd
