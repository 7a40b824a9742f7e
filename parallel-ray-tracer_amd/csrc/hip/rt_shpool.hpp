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

// the pool's cursor past exhausted lights: the next light with owners past the back-face test (wave-uniform; one
// ballot per light, the skip / shadow counts per owner as path_step keeps them)
__device__ __forceinline__ void pool_advance(const DScene& s, bool has, v3 ip, v3 n, int nl, int& cj,
                                             unsigned long long& cm, Ctr& c) {
    while (cm == 0 && cj + 1 < nl) {
        cj = uni(cj + 1);
        const v3 tmp2 = sub(xyz(s.lights[2 * cj]), ip);
        const bool ok = has && !(dot(tmp2, n) < 0);
        if (has) {
            if (ok) c.shad++;
            else c.skip++;
        }
        cm = uni64(__ballot(ok));
    }
}

// The shadow rays of one bounce level of the calling lanes' paths, walked as a wave-level pool.
// has: this lane's path hit a surface at this level (hit point ip, normal n). Returns bit j = 1 iff light j is
// visible from ip along the reference's shadow ray; lights behind the surface (dot(L - ip, n) < 0, the
// reference's early-out, raytracer.c:66-67) are not walked and read 0. regroup: idle lanes that trigger a refill
// (all lanes idle always do). Must be called by every lane of the wave that runs the path loop (uniform flow).
template <bool COUNT>
__device__ __forceinline__ unsigned shadow_pool(const DScene& s, bool has, v3 ip, v3 n, int* __restrict__ stk,
                                                int* __restrict__ sstk, int wcap, int regroup, unsigned* visw,
                                                Ctr& c) {
    const unsigned lane = threadIdx.x & 63u;
    const unsigned long long all = uni64(__ballot(1));
    const int nl = s.n_lights;
    const DWide& W = wide_for(s, true);  // |d| = 1: the unit-direction view
    visw[lane] = 0u;  // the wave's 64 visibility words (LDS): bit j of word p = light j visible from lane p's hit
    // the cursor (wave-uniform): light cj, and the owner lanes whose ray toward cj is still unassigned
    int cj = -1;
    unsigned long long cm = 0;
#define PRT_POOL_ADVANCE() pool_advance(s, has, ip, n, nl, cj, cm, c)
    // this lane's ray (owner lane | light << 8) and its walk state (visible_wide's)
    bool busy = false;
    int wo = 0;
    v3 o = ip, d = ip;
    RayPre p = {};
    unsigned oct = 0;
    float ld2 = 0.0f, reach = 0.0f, best = FMAX;
    int sp = 0;
    WNode N = {};
    for (;;) {
        PRT_POOL_ADVANCE();
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
                    wo = kth_bit(cm, k) | (cj << 8);
                    got = true;
                }
                if (nreq >= nav) {
                    req = uni64(drop_low(req, nav));
                    cm = 0ull;
                    PRT_POOL_ADVANCE();
                } else {
                    cm = uni64(drop_low(cm, nreq));
                    req = 0ull;
                }
            }
            // the owner's hit point (every lane reads: a cross-lane read needs its source lane active)
            const int src = wo & 63;
            const float px = __shfl(ip.x, src, 64), py = __shfl(ip.y, src, 64), pz = __shfl(ip.z, src, 64);
            if (got) {
                // the reference's shadow ray, light_v (raytracer.c:62-99) as path_step forms it
                const v3 ipo = mk(px, py, pz);
                const v3 Lp = xyz(s.lights[2 * (wo >> 8)]);
                v3 l = sub(Lp, ipo);
                const float mg = mag(l);
                l = dvs(l, mg);
                const v3 tmp = sub(ipo, Lp);
                ld2 = dot(tmp, tmp);
                o = ipo;
                d = l;
                if (degenerate(d)) {  // zero direction component: the reference's NaN slabs, walked strictly
                    c.fb++;
                    if (visible_walk<true, COUNT, true>(s.ref, o, d, ld2, sstk ? sstk : stk, c))
                        atomicOr(visw + (wo & 63), 1u << ((wo >> 8) & 31));
                } else {
                    p = ray_pre(o, d);
                    oct = (p.ix < 0.0f ? 1u : 0u) | (p.iy < 0.0f ? 2u : 0u) | (p.iz < 0.0f ? 4u : 0u);
                    best = FMAX;
                    reach = shadow_reach(o, ld2);
                    sp = 0;
                    N = wload(W, 0);
                    busy = true;
                }
            }
        }
        // walk until the wave is idle, or enough of it to refill while work is left: visible_wide's loop, one
        // ballot per step
        const bool more = cm != 0 || cj + 1 < nl;
        for (;;) {
            if (busy) {  // one step of visible_wide
                unsigned nh, th, imask, nlf;
                int cb, tb;
                wide_node<COUNT>(N, p, oct, fminf(best * PRUNE_SLACK, reach), nh, th, cb, tb, imask, nlf, SHADOW_ORDER_XOR);
                if (COUNT) {
                    c.shi++;
                    c.shl += nlf;
                    c.nb += 10;
                    count_step(c, true);
                }
                const int next = wide_next(nh, cb, imask, oct ^ SHADOW_ORDER_XOR, sp, stk, wcap);
                N = wload(W, next >= 0 ? next : 0);  // unconditional (closest_wide)
                bool occ = false;
                while (th) {
                    const int i = tb + __builtin_ctz(th);
                    th &= th - 1u;
                    int k;
                    const float tt = hit_triangle(o, d, W.tris + 3 * i, k);
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
                    if (!occ && next == -2) c.err++;
                    if (!occ) atomicOr(visw + (wo & 63), 1u << ((wo >> 8) & 31));  // the owner's visibility bit
                    busy = false;
                }
            }
            const unsigned long long id2 = uni64(__ballot(!busy));
            if (id2 == all || (more && __builtin_popcountll(id2) >= regroup)) break;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    return visw[lane];
}
#undef PRT_POOL_ADVANCE

// trace_path (rt_kernels.hpp) with each level's shadow rays walked by shadow_pool: the path loop runs in step over
// the wave (a lane whose path has ended stays in it as a shadow worker) and a level's colour is formed after the
// pool with path_step's expressions in the reference's order. Path levels in the path buffer (PB kernels).
template <int MAXB, bool COUNT, int PB>
__device__ v3 trace_path_shp(const KArgs& A, v3 o, v3 d, int* __restrict__ stk, Ctr& c, int& hit0, float& t0,
                             int bh_pix, int* __restrict__ sstk, int wcap) {
    static_assert(PB != 0, "the shadow pool keeps path levels in a path buffer");
    float4* pb;
    if constexpr (PB == 2) {
        extern __shared__ int lds_dyn[];
        pb = (float4*)(lds_dyn + 2 * wcap * BLOCK) + (size_t)((threadIdx.x >> 6) * MAXB) * 64 + (threadIdx.x & 63);
    } else {
        pb = A.pathbuf + ((size_t)(blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6)) * MAXB) * 64 + (threadIdx.x & 63);
    }
    unsigned* visw;  // the shadow pool's visibility words: after the path buffer (PB = 2, launch_paths adds them)
    if constexpr (PB == 2) {
        extern __shared__ int lds_dyn[];
        visw = (unsigned*)((float4*)(lds_dyn + 2 * wcap * BLOCK) + (size_t)BLOCK * MAXB) + (threadIdx.x & ~63u);
    } else {
        __shared__ unsigned visw_s[BLOCK];
        visw = visw_s + (threadIdx.x & ~63u);
    }
    const DScene& s = A.s;
    const v3 amb = mk(s.amb_x, s.amb_y, s.amb_z);
    int L = 0;
    bool tail = false, alive = true;
    for (int it = 0; it < A.bounces; ++it) {
        if (uni64(__ballot(alive)) == 0ull) break;
        bool has = false;
        v3 ip = mk(0.0f, 0.0f, 0.0f), n = ip;
        int m = 0;
        if (alive) {  // raytracer.c:101-147 as path_step
            float best;
            int nd;
            if (it == 0) c.prim++;
            else c.refl++;
            const int orig = closest<false, COUNT, true>(s, o, d, best, nd, stk, c, sstk, wcap, it > 0);
            if (it == 0) {
                hit0 = orig;
                t0 = best;
            }
            if (A.bounce_hit && bh_pix >= 0) A.bounce_hit[(size_t)bh_pix * A.bounces + it] = orig;
            if (orig < 0) {  // raytracer.c:132-135
                pb[it * 64] = make_float4(0.0f + amb.x, 0.0f + amb.y, 0.0f + amb.z, __int_as_float(0));
                L = it + 1;
                tail = false;
                alive = false;
            } else {
                c.hits++;
                ip = add(o, mul(d, best));
                const float4 sh0 = s.shade[2 * orig], sh1 = s.shade[2 * orig + 1];
                m = __float_as_int(sh0.w);
                n = nd ? xyz(sh1) : xyz(sh0);
                has = true;
            }
        }
        const unsigned vis = shadow_pool<COUNT>(s, has, ip, n, stk, sstk, wcap, A.regroup, visw, c);
        if (has) {  // raytracer.c:144-172 as path_step, the lights' visibility from the pool
            const v3 kd0 = xyz(s.mats[3 * m + 1]);
            v3 col = mk(0.0f + kd0.x * amb.x, 0.0f + kd0.y * amb.y, 0.0f + kd0.z * amb.z);
            const v3 v = mul(d, -1.0f);
            for (int j = 0; j < s.n_lights; ++j) {
                const v3 Lp = xyz(s.lights[2 * j]);
                v3 l = sub(Lp, ip);
                float mg = mag(l);
                l = dvs(l, mg);
                mg *= mg;
                const v3 tmp2 = sub(Lp, ip);
                const int V = dot(tmp2, n) < 0 ? 0 : (int)((vis >> j) & 1u);
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

}  // namespace rtd
