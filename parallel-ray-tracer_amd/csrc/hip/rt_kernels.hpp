// rt_kernels.hpp — the per-pixel hot path as HIP kernels for gfx950.
//
// One kernel per frame does everything the reference does per pixel (cpu/src/main.c:228-239 +
// cpu/src/raytracer.c:101-177): primary ray, closest-hit BVH traversal, Lambert/Blinn shading with
// one any-hit shadow ray per light, up to BOUNCES reflection rays, and the clamp.
//
// The reference recursion  raytrace(o,d,i) = c_i + kr_i * raytrace(P_i, r_i, i+1)  is evaluated
// iteratively: each level's colour c_i and material are kept in registers and the chain is folded
// from the deepest level outwards, so every float add/mul happens in the reference's order
// (the GPU reference's forward accumulation, gpu/src/raytracer.cu:61-116, does not: it differs by
// ~1e-7).
//
// Two traversal walks:
//   strict : the reference BVH in the reference's order with the reference's exact slab divisions
//            (bvh.c:48-59,269-358), including its IEEE special cases: a zero direction component
//            makes 0/0 = NaN slabs, and fminf/fmaxf then cull boxes whose face contains the ray.
//            Bit-exact by construction.
//   fast   : the acceleration BVH with a reciprocal-FMA slab test on conservatively inflated boxes.
//            Its result is the reference's except where the reference's answer depends on traversal
//            order or on the NaN special cases; those rays are detected and re-walked strictly:
//              - rays with a zero direction component (the NaN-slab cases) walk strictly from the start;
//              - closest hits that end on an exact tie in t (first-found wins in the reference,
//                bvh.c:331) are re-walked strictly.
// Kernels:
//   k_tiles  : one thread per pixel, 16x16-pixel workgroups (4 waves of 8x8), LDS traversal stack.
//   k_persist: persistent waves pulling 8x8 pixel tiles from an atomic counter.
#pragma once
#include "rt_device.hpp"

namespace rtd {

constexpr int BLOCK = 256;
constexpr int STACK = 34;  // max stack = max depth (32, bvh.c:84) + 2
enum {
    C_PRIM, C_REFL, C_SHAD, C_SKIP, C_HITS, C_CHI, C_CHL, C_CHT, C_SHI, C_SHL, C_SHT, C_PIX, C_ERR, C_FALLBACK,
    C_NB,  // node/leaf record bytes read, in 8-B units (RT_FLAG_COUNTERS)
    C_WS,  // wave-level wide-node steps (RT_FLAG_COUNTERS): lane visits / (64 x this) = SIMD efficiency
    C_WSH,  // of which shadow walks' (k_persist's walks, RT_FLAG_COUNTERS)
    C_Q1, C_Q2, C_Q3, C_Q4,  // wave steps with 1-16 / 17-32 / 33-48 / 49-64 active lanes (same)
    NLANE = 21,              // the counters above: per lane, summed over the wave at the end (flush)
    // k_persist's wave steps by walk kind (closest, shadow) x bounce level (0, 1, 2, 3+) x active lanes (1-16, 17-32,
    // 33-48, 49-64): [kind][level][quarter], 32 slots added to by the wave's first active lane (RT_FLAG_COUNTERS)
    C_HIST = NLANE,
    NCOUNT = NLANE + 32
};

struct Ctr {
    unsigned prim, refl, shad, skip, hits, chi, chl, cht, shi, shl, sht, pix, err, fb, nb, ws, wsh, q1, q2, q3, q4;
    unsigned lvl;    // the bounce level of the walks the lane runs (the histogram's level)
    unsigned* hist;  // RT_FLAG_COUNTERS kernels that keep the histogram: the workgroup's 32 slots in LDS (hist_lds)
    // evm (k_persist's production builds): the ray / pixel / fallback / error events are added to the workgroup's LDS
    // words `ev` (C_* slots) by one lane per wave and event (ev_add) instead of being counted in eight vector registers
    // held across every walk (at the 4-wave kernels' 128-VGPR cap those registers were spills)
    bool evm;
    unsigned* ev;
    // LDS_TOP kernels: the first NTOP wide nodes (the root and its interior children, breadth-first) of the primary
    // view [0] and of the unit-direction view [1], staged in the workgroup's LDS (stage_top); null: none
    const float4* top[2];
};

// The workgroup's event counters of an evm kernel (k_persist without RT_FLAG_COUNTERS): 16 words of LDS, C_PRIM ..
// C_FALLBACK, added to the launch's counters once at the end.
template <bool EV>
__device__ __forceinline__ unsigned* ev_lds() {
    __shared__ unsigned e[16];
    return e;
}
// one event for every active lane: the wave's first active lane adds their number (divergent code included)
__device__ __forceinline__ void ev_add(unsigned* ev, int slot) {
    const unsigned long long ex = __builtin_amdgcn_read_exec();
    if ((threadIdx.x & 63u) == (unsigned)__builtin_ctzll(ex)) atomicAdd(ev + slot, (unsigned)__builtin_popcountll(ex));
}
// LDS_TOP: the two views' top nodes (NTOP each, 1,440 B per workgroup), copied by the workgroup at kernel start
constexpr int NTOP = 9;  // the root + its <= 8 interior children (breadth-first records 0 .. 8)
#ifndef PRT_LDS_TOP
#define PRT_LDS_TOP 0
#endif
constexpr bool LDS_TOP = PRT_LDS_TOP != 0;
template <bool T>
__device__ __forceinline__ float4* top_lds() {
    __shared__ float4 t[2 * NTOP * 5];
    return t;
}
#define CTR_INC(c, field, slot)          \
    do {                                 \
        if ((c).evm) ev_add((c).ev, slot); \
        else (c).field++;                \
    } while (0)

// The wave-step histogram of a counting k_persist workgroup (LDS atomics; the 32 slots go to counters + C_HIST at the
// end). Instantiated only by the counting kernels, so the others' LDS budget is untouched.
template <bool COUNT>
__device__ __forceinline__ unsigned* hist_lds() {
    __shared__ unsigned h[32];
    return h;
}

__device__ __forceinline__ unsigned wave_sum(unsigned v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

template <bool COUNT>
__device__ __forceinline__ void flush(const Ctr& c, unsigned long long* g) {
    const bool l0 = (threadIdx.x & 63) == 0;
    unsigned v[NLANE] = {c.prim, c.refl, c.shad, c.skip, c.hits, c.chi, c.chl, c.cht, c.shi, c.shl, c.sht,
                          c.pix,  c.err,  c.fb,   c.nb,   c.ws,   c.wsh, c.q1,  c.q2,  c.q3,  c.q4};
#pragma unroll
    for (int i = 0; i < NLANE; i++) {
        if (!COUNT && ((i >= C_CHI && i <= C_SHT) || i >= C_NB)) continue;
        unsigned s = wave_sum(v[i]);
        if (l0 && s) atomicAdd(g + i, (unsigned long long)s);
    }
}

__device__ __forceinline__ bool degenerate(v3 d) { return d.x == 0.0f || d.y == 0.0f || d.z == 0.0f; }
// v is one of the n sorted face coordinates f (lower bound; -0 == +0 counts as equal)
__device__ __forceinline__ bool on_face(const float* __restrict__ f, int n, float v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (f[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo < n && f[lo] == v;
}
// a degenerate direction (a zero component) whose origin lies on no box face of the reference tree along each zero
// axis: the reference's slab test then divides no 0 by 0 -- (lo - o) / 0 is an infinity -- and behaves as the
// ordinary one, so the fast walk finds what the reference finds (the even-width centre column's primary rays: ~1,300
// strict walks per dragon frame on most cameras of a walkthrough, +0.2-0.4 ms per single frame; their reflections
// off axis-aligned walls). An origin on such a face (a camera coordinate a vertex shares) walks strictly.
__device__ __forceinline__ bool degenerate_ok(const DScene& s, v3 o, v3 d) {
    if (!s.faces) return false;
    if (d.x == 0.0f && on_face(s.faces, s.n_face[0], o.x)) return false;
    if (d.y == 0.0f && on_face(s.faces + s.n_face[0], s.n_face[1], o.y)) return false;
    if (d.z == 0.0f && on_face(s.faces + s.n_face[0] + s.n_face[1], s.n_face[2], o.z)) return false;
    return o.x == o.x && o.y == o.y && o.z == o.z;
}

// The reference walk reaches triangle t (original index) of a degenerate ray (a zero component of d): no child box
// on its reference path, leaf to root, has a face at the origin's coordinate along a zero axis -- those the
// reference's slab test culls (0 / 0, §2). Every box on the path holds the hit point, so it is on no other side of the
// origin there. The fast walk's winner t, reached, is then the reference's (nothing is hit before it).
__device__ __forceinline__ bool ref_reaches(const DScene& s, int t, v3 o, v3 d) {
    const int leaf = s.ref_path[t];
    int cur = ~leaf, r = s.ref_path[s.n_tris + leaf];
    for (int depth = 0; r >= 0; depth++) {
        if (depth > 64) return false;  // (a malformed path: the strict walk decides)
        const float4* N = s.ref.nodes + 4 * r;
        const float4 a = N[0], b = N[1], e = N[2], q = N[3];
        const bool left = __float_as_int(q.x) == cur;
        const v3 lo = left ? mk(a.x, a.y, a.z) : mk(b.z, b.w, e.x);
        const v3 hi = left ? mk(a.w, b.x, b.y) : mk(e.y, e.z, e.w);
        if (d.x == 0.0f && (lo.x == o.x || hi.x == o.x)) return false;
        if (d.y == 0.0f && (lo.y == o.y || hi.y == o.y)) return false;
        if (d.z == 0.0f && (lo.z == o.z || hi.z == o.z)) return false;
        cur = r;
        r = __float_as_int(q.z);
    }
    return true;
}

// fast-walk pruning: visit a box whose entry is within 4 ulp of the best hit, so that a triangle tied
// with the best hit is always reached (and the tie detected) despite the reciprocal test's rounding.
constexpr float PRUNE_SLACK = 1.0000005f;

// Shadow rays (fast walks): a triangle can occlude only if ld2 > |o - (o + d t)|^2 (bvh.c:283-290), which
// holds for no t beyond this bound, so boxes entered past it are pruned from the start. Margins: |d| = 1
// within 2 ulp (l is normalised, raytracer.c:153), and the rounding of ip = o + d t and o - ip is at most
// a few ulp of max|o| absolute; 1e-3 relative + 1e-5 max|o| exceed both by > 50x. The result ("some
// triangle nearer than the light") does not depend on which farther boxes are visited.
__device__ __forceinline__ float shadow_reach(v3 o, float ld2) {
    const float om = fmaxf(fmaxf(__builtin_fabsf(o.x), __builtin_fabsf(o.y)), __builtin_fabsf(o.z));
    return __builtin_sqrtf(ld2) * 1.001f + om * 1e-5f;
}

// ---------------------------------------------------------------- one interior node
// Entry distances of both children of record `ref`, nearer child first (empty child / miss: FMAX).
template <bool STRICT>
__device__ __forceinline__ void children(const DBvh& B, int ref, v3 o, v3 d, const RayPre& p, int& ni, float& nt,
                                         int& fi, float& ft) {
    const float4* N = B.nodes + 4 * ref;
    const float4 a = N[0], b = N[1], e = N[2], r = N[3];
    ni = __float_as_int(r.x);
    fi = __float_as_int(r.y);
    if (STRICT) {
        nt = box_exact(mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), o, d);
        ft = box_exact(mk(b.z, b.w, e.x), mk(e.y, e.z, e.w), o, d);
    } else {
        nt = box_fast(a.x, a.y, a.z, a.w, b.x, b.y, p);
        ft = box_fast(b.z, b.w, e.x, e.y, e.z, e.w, p);
    }
    if (ni == EMPTY_REF) nt = FMAX;
    if (fi == EMPTY_REF) ft = FMAX;
    if (ft < nt) {
        const int ti = ni;
        const float tt = nt;
        ni = fi;
        nt = ft;
        fi = ti;
        ft = tt;
    }
}

// children<true> with each child's slab exit as well (nx, fx): the strict order and entries bit for bit
__device__ __forceinline__ void children_out(const DBvh& B, int ref, v3 o, v3 d, int& ni, float& nt, float& nx, int& fi,
                                             float& ft, float& fx) {
    const float4* N = B.nodes + 4 * ref;
    const float4 a = N[0], b = N[1], e = N[2], r = N[3];
    ni = __float_as_int(r.x);
    fi = __float_as_int(r.y);
    nt = box_exact_out(mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), o, d, nx);
    ft = box_exact_out(mk(b.z, b.w, e.x), mk(e.y, e.z, e.w), o, d, fx);
    if (ni == EMPTY_REF) nt = FMAX;
    if (fi == EMPTY_REF) ft = FMAX;
    if (ft < nt) {
        const int ti = ni;
        const float tt = nt, tx = nx;
        ni = fi;
        nt = ft;
        nx = fx;
        fi = ti;
        ft = tt;
        fx = tx;
    }
}

// Is a child whose box is entered at t worth visiting? Strict: the reference's test (bvh.c:343-352).
template <bool STRICT>
__device__ __forceinline__ bool visit(float t, float best) {
    if (STRICT) return t < best;
    return t <= best * PRUNE_SLACK && t != FMAX;
}

// A per-pixel output index as the compiler cannot see through (OPAQUE_OUT): the 64-bit output addresses formed from it
// are made where they are stored instead of once per pixel and held -- or spilled -- across the path's walks (the
// per-level pool kernel spilled three of them, 24 B per lane stored per pixel; the packed spp > 1 build one per sample).
#ifndef PRT_OPAQUE_OUT
#define PRT_OPAQUE_OUT 1
#endif
__device__ __forceinline__ int opaque(int v) {
    if (PRT_OPAQUE_OUT) __asm__ volatile("" : "+v"(v));
    return v;
}

// ---------------------------------------------------------------- closest hit
// bvh_traverse, cpu/src/bvh.c:317-358. Stack of node refs in LDS, [depth][lane] so that the 64 lanes
// of a wave always hit 64 distinct banks whatever their stack depths.
// REG: the node to visit next is kept in a register and only the farther child goes through the LDS
// stack (the reference pushes far then near and pops near at once: the same visiting sequence, one
// LDS round trip less on the dependent chain of most steps).
// Returns the leaf position of the best hit in hp (-1: none); `tie` = the final best was matched by
// another triangle (fast walk only).
// CUT (the strict walk of an exact tie, closest()): also skip a child the ray leaves before `cut` -- the reference
// would visit it, but every triangle in it is hit before cut or not at all, and no triangle is hit before the tie's
// t, so it holds none the walk could take: the same triangles are taken in the same order, the same one wins, without
// the walk through every box the ray crosses on its way to the tie (most of what the bounded re-walk visited).
template <bool STRICT, bool COUNT, bool REG = true, bool CUT = false>
__device__ __forceinline__ void closest_walk(const DBvh& B, v3 o, v3 d, float& best, int& hp, int& nd, bool& tie,
                                             int* __restrict__ stk, Ctr& c, float cut = 0.0f) {
    RayPre p = {};
    if (!STRICT) p = ray_pre(o, d);
    int sp = 0, cur = B.root;
    if (!REG) {
        stk[0] = B.root;
        sp = 1;
    }
    for (;;) {
        if (!REG) {
            if (sp == 0) break;
            cur = stk[(--sp) * BLOCK];
        }
        if (cur < 0) {
            const int2 lf = B.leaves[~cur];
            if (COUNT) {
                c.chl++;
                c.nb += 1;
            }
            for (int i = lf.x; i < lf.x + lf.y; ++i) {
                int k;
                const float tt = hit_triangle(o, d, B.tris + 3 * i, k);
                if (COUNT) c.cht++;
                if (tt < best) {
                    best = tt;
                    nd = k;
                    hp = i;
                    if (!STRICT) tie = false;
                } else if (!STRICT && tt == best && tt != FMAX) {
                    tie = true;
                }
            }
        } else {
            if (COUNT) {
                c.chi++;
                c.nb += 8;
            }
            int ni, fi;
            float nt, ft;
            bool vn, vf;
            if constexpr (CUT) {
                float nx, fx;
                children_out(B, cur, o, d, ni, nt, nx, fi, ft, fx);
                vn = visit<STRICT>(nt, best) && !(nx < cut);
                vf = visit<STRICT>(ft, best) && !(fx < cut);
            } else {
                children<STRICT>(B, cur, o, d, p, ni, nt, fi, ft);
                vn = visit<STRICT>(nt, best);
                vf = visit<STRICT>(ft, best);
            }
            if (sp + 2 > STACK) {  // cannot happen for depth <= 32 BVHs; reported, never silent
                CTR_INC(c, err, C_ERR);
                break;
            }
            if (REG) {
                if (vn) {
                    if (vf) stk[(sp++) * BLOCK] = fi;
                    cur = ni;
                    continue;
                }
                if (vf) {
                    cur = fi;
                    continue;
                }
            } else {
                if (vf) stk[(sp++) * BLOCK] = fi;
                if (vn) stk[(sp++) * BLOCK] = ni;
                continue;
            }
        }
        if (REG) {
            if (sp == 0) break;
            cur = stk[(--sp) * BLOCK];
        }
    }
}

// Any hit toward a light: bvh_light_traverse, cpu/src/bvh.c:269-315 (returns visibility).
// Occluded iff some triangle hit closer than the light exists: independent of the visiting order.
template <bool STRICT, bool COUNT, bool REG = true>
__device__ __forceinline__ bool visible_walk(const DBvh& B, v3 o, v3 d, float ld2, int* __restrict__ stk, Ctr& c) {
    RayPre p = {};
    if (!STRICT) p = ray_pre(o, d);
    // fast walk: prune at the light (visit(t, best) tests t <= best * PRUNE_SLACK); strict: the reference's walk
    float best = STRICT ? FMAX : shadow_reach(o, ld2);
    int sp = 0, cur = B.root;
    if (!REG) {
        stk[0] = B.root;
        sp = 1;
    }
    for (;;) {
        if (!REG) {
            if (sp == 0) break;
            cur = stk[(--sp) * BLOCK];
        }
        if (cur < 0) {
            const int2 lf = B.leaves[~cur];
            if (COUNT) {
                c.shl++;
                c.nb += 1;
            }
            for (int i = lf.x; i < lf.x + lf.y; ++i) {
                int k;
                const float tt = hit_triangle(o, d, B.tris + 3 * i, k);
                if (COUNT) c.sht++;
                if (tt < best) {
                    best = tt;
                    const v3 ip = add(o, mul(d, best));
                    const v3 oi = sub(o, ip);
                    if (ld2 > dot(oi, oi)) return false;
                }
            }
        } else {
            if (COUNT) {
                c.shi++;
                c.nb += 8;
            }
            int ni, fi;
            float nt, ft;
            children<STRICT>(B, cur, o, d, p, ni, nt, fi, ft);
            const bool vn = visit<STRICT>(nt, best), vf = visit<STRICT>(ft, best);
            if (sp + 2 > STACK) {
                CTR_INC(c, err, C_ERR);
                break;
            }
            if (REG) {
                if (vn) {
                    if (vf) stk[(sp++) * BLOCK] = fi;
                    cur = ni;
                    continue;
                }
                if (vf) {
                    cur = fi;
                    continue;
                }
            } else {
                if (vf) stk[(sp++) * BLOCK] = fi;
                if (vn) stk[(sp++) * BLOCK] = ni;
                continue;
            }
        }
        if (REG) {
            if (sp == 0) break;
            cur = stk[(--sp) * BLOCK];
        }
    }
    return true;
}

// ---------------------------------------------------------------- 8-wide quantised walk (fast)
// Node-group traversal (after Ylitie et al., "Efficient Incoherent Ray Traversal on GPUs Through
// Compressed Wide BVHs", HPG 2017): one visit tests all 8 child boxes, tests the triangles of every
// hit leaf slot at once, and keeps the hit interior children as ONE stack entry (child base, imask,
// hit bits) popped child by child in the order k ^ octant(ray) (near first, no sort).
// Same result semantics as closest_walk<false>: min t over all triangles, boxes pruned at
// best * PRUNE_SLACK so that exact ties are always met and reported.
constexpr int WSTACK = 16;  // node-group entries in the STACK-int LDS column; builder depth <= 16
// A stack entry is two words (child base; interior mask << 8 | hit bits). PK (the shadow-pool kernels): one word
// (child base << 8 | hit bits) plus the interior mask as one byte, four entries' bytes to a word after the wcap entry
// words -- 5 bytes per entry, so that the all-levels pool's path buffer fits 4 workgroups per CU beside the stack of
// deeper trees (sportscar depth 14, two_cars 12) -- at 4 more VALU per push / pop. The pool kernels pack, and so does
// PERSIST4's SHP = 3 build (packed stack entries plus packed triangle tests, which together win). The packed child
// base has 24 bits: wide trees of at most WIDE_MAX_NODES nodes; the host (rt_hip.hip persist_kernel, shp_ok) runs the
// unpacked builds for larger trees.
constexpr int WIDE_MAX_NODES = 1 << 24;
__host__ __device__ constexpr int wstack_words(int wcap, bool pk) { return pk ? wcap + (wcap + 3) / 4 : 2 * wcap; }
// A child box left before t = EPS holds no hit: hit_triangle accepts t > EPS only (raytracer.c:56), and the
// computed far plane lies beyond the true box by the inflation (>= 20x the triangle test's rounding of t), so
// every triangle point inside has t below the computed exit. Testing the interval from EPS instead of 0 prunes
// such boxes for free — above all the flat boxes of the surface a shadow or reflection ray starts on (a wall's
// whole subtree is a stack of flat boxes around the ray's origin).
constexpr float BOX_TMIN = EPS;
// Shadow walks visit a node's hit children FAR first (visiting order k ^ (octant ^ 7): from the light's side
// toward the ray origin; the closest walks stay near-first). An any-hit walk's result does not depend on the
// order; far-first meets an occluder sooner on average — a shadow ray leaves a surface whose own neighbourhood
// (first in near-first order) cannot occlude it. Same box, 16-frame batches: dragon 0.810 -> 0.804 ms per
// frame, car_boxed 0.922 -> 0.884, sportscar 1.374 -> 1.334; wave steps -2 / -5 / -4 %.
constexpr unsigned SHADOW_ORDER_XOR = 7u;

// 1 in the lowest active lane of the wave, 0 elsewhere (wave-level step counting)
__device__ __forceinline__ unsigned first_active_lane() {
    const unsigned long long ex = __builtin_amdgcn_read_exec();
    return (unsigned)((threadIdx.x & 63u) == (unsigned)__builtin_ctzll(ex));
}

// Diagnostics build (PRT_DEFS=-DPRT_DIAG_TRI): the lane-count bins q1 / q2 count the wave iterations of the closest /
// shadow walks' triangle loops instead (their SIMD efficiency = c.cht / (64 q1), c.sht / (64 q2)).
#ifdef PRT_DIAG_TRI
#define PRT_TRI_ITER(c, q) \
    do {                   \
        if (COUNT) (c).q += first_active_lane(); \
    } while (0)
#else
#define PRT_TRI_ITER(c, q) \
    do {                   \
    } while (0)
#endif

// k_persist's walks (RT_FLAG_COUNTERS): one wave step, by walk kind and by the number of active lanes
__device__ __forceinline__ void count_step(Ctr& c, bool shadow) {
    const unsigned long long ex = __builtin_amdgcn_read_exec();
    const unsigned f = (unsigned)((threadIdx.x & 63u) == (unsigned)__builtin_ctzll(ex));
    const unsigned b = ((unsigned)__builtin_popcountll(ex) - 1u) >> 4;
    c.ws += f;
    if (shadow) c.wsh += f;
#ifndef PRT_DIAG_TRI
    c.q1 += b == 0 ? f : 0u;
    c.q2 += b == 1 ? f : 0u;
    c.q3 += b == 2 ? f : 0u;
    c.q4 += b == 3 ? f : 0u;
#endif
    if (c.hist && f) atomicAdd(c.hist + (shadow ? 16u : 0u) + 4u * (c.lvl < 3u ? c.lvl : 3u) + b, 1u);
}

// Plane decoding (rt_wide.cpp): plane = fmaf(2^e, QBIAS + q, p). QBIAS + q is an f16 integer with the bits
// 0x6400 | q, so one v_perm_b32 makes two of them from two plane bytes of a node word (the constant bytes 0x64 from
// its second source), and v_fma_mix_f32 converts a half inside the FMA: t = (QBIAS + q) * k + a with the product
// exact and one rounding -- fmaf((float)(QBIAS + q), k, a) bit for bit (checked exhaustively over q and 2^31 (k, a)
// pairs incl. specials on the GPU, tools/mix/mix_check.hip). Per node visit: 24 perms + 48 FMAs instead of 48 byte
// conversions + 48 FMAs.
constexpr unsigned QBIAS = 1024u;
// A node word holds one slot pair's planes of one axis (qlo[2j], qhi[2j], qlo[2j+1], qhi[2j+1]); the byte selector picks
// the pair's near or far planes by the ray's sign on that axis (plane_sel), so no per-node select of words is needed.
__device__ __forceinline__ unsigned plane_pair(unsigned w, unsigned sel) {  // two planes of a word -> two f16 halves
    return __builtin_amdgcn_perm(w, 0x64646464u, sel);
}
// the selector of a pair's near (far = false: far) planes: bytes 0 / 2 (the lo planes) or 1 / 3 (hi) of the word
// (perm indices 4..7), each under a constant 0x64 byte (index 0)
#ifndef PRT_SEL_FAR_XOR
#define PRT_SEL_FAR_XOR 1
#endif
__device__ __forceinline__ unsigned plane_sel(bool neg, bool near) {
    return (neg == near) ? 0x00070005u : 0x00060004u;
}
// 2 h + c with the compare's lane mask as the carry: one instruction per slot where a select and an OR took two
#ifndef PRT_HIT_ADDC
#define PRT_HIT_ADDC 1
#endif
constexpr bool HIT_ADDC = PRT_HIT_ADDC != 0;
__device__ __forceinline__ unsigned shift_in(unsigned h, bool c) {
    const unsigned long long m = __builtin_amdgcn_ballot_w64(c);
    unsigned r;
    unsigned long long co;
    __asm__("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(co) : "v"(h), "s"(m));
    return r;
}
__device__ __forceinline__ unsigned far_sel(unsigned near_sel) {
    unsigned r;
    __asm__ volatile("v_xor_b32 %0, 0x10001, %1" : "=v"(r) : "v"(near_sel));
    return r;
}
__device__ __forceinline__ float max_raw(float a, float b) {
    float r;
    __asm__("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float min_raw(float a, float b) {
    float r;
    __asm__("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float max3_raw(float a, float b, float c) {
    float r;
    __asm__("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float min3_raw(float a, float b, float c) {
    float r;
    __asm__("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float fma_half(unsigned h2, int hi, float k, float a) {  // fmaf(f16 half of h2, k, a)
    float r;
    if (hi) __asm__("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h2), "v"(k), "v"(a));
    else __asm__("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h2), "v"(k), "v"(a));
    return r;
}
// fma_half with the result clamped to [0, 1] by the instruction's clamp bit (the shadow walks' rescaled t, below)
__device__ __forceinline__ float fma_half_clamp(unsigned h2, int hi, float k, float a) {
    float r;
    if (hi)
        __asm__("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0] clamp" : "=v"(r) : "v"(h2), "v"(k), "v"(a));
    else __asm__("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0] clamp" : "=v"(r) : "v"(h2), "v"(k), "v"(a));
    return r;
}

// Shadow walks on rescaled t (PRT_SHADOW_CLAMP). A shadow walk's box interval is tested against [BOX_TMIN, reach]
// with reach fixed per ray (shadow_reach: a hit beyond it cannot occlude, and the walk ends at the first occluder, so
// the running `best` only ever pruned between the light and reach). With t' = (t - BOX_TMIN) / (reach - BOX_TMIN) the
// interval is [0, 1], which the plane FMA's clamp bit applies for free: the ray's constants are rescaled once
// (ray_pre_shadow), and the slot test is max3(clamped near) < min3(clamped far) -- 2 VALU per slot (16 per visit)
// fewer than the max / min with BOX_TMIN and lim. Strict <: a box left before BOX_TMIN or entered after reach clamps
// both ends to 0 or both to 1 and fails it; a box holding a point t* in (BOX_TMIN, reach] has every computed near
// below t*' and every far above it by the inflation's margin (the rescale adds 2-3 ulp of max|coord| / |d| of rounding
// to the few the plane FMA had, still covered >= 10x by 2^-16 max|coord|), so lo' < t*' <= hi' or lo' <= t*' < hi'.
#ifndef PRT_SHADOW_CLAMP
#define PRT_SHADOW_CLAMP 1
#endif
constexpr bool SHADOW_CLAMP = PRT_SHADOW_CLAMP != 0;
__device__ __forceinline__ RayPre ray_pre_shadow(v3 o, v3 d, float reach) {
    RayPre p = ray_pre(o, d);
    if (SHADOW_CLAMP) {
        // s <= 1 / (reach - BOX_TMIN) up to one rounding, then 2^-20 smaller: the [0, 1] of t' covers [BOX_TMIN, reach]
        // (reach <= BOX_TMIN: nothing can occlude; any positive scale is then conservative)
        const float span = reach - BOX_TMIN;
        const float s = span > 1e-30f ? (1.0f / span) * 0.999999f : 1.0f;
        p.ox = (p.ox + BOX_TMIN) * s;
        p.ix *= s;
        p.iy *= s;
        p.iz *= s;
        p.oy = (p.oy + BOX_TMIN) * s;
        p.oz = (p.oz + BOX_TMIN) * s;
    }
    return p;
}
// The closest walks' lim moves with every hit, so their t is only shifted and scaled by the exact 2^-40
// (ray_pre_closest; PRT_CLOSEST_CLAMP): [BOX_TMIN, BOX_TMIN + 2^40] is [0, 1], the clamp bit applies the lower end, and
// the upper end stays an explicit min with the scaled lim (closest_lim): 1 VALU per slot fewer. No hit distance of
// a scene comes near 2^40, and 2^-40 keeps the planes' scale 2^e / d far from the denormals; a zero direction
// component's 1e20 reciprocal (safe_dir) only sends that axis' slab ends to 0 and 1 together, as to -/+huge before.
#ifndef PRT_CLOSEST_CLAMP
#define PRT_CLOSEST_CLAMP 1
#endif
constexpr bool CLOSEST_CLAMP = PRT_CLOSEST_CLAMP != 0;
constexpr float CLAMP_SCALE = 0x1p-40f;
__device__ __forceinline__ RayPre ray_pre_closest(v3 o, v3 d) {
    RayPre p = ray_pre(o, d);
    if (CLOSEST_CLAMP) {
        p.ox = (p.ox + BOX_TMIN) * CLAMP_SCALE;
        p.oy = (p.oy + BOX_TMIN) * CLAMP_SCALE;
        p.oz = (p.oz + BOX_TMIN) * CLAMP_SCALE;
        p.ix *= CLAMP_SCALE;
        p.iy *= CLAMP_SCALE;
        p.iz *= CLAMP_SCALE;
    }
    return p;
}
// the closest walks' box limit: best * PRUNE_SLACK, or under CLOSEST_CLAMP that limit in the rescaled t (one FMA, one
// rounding of a value 4 ulp above best: ties stay reached)
__device__ __forceinline__ float closest_lim(float best) {
    if (CLOSEST_CLAMP) return __builtin_fmaf(best, PRUNE_SLACK * CLAMP_SCALE, -BOX_TMIN * CLAMP_SCALE);
    return best * PRUNE_SLACK;
}

// Tests the 8 children of wide node `node`: nh = hit interior slots as bits (s ^ oct), th = triangle
// bits (relative to tbase) of every hit leaf slot.
struct WNode {
    float4 f0, f1, f2, f3, f4;
};
// The upper levels in LDS (LDS_TOP, north star "LDS-staged upper BVH levels"): every walk starts with the root and
// most continue into its children; with `top` set, a node below NTOP is read from the workgroup's LDS copy. The
// address is selected, not branched on (a flat load serves both), so the next-node load stays unconditional.
// PRT_PIN_NODE: the node's five float4 held in register quads at the walk loop's head (an empty asm), so that the
// loads of the next node land where the node test reads them
#ifndef PRT_PIN_NODE
#define PRT_PIN_NODE 1
#endif
typedef float pin4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void pin_q(float4& f) {
    pin4 v = {f.x, f.y, f.z, f.w};
    __asm__ volatile("" : "+v"(v));
    f = make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void pin_node(WNode& N) {
    if (PRT_PIN_NODE) {
        pin_q(N.f0);
        pin_q(N.f1);
        pin_q(N.f2);
        pin_q(N.f3);
        pin_q(N.f4);
    }
}
__device__ __forceinline__ WNode wload(const DWide& W, int node, const float4* top = nullptr) {
    const float4* N = (top && node < NTOP) ? top + 5 * node : W.nodes + 5 * node;
    return WNode{N[0], N[1], N[2], N[3], N[4]};
}
// The walks' node array as a value held in scalar registers for the whole walk (PRT_PIN_BASE): read from the kernel
// arguments once. Without it the compiler, short of scalar registers, re-read W.nodes from the kernel arguments at
// every step (an s_load rematerialised instead of a spill), and that load's s_waitcnt lgkmcnt(0) sat between the
// stack pop and the next node's loads, waiting for every LDS operation of the step as well. The view of a walk is
// the same for every lane of the wave (the bounce level or the pool's fixed view decides it).
#ifndef PRT_PIN_BASE
#define PRT_PIN_BASE 1
#endif
// (a global-address-space pointer: its loads stay global_load, which the compiler waits for by vmcnt alone; a generic
// pointer's flat loads are waited for with lgkmcnt too)
typedef const pin4 __attribute__((address_space(1))) * gnodes;
__device__ __forceinline__ gnodes walk_base(const float4* p) {
    unsigned long long v = (unsigned long long)p;
    if (PRT_PIN_BASE) __asm__ volatile("" : "+s"(v));
    return (gnodes)v;
}
__device__ __forceinline__ float4 f4(pin4 v) { return make_float4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ WNode wload_at(gnodes base, int node, const float4* top = nullptr) {
    if (LDS_TOP && top && node < NTOP) {
        const float4* N = top + 5 * node;
        return WNode{N[0], N[1], N[2], N[3], N[4]};
    }
    gnodes N = base + 5 * node;
    return WNode{f4(N[0]), f4(N[1]), f4(N[2]), f4(N[3]), f4(N[4])};
}


// LATE (PRT_LATE_TRIS): th returns the hit leaf SLOTS (bits 0..7) and the walk forms the triangle bits from them with
// leaf_tris after it has issued the next node's loads (the slot loop is off the dependent chain from this node's
// loads to the next node's)
#ifndef PRT_LATE_TRIS
#define PRT_LATE_TRIS 1
#endif
constexpr bool LATE_TRIS = PRT_LATE_TRIS != 0;
// CLAMP 1: p is ray_pre_shadow's (t rescaled so that [BOX_TMIN, reach] is [0, 1]); lim is unused. CLAMP 2: p is
// ray_pre_closest's, lim closest_lim's
template <bool COUNT, bool LATE = false, int CLAMP = 0>
__device__ __forceinline__ void wide_node(const WNode& nd, const RayPre& p, unsigned oct, float lim, unsigned& nh,
                                          unsigned& th, int& cbase, int& tbase, unsigned& imask, unsigned& nleaf,
                                          unsigned ord_xor = 0u) {
    const float4 f0 = nd.f0, f1 = nd.f1, f2 = nd.f2, f3 = nd.f3, f4 = nd.f4;
    const unsigned e = __float_as_uint(f0.w);  // exponents (signed bytes) | interior mask
    imask = e >> 24;
    cbase = __float_as_int(f1.x);
    tbase = __float_as_int(f1.y);
    const unsigned m[2] = {__float_as_uint(f1.z), __float_as_uint(f1.w)};
    // The ray in the node's grid: plane q of axis x is entered at t = fma(q, 2^ex / d.x, (p.x - o.x) / d.x),
    // computed as fma(1024 + q, kx, ax) (fma_half) with kx = 2^ex * (1/d.x) (exact: power-of-two scale) and
    // ax = fma(p.x, 1/d.x, -o.x/d.x): one FMA per plane. Its rounding reach (a few ulp of max|coord| / |d|)
    // is covered >= 20x by the boxes' inflation (2^-16 max|coord|, rt_hip.hip).
    const float ax = __builtin_fmaf(f0.x, p.ix, -p.ox), ay = __builtin_fmaf(f0.y, p.iy, -p.oy),
                az = __builtin_fmaf(f0.z, p.iz, -p.oz);
    const float kx = __builtin_ldexpf(p.ix, (int)(signed char)(e & 0xFFu)),
                ky = __builtin_ldexpf(p.iy, (int)(signed char)((e >> 8) & 0xFFu)),
                kz = __builtin_ldexpf(p.iz, (int)(signed char)((e >> 16) & 0xFFu));
    // near / far plane bytes per axis from the direction signs (== min / max of the two slab ends): byte selectors
    // (loop-invariant over the walk: oct is the ray's)
    const bool bx = (oct & 1u) != 0, by = (oct & 2u) != 0, bz = (oct & 4u) != 0;
    const unsigned nsx = plane_sel(bx, true), nsy = plane_sel(by, true), nsz = plane_sel(bz, true);
#if PRT_SEL_FAR_XOR
    // far = near with the other byte of each plane pair, derived per node (a volatile XOR: hoisted, the compiler
    // would hold three more loop-invariant registers and spill)
    const unsigned fsx = far_sel(nsx), fsy = far_sel(nsy), fsz = far_sel(nsz);
#else
    const unsigned fsx = plane_sel(bx, false), fsy = plane_sel(by, false), fsz = plane_sel(bz, false);
#endif
    const unsigned wx[4] = {__float_as_uint(f2.x), __float_as_uint(f2.y), __float_as_uint(f2.z), __float_as_uint(f2.w)},
                   wy[4] = {__float_as_uint(f3.x), __float_as_uint(f3.y), __float_as_uint(f3.z), __float_as_uint(f3.w)},
                   wz[4] = {__float_as_uint(f4.x), __float_as_uint(f4.y), __float_as_uint(f4.z), __float_as_uint(f4.w)};
    unsigned hit8 = 0;  // bit s: child slot s entered within [0, lim]
#pragma unroll
    for (int s = HIT_ADDC ? 7 : 0; HIT_ADDC ? s >= 0 : s < 8; s += HIT_ADDC ? -1 : 1) {
        const int j = s >> 1, hb = s & 1;
        if constexpr (CLAMP == 2) {  // (ray_pre_closest)
            const float tnx = fma_half_clamp(plane_pair(wx[j], nsx), hb, kx, ax);
            const float tfx = fma_half(plane_pair(wx[j], fsx), hb, kx, ax);
            const float tny = fma_half_clamp(plane_pair(wy[j], nsy), hb, ky, ay);
            const float tfy = fma_half(plane_pair(wy[j], fsy), hb, ky, ay);
            const float tnz = fma_half_clamp(plane_pair(wz[j], nsz), hb, kz, az);
            const float tfz = fma_half(plane_pair(wz[j], fsz), hb, kz, az);
            const float lo = max3_raw(tnx, tny, tnz);
            const float hi = min3_raw(tfx, tfy, min_raw(tfz, lim));
            if (HIT_ADDC) hit8 = shift_in(hit8, lo < hi);
            else hit8 |= lo < hi ? (1u << s) : 0u;
            continue;
        }
        if constexpr (CLAMP == 1) {  // (ray_pre_shadow)
            const float tnx = fma_half_clamp(plane_pair(wx[j], nsx), hb, kx, ax);
            const float tfx = fma_half_clamp(plane_pair(wx[j], fsx), hb, kx, ax);
            const float tny = fma_half_clamp(plane_pair(wy[j], nsy), hb, ky, ay);
            const float tfy = fma_half_clamp(plane_pair(wy[j], fsy), hb, ky, ay);
            const float tnz = fma_half_clamp(plane_pair(wz[j], nsz), hb, kz, az);
            const float tfz = fma_half_clamp(plane_pair(wz[j], fsz), hb, kz, az);
            const float lo = max3_raw(tnx, tny, tnz);
            const float hi = min3_raw(tfx, tfy, tfz);
            if (HIT_ADDC) hit8 = shift_in(hit8, lo < hi);
            else hit8 |= lo < hi ? (1u << s) : 0u;
            continue;
        }
        const float tnx = fma_half(plane_pair(wx[j], nsx), hb, kx, ax);
        const float tfx = fma_half(plane_pair(wx[j], fsx), hb, kx, ax);
        const float tny = fma_half(plane_pair(wy[j], nsy), hb, ky, ay);
        const float tfy = fma_half(plane_pair(wy[j], fsy), hb, ky, ay);
        const float tnz = fma_half(plane_pair(wz[j], nsz), hb, kz, az);
        const float tfz = fma_half(plane_pair(wz[j], fsz), hb, kz, az);
        // Inflation (2^-16 max|coord|) puts every computed near plane strictly before and every far plane
        // strictly after the child's true box, per axis, so the interval below contains the true one; the
        // folded test max(tmin, BOX_TMIN) <= min(tmax, lim) only adds visits: conservative (BOX_TMIN below).
        // (max3 / min3 of the asm results directly: fmaxf / fminf would first canonicalise each asm output, one
        // v_max_f32 per plane; the entries are never NaN here -- zero direction components walk strictly)
        const float lo = max3_raw(tnx, tny, max_raw(tnz, BOX_TMIN));
        const float hi = min3_raw(tfx, tfy, min_raw(tfz, lim));
        if (HIT_ADDC) hit8 = shift_in(hit8, lo <= hi);  // (slots 7 .. 0: slot s ends at bit s)
        else hit8 |= lo <= hi ? (1u << s) : 0u;
    }
    // interior hits, permuted into visiting order: bit k = slot k ^ oct (XOR by oct swaps bits, pairs and
    // nibbles of the 8-bit mask)
    unsigned x = hit8 & imask;
    const unsigned ord = oct ^ ord_xor;  // visiting order k ^ ord (ord_xor 7: far children first)
    x = (ord & 1u) ? (((x & 0x55u) << 1) | ((x >> 1) & 0x55u)) : x;
    x = (ord & 2u) ? (((x & 0x33u) << 2) | ((x >> 2) & 0x33u)) : x;
    x = (ord & 4u) ? (((x & 0x0Fu) << 4) | ((x >> 4) & 0x0Fu)) : x;
    nh = x;
    // triangles of the hit leaf slots (meta = count << 5 | offset; an empty slot's inverted box never
    // passes the test above except through underflow, and its meta 0 adds nothing then)
    unsigned lh = hit8 & ~imask;
    th = 0;
    nleaf = 0;
    if constexpr (LATE) {  // (the slots; leaf_tris later)
        th = lh;
        return;
    }
    while (lh) {
        const unsigned sl = (unsigned)__builtin_ctz(lh);
        lh &= lh - 1u;
        const unsigned meta = (m[sl >> 2] >> (8u * (sl & 3u))) & 0xFFu;
        th |= ((1u << (meta >> 5)) - 1u) << (meta & 31u);
        if (COUNT) nleaf += meta ? 1u : 0u;
    }
}

// The triangle bits (relative to the node's tri base) of hit leaf slots lh, from the node's meta words m0 / m1 (f1.z,
// f1.w): wide_node's loop, for the LATE walks
template <bool COUNT>
__device__ __forceinline__ unsigned leaf_tris(unsigned lh, unsigned m0, unsigned m1, unsigned& nleaf) {
    unsigned th = 0;
    nleaf = 0;
    while (lh) {
        const unsigned sl = (unsigned)__builtin_ctz(lh);
        lh &= lh - 1u;
        const unsigned meta = ((sl < 4u ? m0 : m1) >> (8u * (sl & 3u))) & 0xFFu;
        th |= ((1u << (meta >> 5)) - 1u) << (meta & 31u);
        if (COUNT) nleaf += meta ? 1u : 0u;
    }
    return th;
}

// The node visited after this one: the nearest remaining hit child of this node, else the top group
// of the stack (pushing / re-pushing the rest). It does not depend on this node's triangle tests, so
// the walks issue its loads BEFORE those tests and their latency overlaps them. -1: walk done; -2: stack
// overflow (reported, never silent).
template <bool PK = false>
__device__ __forceinline__ int wide_next(unsigned nh, int cb, unsigned imask, unsigned oct, int& sp,
                                         int* __restrict__ stk, int wcap = WSTACK) {
    if (!nh) {
        if (sp == 0) return -1;
        --sp;
        if constexpr (PK) {
            const unsigned e = (unsigned)stk[sp * BLOCK];
            cb = (int)(e >> 8);
            nh = e & 0xFFu;
            imask = reinterpret_cast<const unsigned char*>(stk + (wcap + (sp >> 2)) * BLOCK)[sp & 3];
        } else {
            cb = stk[(2 * sp) * BLOCK];
            const unsigned bits = (unsigned)stk[(2 * sp + 1) * BLOCK];
            imask = bits >> 8;
            nh = bits & 0xFFu;
        }
    }
    const unsigned slot = (unsigned)__builtin_ctz(nh) ^ oct;
    nh &= nh - 1u;
    if (nh) {
        if (sp >= wcap) return -2;
        if constexpr (PK) {
            stk[sp * BLOCK] = (int)(((unsigned)cb << 8) | nh);
            reinterpret_cast<unsigned char*>(stk + (wcap + (sp >> 2)) * BLOCK)[sp & 3] = (unsigned char)imask;
        } else {
            stk[(2 * sp) * BLOCK] = cb;
            stk[(2 * sp + 1) * BLOCK] = (int)((imask << 8) | nh);
        }
        ++sp;
    }
    return cb + __popc(imask & ((1u << slot) - 1u));
}

// wide_next with the stack's top entry cached in registers (PRT_TOP_CACHE): (t0, t1) hold the LDS words of entry sp - 1
// as the previous step left them, read back after every step's stack update, so that a pop takes its entry from
// registers instead of waiting for an LDS read on the chain from this node's loads to the next node's. The read-back
// is unconditional (its result is used only by a later pop, whose wait it has long passed) -- a load under a branch
// merged into loop-carried registers would be waited for at the merge.
#ifndef PRT_TOP_CACHE
#define PRT_TOP_CACHE 0
#endif
constexpr bool TOP_CACHE = PRT_TOP_CACHE != 0;
struct TopC {
    unsigned t0 = 0, t1 = 0;
};
template <bool PK = false>
__device__ __forceinline__ int wide_next_tc(unsigned nh, int cb, unsigned imask, unsigned oct, int& sp, TopC& tc,
                                            int* __restrict__ stk, int wcap = WSTACK) {
    if (!nh) {
        if (sp == 0) return -1;
        --sp;
        if constexpr (PK) {
            cb = (int)(tc.t0 >> 8);
            nh = tc.t0 & 0xFFu;
            imask = tc.t1 & 0xFFu;
        } else {
            cb = (int)tc.t0;
            imask = tc.t1 >> 8;
            nh = tc.t1 & 0xFFu;
        }
    }
    const unsigned slot = (unsigned)__builtin_ctz(nh) ^ oct;
    nh &= nh - 1u;
    if (nh) {
        if (sp >= wcap) return -2;
        if constexpr (PK) {
            stk[sp * BLOCK] = (int)(((unsigned)cb << 8) | nh);
            reinterpret_cast<unsigned char*>(stk + (wcap + (sp >> 2)) * BLOCK)[sp & 3] = (unsigned char)imask;
        } else {
            stk[(2 * sp) * BLOCK] = cb;
            stk[(2 * sp + 1) * BLOCK] = (int)((imask << 8) | nh);
        }
        ++sp;
    }
    return cb + __popc(imask & ((1u << slot) - 1u));
}
// the top entry's read-back (TOP_CACHE), placed after the next node's loads are issued: its LDS waits never delay them
template <bool PK>
__device__ __forceinline__ void top_reload(int sp, TopC& tc, const int* __restrict__ stk, int wcap) {
    if constexpr (TOP_CACHE) {
        const int ti = sp > 0 ? sp - 1 : 0;  // (sp == 0: a word no pop reads)
        if constexpr (PK) {
            tc.t0 = (unsigned)stk[ti * BLOCK];
            tc.t1 = reinterpret_cast<const unsigned char*>(stk + (wcap + (ti >> 2)) * BLOCK)[ti & 3];
        } else {
            tc.t0 = (unsigned)stk[(2 * ti) * BLOCK];
            tc.t1 = (unsigned)stk[(2 * ti + 1) * BLOCK];
        }
    }
}
// the walks' step: wide_next or wide_next_tc (then top_reload after the next node's loads)
template <bool PK>
__device__ __forceinline__ int wide_step_next(unsigned nh, int cb, unsigned imask, unsigned oct, int& sp, TopC& tc,
                                              int* __restrict__ stk, int wcap) {
    if constexpr (TOP_CACHE) return wide_next_tc<PK>(nh, cb, imask, oct, sp, tc, stk, wcap);
    else return wide_next<PK>(nh, cb, imask, oct, sp, stk, wcap);
}

// A wave's LDS queue of packed triangle tests (TQ): TQ_CAP jobs (owner lane << 26 | triangle), then 128 words of
// per-owner results, then the queue's counter. Between packed steps the result words, the job words 64..127 (the
// closest walk's flags) and the counter are 0 (tq_clear): minima are kept complemented, by atomic max.
// A job's triangle (a position in the view's leaf-ordered triangles) has 26 bits: the TQ builds serve scenes of fewer
// than TQ_MAX_TRIS triangles; the host (rt_hip.hip persist_kernel, shp_ok) runs the builds without TQ for larger ones.
constexpr int TQ_CAP = 128;
constexpr int TQ_MAX_TRIS = 1 << 26;
// The shadow walks' triangle tests with the exact reciprocal (rcp_ieee, bit-identical to the IEEE division): same box,
// 20-frame batches, dragon 0.559 -> 0.556 ms per frame, car_boxed 0.811 -> 0.807, sportscar 0.838 -> 0.831
// (profiles/r5e; round 4 had measured the opposite on a kernel that spilled)
#ifndef PRT_SHADOW_RCP
#define PRT_SHADOW_RCP 1
#endif
constexpr bool SHADOW_RCP = PRT_SHADOW_RCP != 0;
static_assert(TQ_MAX_TRIS == 0x3FFFFFF + 1 && 63u << 26 >> 26 == 63u, "job = owner lane (6 bits) << 26 | triangle");
constexpr int TQ_OCC = TQ_CAP, TQ_T = TQ_CAP + 64, TQ_CNT = TQ_CAP + 128, TQ_WORDS = TQ_CAP + 132;
// the waves' queues of a kernel without dynamic LDS (the 3-wave k_persist): a static array
__device__ __forceinline__ int* tq_static() {
    __shared__ int q[BLOCK / 64 * TQ_WORDS];
    return q + (threadIdx.x >> 6) * TQ_WORDS;
}
__device__ __forceinline__ void tq_clear(int* tq) {
    const unsigned lane = threadIdx.x & 63u;
    tq[64 + lane] = 0;
    tq[TQ_OCC + lane] = 0;
    tq[TQ_T + lane] = 0;
    if (lane == 0u) tq[TQ_CNT] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}
// a step packs its triangle tests when some lane holds at least TQ_MIN of them (the per-lane loop would run that many
// rounds; a packed round costs about 1.5 of them). Same box, dragon 20-frame batches: TQ_MIN 2 / 3 / 4 = 0.573 /
// 0.575 / 0.579 ms per frame.
#ifndef PRT_TQ_MIN
#define PRT_TQ_MIN 2
#endif
constexpr unsigned TQ_MIN = PRT_TQ_MIN;

// The closest walk's packed triangle tests (TQ): the lanes active in this step test the step's (owner, triangle)
// pairs, one each (single round: at most as many pairs as active lanes), with the owner's ray fetched by
// ds_bpermute. The results go back through the owner's LDS slots: the least (t, triangle) key by a 64-bit LDS
// atomic max of its complement, then the winner's side (nd) and a tie flag (another pair with the same t) in one flag word. The owner
// then applies the sequential loop's rule to the step's minimum m: m < best takes it (tie iff two pairs hit at m),
// m == best (a hit) marks a tie -- the state the per-lane loop would leave, which is what the strict re-walk of a
// tie relies on. Returns false when the step's pairs do not fit one round (the caller runs the loop).
template <bool COUNT>
__device__ __forceinline__ bool closest_tris_packed(const DWide& W, v3 o, v3 d, unsigned th, int tb, float& best,
                                                    int& hp, int& nd, bool& tie, int* tq, Ctr& c) {
    const unsigned lane = threadIdx.x & 63u;
    const unsigned long long ex = __builtin_amdgcn_read_exec();
    const unsigned na = (unsigned)__builtin_popcountll(ex);
    const unsigned rk = __builtin_amdgcn_mbcnt_hi((unsigned)(ex >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)ex, 0u));
    unsigned* cnt = reinterpret_cast<unsigned*>(tq + TQ_CNT);
    const unsigned nt = (unsigned)__builtin_popcount(th);
    unsigned pos = 0u;
    if (nt) pos = atomicAdd(cnt, nt);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const unsigned T = (unsigned)__builtin_amdgcn_readfirstlane((int)atomicAdd(cnt, 0u));
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (rk == 0u) *cnt = 0u;
    if (T > na) return false;
    for (unsigned m = th; m; m &= m - 1u) tq[pos++] = (int)((lane << 26) | (unsigned)(tb + __builtin_ctz(m)));
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const bool has = rk < T;
    const unsigned job = has ? (unsigned)tq[rk] : lane << 26;
    const int ow = (int)(job >> 26);
    const v3 oo = mk(__shfl(o.x, ow, 64), __shfl(o.y, ow, 64), __shfl(o.z, ow, 64));
    const v3 dd = mk(__shfl(d.x, ow, 64), __shfl(d.y, ow, 64), __shfl(d.z, ow, 64));
    unsigned long long* key = reinterpret_cast<unsigned long long*>(tq + TQ_OCC);  // complemented keys, 0 = none
    unsigned* flag = reinterpret_cast<unsigned*>(tq + 64);  // (the job words 64..127: free in a single round)
    const unsigned tri = job & 0x3FFFFFFu;
    float tt = FMAX;
    int k = 0;
    if (has) {
        PRT_TRI_ITER(c, q1);
        tt = hit_triangle<true>(oo, dd, W.tris + 3 * (int)tri, k);
        if (COUNT) c.cht++;
        if (tt < FMAX) atomicMax(key + ow, ~(((unsigned long long)__float_as_uint(tt) << 32) | tri));
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (has && tt < FMAX) {
        const unsigned long long kw = ~key[ow];
        if ((unsigned)(kw >> 32) == __float_as_uint(tt)) atomicOr(flag + ow, (unsigned)kw == tri ? (unsigned)k : 2u);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (nt) {
        const unsigned long long kc = key[lane];
        const unsigned fl = flag[lane];
        // (zeroed through an opaque 32-bit zero: a 64-bit constant pair is one the register allocator spills rather
        // than rematerialises, and its reload waits for the next node's load)
        const int z = opaque(0);
        reinterpret_cast<int*>(key + lane)[0] = z;
        reinterpret_cast<int*>(key + lane)[1] = z;
        flag[lane] = z;
        const unsigned long long kw = ~kc;
        const float mt = __uint_as_float((unsigned)(kw >> 32));
        if (kc != 0ull) {
            if (mt < best) {
                best = mt;
                hp = (int)(unsigned)kw;
                nd = (int)(fl & 1u);
                tie = (fl & 2u) != 0u;
            } else if (mt == best) {
                tie = true;
            }
        }
    }
    return true;
}

// The shadow walks' packed triangle tests (TQ), as closest_tris_packed: a pair occludes the owner's ray when its
// triangle is hit nearer than the light (the reference's per-triangle test, bvh.c:283-290); the nearest hit (for the
// walk's box pruning) goes back complemented by atomic max.
template <bool COUNT>
__device__ __forceinline__ bool shadow_tris_packed(const DWide& W, v3 o, v3 d, float ld2, unsigned th, int tb,
                                                   float& best, bool& occ, int* tq, Ctr& c) {
    const unsigned lane = threadIdx.x & 63u;
    const unsigned long long ex = __builtin_amdgcn_read_exec();
    const unsigned na = (unsigned)__builtin_popcountll(ex);
    const unsigned rk = __builtin_amdgcn_mbcnt_hi((unsigned)(ex >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)ex, 0u));
    unsigned* cnt = reinterpret_cast<unsigned*>(tq + TQ_CNT);
    const unsigned nt = (unsigned)__builtin_popcount(th);
    unsigned pos = 0u;
    if (nt) pos = atomicAdd(cnt, nt);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const unsigned T = (unsigned)__builtin_amdgcn_readfirstlane((int)atomicAdd(cnt, 0u));
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (rk == 0u) *cnt = 0u;
    if (T > na) return false;
    for (unsigned m = th; m; m &= m - 1u) tq[pos++] = (int)((lane << 26) | (unsigned)(tb + __builtin_ctz(m)));
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const bool has = rk < T;
    const unsigned job = has ? (unsigned)tq[rk] : lane << 26;
    const int ow = (int)(job >> 26);
    const v3 oo = mk(__shfl(o.x, ow, 64), __shfl(o.y, ow, 64), __shfl(o.z, ow, 64));
    const v3 dd = mk(__shfl(d.x, ow, 64), __shfl(d.y, ow, 64), __shfl(d.z, ow, 64));
    const float l2 = __shfl(ld2, ow, 64);
    if (has) {
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
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (nt) {
        occ = tq[TQ_OCC + lane] != 0;
        const unsigned tc = (unsigned)tq[TQ_T + lane];
        if (tc) best = fminf(best, __uint_as_float(~tc));
        tq[TQ_OCC + lane] = 0;
        tq[TQ_T + lane] = 0;
    }
    return true;
}

// PIPE: software-pipeline the leaf triangles (the next triangle's loads issued before this one's test);
// pays where registers allow (the split kernels), not in k_persist (spills at its 168-VGPR cap).
// TQ: a step whose lanes hold 3+ triangles tests them packed (closest_tris_packed; tq: the wave's queue).
template <bool COUNT, bool PIPE = false, bool PK = false, bool TQ = false>
__device__ __forceinline__ void closest_wide(const DWide& W, v3 o, v3 d, float& best, int& hp, int& nd, bool& tie,
                                             int* __restrict__ stk, Ctr& c, int wcap = WSTACK, int* tq = nullptr,
                                             const float4* top = nullptr) {
    const RayPre p = ray_pre_closest(o, d);
    const unsigned oct = (p.ix < 0.0f ? 1u : 0u) | (p.iy < 0.0f ? 2u : 0u) | (p.iz < 0.0f ? 4u : 0u);
    int sp = 0;
    TopC tc;
    const gnodes nbase = walk_base(W.nodes);
    WNode N = wload_at(nbase, 0, top);
    for (;;) {
        unsigned nh, th, imask, nl;
        int cb, tb;
        pin_node(N);
        wide_node<COUNT, LATE_TRIS, CLOSEST_CLAMP ? 2 : 0>(N, p, oct, closest_lim(best), nh, th, cb, tb, imask, nl);
        const unsigned m0 = __float_as_uint(N.f1.z), m1 = __float_as_uint(N.f1.w);
        const int next = wide_step_next<PK>(nh, cb, imask, oct, sp, tc, stk, wcap);
        // the next node's loads go out before this node's triangle tests, unconditionally (a walk that has ended
        // reloads the root): a load under a branch is copied into the merged register right after it, and that
        // copy waits for the load (dragon 0.712 -> 0.689 ms per frame, sportscar 0.931 -> 0.901, car_boxed 0.870 -> 0.858)
        N = wload_at(nbase, next >= 0 ? next : 0, top);
        top_reload<PK>(sp, tc, stk, wcap);
        if constexpr (LATE_TRIS) th = leaf_tris<COUNT>(th, m0, m1, nl);
        if (COUNT) {
            c.chi++;
            c.chl += nl;
            c.nb += 10;
            count_step(c, false);
        }
        if constexpr (TQ) {
            if (__builtin_amdgcn_readfirstlane((int)(__ballot(__builtin_popcount(th) >= TQ_MIN) != 0ull)) &&
                closest_tris_packed<COUNT>(W, o, d, th, tb, best, hp, nd, tie, tq, c))
                th = 0u;
        }
        if (!PIPE) {
            while (th) {
                PRT_TRI_ITER(c, q1);
                const int i = tb + __builtin_ctz(th);
                th &= th - 1u;
                int k;
                const float tt = hit_triangle<true>(o, d, W.tris + 3 * i, k);
                if (COUNT) c.cht++;
                if (tt < best) {
                    best = tt;
                    nd = k;
                    hp = i;
                    tie = false;
                } else if (tt == best && tt != FMAX) {
                    tie = true;
                }
            }
        }
        if (PIPE && th) {  // the next triangle's loads go out before this one's test
            int i = tb + __builtin_ctz(th);
            th &= th - 1u;
            float4 ta = W.tris[3 * i], tb4 = W.tris[3 * i + 1], tc = W.tris[3 * i + 2];
            for (;;) {
                const bool more = th != 0u;
                int i2 = 0;
                float4 na = ta, nb = tb4, nc = tc;
                if (more) {
                    i2 = tb + __builtin_ctz(th);
                    th &= th - 1u;
                    na = W.tris[3 * i2];
                    nb = W.tris[3 * i2 + 1];
                    nc = W.tris[3 * i2 + 2];
                }
                int k;
                const float tt = hit_triangle_v(o, d, ta, tb4, tc, k);
                if (COUNT) c.cht++;
                if (tt < best) {
                    best = tt;
                    nd = k;
                    hp = i;
                    tie = false;
                } else if (tt == best && tt != FMAX) {
                    tie = true;
                }
                if (!more) break;
                i = i2;
                ta = na;
                tb4 = nb;
                tc = nc;
            }
        }
        if (next < 0) {
            if (next == -2) CTR_INC(c, err, C_ERR);
            break;
        }
    }
}

template <bool COUNT, bool PIPE = false, bool PK = false, bool TQ = false>
__device__ __forceinline__ bool visible_wide(const DWide& W, v3 o, v3 d, float ld2, int* __restrict__ stk, Ctr& c,
                                             int wcap = WSTACK, int* tq = nullptr, const float4* top = nullptr) {
    const float reach = shadow_reach(o, ld2);
    const RayPre p = ray_pre_shadow(o, d, reach);
    const unsigned oct = (p.ix < 0.0f ? 1u : 0u) | (p.iy < 0.0f ? 2u : 0u) | (p.iz < 0.0f ? 4u : 0u);
    float best = FMAX;
    int sp = 0;
    TopC tc;
    const gnodes nbase = walk_base(W.nodes);
    WNode N = wload_at(nbase, 0, top);
    for (;;) {
        unsigned nh, th, imask, nl;
        int cb, tb;
        pin_node(N);
        wide_node<COUNT, LATE_TRIS, SHADOW_CLAMP ? 1 : 0>(N, p, oct, fminf(best * PRUNE_SLACK, reach), nh, th, cb, tb, imask,
                                                  nl, SHADOW_ORDER_XOR);
        const unsigned m0 = __float_as_uint(N.f1.z), m1 = __float_as_uint(N.f1.w);
        const int next = wide_step_next<PK>(nh, cb, imask, oct ^ SHADOW_ORDER_XOR, sp, tc, stk, wcap);
        N = wload_at(nbase, next >= 0 ? next : 0, top);  // unconditional (closest_wide)
        top_reload<PK>(sp, tc, stk, wcap);
        if constexpr (LATE_TRIS) th = leaf_tris<COUNT>(th, m0, m1, nl);
        if (COUNT) {
            c.shi++;
            c.shl += nl;
            c.nb += 10;
            count_step(c, true);
        }
        if constexpr (TQ) {
            bool occ = false;
            if (__builtin_amdgcn_readfirstlane((int)(__ballot(__builtin_popcount(th) >= TQ_MIN) != 0ull)) &&
                shadow_tris_packed<COUNT>(W, o, d, ld2, th, tb, best, occ, tq, c)) {
                if (occ) return false;
                th = 0u;
            }
        }
        if (!PIPE) {
            while (th) {
                PRT_TRI_ITER(c, q2);
                const int i = tb + __builtin_ctz(th);
                th &= th - 1u;
                int k;
                const float tt = hit_triangle<SHADOW_RCP>(o, d, W.tris + 3 * i, k);
                if (COUNT) c.sht++;
                if (tt < best) {
                    best = tt;
                    const v3 ip = add(o, mul(d, best));
                    const v3 oi = sub(o, ip);
                    if (ld2 > dot(oi, oi)) return false;
                }
            }
        }
        if (PIPE && th) {  // software-pipelined as in closest_wide
            int i = tb + __builtin_ctz(th);
            th &= th - 1u;
            float4 ta = W.tris[3 * i], tb4 = W.tris[3 * i + 1], tc = W.tris[3 * i + 2];
            for (;;) {
                const bool more = th != 0u;
                float4 na = ta, nb = tb4, nc = tc;
                if (more) {
                    const int i2 = tb + __builtin_ctz(th);
                    th &= th - 1u;
                    na = W.tris[3 * i2];
                    nb = W.tris[3 * i2 + 1];
                    nc = W.tris[3 * i2 + 2];
                }
                int k;
                const float tt = hit_triangle_v(o, d, ta, tb4, tc, k);
                if (COUNT) c.sht++;
                if (tt < best) {
                    best = tt;
                    const v3 ip = add(o, mul(d, best));
                    const v3 oi = sub(o, ip);
                    if (ld2 > dot(oi, oi)) return false;
                }
                if (!more) break;
                ta = na;
                tb4 = nb;
                tc = nc;
            }
        }
        if (next < 0) {
            if (next == -2) CTR_INC(c, err, C_ERR);
            break;
        }
    }
    return true;
}

// The fast walk's wide view for a ray: the unit-direction view (a superset of every triangle such a ray can hit)
// for reflection and shadow rays; for primary rays (unnormalised directions, main.c:229-233) the primary view when
// the host found this launch's directions short enough for it, else the full one
__device__ __forceinline__ const DWide& wide_for(const DScene& s, bool unit) {
    if (unit) return s.unit.nodes ? s.unit : s.wide;
    return s.prim.nodes ? s.prim : s.wide;
}

// An exact tie (two triangles at the least t, tmin) is resolved by the reference's own walk (bvh_traverse: the first
// triangle it meets at tmin wins), started with best = tie_bound(tmin) instead of FLT_MAX. That walk visits the nodes
// the full walk visits in the same order, except subtrees entered at or beyond the bound; those hold no triangle
// at tmin (a box's computed entry exceeds a triangle's computed t inside it by rounding only: ~1e-7 of the
// coordinates, against a bound (tmin + max|o|) * 2^-10 past tmin). Triangles it accepts below the bound before
// reaching tmin make its best equal the full walk's best from then on. So it meets the same first triangle at tmin
// -- and, from the bound on, visits only a short prefix of the ray. Nothing found (never expected): the full walk.
// Same box (profiles/r5j): the re-walks cost car_boxed 2.3 % of its batch time and a third of its single frames.
#ifndef PRT_TIE_BOUNDED
#define PRT_TIE_BOUNDED 1
#endif
constexpr bool TIE_BOUNDED = PRT_TIE_BOUNDED != 0;
#ifndef PRT_TIE_CUT
#define PRT_TIE_CUT 1
#endif
constexpr bool TIE_CUT = PRT_TIE_CUT != 0;
__device__ __forceinline__ float tie_bound(v3 o, float tmin) {
    const float om = fmaxf(fmaxf(__builtin_fabsf(o.x), __builtin_fabsf(o.y)), __builtin_fabsf(o.z));
    return tmin + (tmin + om) * 0x1p-10f;
}

// Closest hit with the kernel's policy; returns the ORIGINAL triangle index (-1 = miss).
// sstk (nullable): the binary walks' stack when the wide walk's `stk` holds only wcap entries (DYN kernels)
// unit: d has unit length (a reflection ray): the unit-direction view serves the fast walk
template <bool STRICT, bool COUNT, bool REG = true, bool PIPE = false, bool PK = false, bool TQ = false>
__device__ __forceinline__ int closest(const DScene& s, v3 o, v3 d, float& best, int& nd, int* __restrict__ stk,
                                       Ctr& c, int* __restrict__ sstk = nullptr, int wcap = WSTACK, bool unit = false,
                                       int* tq = nullptr) {
    int* __restrict__ bstk = sstk ? sstk : stk;
    int hp = -1;
    bool tie = false;
    best = FMAX;
    nd = 0;
    // a degenerate ray whose origin lies on a face: the fast walk, then its winner's reference path checked (chk)
    const bool face = degenerate(d) && !degenerate_ok(s, o, d);
    const bool chk = face && s.ref_path != nullptr && o.x == o.x && o.y == o.y && o.z == o.z;
    if (!STRICT && (!face || chk)) {
        bool done = false;  // the fast walk's answer stands
        int orig = -1;
        if (s.wide.nodes) {
            const DWide& W = wide_for(s, unit);
            closest_wide<COUNT, PIPE, PK, TQ>(W, o, d, best, hp, nd, tie, stk, c, wcap, tq, c.top[unit ? 1 : 0]);
            if (!tie) {
                orig = hp >= 0 ? W.tri_orig[hp] : -1;
                done = true;
            }
        } else {
            closest_walk<false, COUNT, REG>(s.acc, o, d, best, hp, nd, tie, bstk, c);
            if (!tie) {
                orig = hp >= 0 ? s.acc.tri_orig[hp] : -1;
                done = true;
            }
        }
        if (done && (!chk || orig < 0 || ref_reaches(s, orig, o, d))) return orig;
        CTR_INC(c, fb, C_FALLBACK);
        if (TIE_BOUNDED && !done) {  // an exact tie at t = best: the reference walk bounded just past it (tie_bound),
                                     // and cut as far before it (boxes the ray leaves before then hold nothing it
                                     // could take)
            const float tb = tie_bound(o, best), cut = best - (tb - best);
            hp = -1;
            nd = 0;
            best = tb;
            closest_walk<true, COUNT, REG, TIE_CUT>(s.ref, o, d, best, hp, nd, tie, bstk, c, cut);
            if (hp >= 0) return s.ref.tri_orig[hp];
        }
        hp = -1;
        best = FMAX;
        nd = 0;
    } else if (!STRICT) {
        CTR_INC(c, fb, C_FALLBACK);
    }
    closest_walk<true, COUNT, REG>(s.ref, o, d, best, hp, nd, tie, bstk, c);
    return hp >= 0 ? s.ref.tri_orig[hp] : -1;
}

template <bool STRICT, bool COUNT, bool REG = true, bool PIPE = false, bool PK = false, bool TQ = false>
__device__ __forceinline__ bool visible(const DScene& s, v3 o, v3 d, float ld2, int* __restrict__ stk, Ctr& c,
                                        int* __restrict__ sstk = nullptr, int wcap = WSTACK, int* tq = nullptr) {
    int* __restrict__ bstk = sstk ? sstk : stk;
    if (!STRICT && (!degenerate(d) || degenerate_ok(s, o, d))) {
        if (s.wide.nodes)  // |d| = 1
            return visible_wide<COUNT, PIPE, PK, TQ>(wide_for(s, true), o, d, ld2, stk, c, wcap, tq, c.top[1]);
        return visible_walk<false, COUNT, REG>(s.acc, o, d, ld2, bstk, c);
    }
    if (!STRICT) CTR_INC(c, fb, C_FALLBACK);
    return visible_walk<true, COUNT, REG>(s.ref, o, d, ld2, bstk, c);
}

// group-cooperative walks (rt_coop.hpp): G lanes per ray
template <int G, bool COUNT>
__device__ __forceinline__ int closest_g(const DScene& s, v3 o, v3 d, float& best, int& nd, int* __restrict__ stk,
                                         Ctr& c, unsigned q, bool unit);
template <int G, bool COUNT>
__device__ __forceinline__ bool visible_g(const DScene& s, v3 o, v3 d, float ld2, int* __restrict__ stk, Ctr& c,
                                          unsigned q);

// ---------------------------------------------------------------- one path (raytrace, iterative)
template <int MAXB>
__device__ __forceinline__ void set3(v3 (&a)[MAXB], int i, v3 v) {
#pragma unroll
    for (int k = 0; k < MAXB; k++)
        if (k == i) a[k] = v;
}
template <int MAXB>
__device__ __forceinline__ void set_u(unsigned (&a)[MAXB], int i, unsigned v) {
#pragma unroll
    for (int k = 0; k < MAXB; k++)
        if (k == i) a[k] = v;
}
template <int MAXB>
__device__ __forceinline__ unsigned get_u(const unsigned (&a)[MAXB], int i) {
    unsigned r = 0;
#pragma unroll
    for (int k = 0; k < MAXB; k++)
        if (k == i) r = a[k];
    return r;
}
template <int MAXB>
__device__ __forceinline__ void seti(int (&a)[MAXB], int i, int v) {
#pragma unroll
    for (int k = 0; k < MAXB; k++)
        if (k == i) a[k] = v;
}

// One level of the reference recursion (raytracer.c:101-177) for a path whose ray at level `it` is
// (o, d): closest hit, Lambert/Blinn with one shadow ray per light, reflection. Stores the level's
// colour and material; returns true when the path ends (L = levels kept, tail = the reference's
// raytrace(.., BOUNCES) returned {0,0,0}), otherwise leaves the reflection ray in (o, d).
// G > 1: the traversals are group-cooperative (rt_coop.hpp), q = the lane's place in its group.
// PB: the level's colour and material go to this lane's path buffer slot pb[it * 64] instead of the
// register arrays (cold values: written once per level, read once by the fold), which frees 4 * MAXB
// registers across the walks for the kernels with the tightest register budget.
// PK / TQ: packed stack entries and packed triangle tests (the SHP = 3 build of PERSIST4; tq: the wave's queue)
template <int MAXB, bool STRICT, bool COUNT, bool REG, int G = 1, bool PB = false, bool PK = false, bool TQ = false>
__device__ __forceinline__ bool path_step(const DScene& s, int bounces, int it, v3& o, v3& d, v3 (&cols)[MAXB],
                                          int (&mats)[MAXB], int& L, bool& tail, int& hit0, float& t0,
                                          int* __restrict__ bh, int bh_pix, int* __restrict__ stk, Ctr& c,
                                          unsigned q = 0, float4* __restrict__ pb = nullptr,
                                          int* __restrict__ sstk = nullptr, int wcap = WSTACK, int* tq = nullptr) {
    const v3 amb = mk(s.amb_x, s.amb_y, s.amb_z);
    float best;
    int nd;
    if (COUNT) c.lvl = (unsigned)it;
    if (it == 0) CTR_INC(c, prim, C_PRIM);
    else CTR_INC(c, refl, C_REFL);
    int orig;
    if constexpr (G > 1) orig = closest_g<G, COUNT>(s, o, d, best, nd, stk, c, q, it > 0);
    else orig = closest<STRICT, COUNT, REG, false, PK, TQ>(s, o, d, best, nd, stk, c, sstk, wcap, it > 0, tq);  // it > 0: |d| = 1
    if (it == 0) {
        hit0 = orig;
        t0 = best;
    }
    if (bh && bh_pix >= 0) bh[(size_t)opaque(bh_pix) * bounces + it] = orig;  // per-level dump (uniform base, nullable)
    if (orig < 0) {  // raytracer.c:132-135
        if constexpr (PB) pb[it * 64] = make_float4(0.0f + amb.x, 0.0f + amb.y, 0.0f + amb.z, __int_as_float(0));
        else set3<MAXB>(cols, it, mk(0.0f + amb.x, 0.0f + amb.y, 0.0f + amb.z));
        L = it + 1;
        tail = false;
        return true;
    }
    CTR_INC(c, hits, C_HITS);
    const v3 ip = add(o, mul(d, best));  // raytracer.c:137-138
    const float4 sh0 = s.shade[2 * orig], sh1 = s.shade[2 * orig + 1];
    const int m = __float_as_int(sh0.w);
    const v3 n = nd ? xyz(sh1) : xyz(sh0);
    const v3 kd0 = xyz(s.mats[3 * m + 1]);
    v3 col = mk(0.0f + kd0.x * amb.x, 0.0f + kd0.y * amb.y, 0.0f + kd0.z * amb.z);  // :144-146
    const v3 v = mul(d, -1.0f);                                                      // :147
    for (int j = 0; j < s.n_lights; ++j) {                                           // :149-160
        // the shadow ray first (light_v, raytracer.c:62-99), then the Lambert/Blinn terms: the same
        // values (pure functions of ip, n, d, the material and the light), fewer of them live across the walk
        const v3 Lp = xyz(s.lights[2 * j]);
        v3 l = sub(Lp, ip);
        float mg = mag(l);
        l = dvs(l, mg);
        mg *= mg;
        const v3 tmp = sub(ip, Lp), tmp2 = sub(Lp, ip);
        const float ld2 = dot(tmp, tmp);
        int V;
        if (dot(tmp2, n) < 0) {
            V = 0;
            CTR_INC(c, skip, C_SKIP);
        } else {
            CTR_INC(c, shad, C_SHAD);
            if constexpr (G > 1) V = visible_g<G, COUNT>(s, ip, l, ld2, stk, c, q) ? 1 : 0;
            else V = visible<STRICT, COUNT, REG, false, PK, TQ>(s, ip, l, ld2, stk, c, sstk, wcap, tq) ? 1 : 0;
        }
        const v3 kl = xyz(s.lights[2 * j + 1]);
        const v3 ks = xyz(s.mats[3 * m]), kd = xyz(s.mats[3 * m + 1]);
        const float ndl = dot(n, l);
        const v3 h = normalize(add(l, v));  // lambert_blinn, raytracer.c:21-33
        const float coeff = fmaxf(0.0f, dot(n, h));
        const v3 cr = mk(kd.x * fmaxf(0.0f, ndl) + ks.x * coeff, kd.y * fmaxf(0.0f, ndl) + ks.y * coeff,
                         kd.z * fmaxf(0.0f, ndl) + ks.z * coeff);
        const float fV = (float)V;
        col.x = col.x + fV * kl.x * cr.x / mg;
        col.y = col.y + fV * kl.y * cr.y / mg;
        col.z = col.z + fV * kl.z * cr.z / mg;
    }
    const v3 dd = mul(v, -1.0f);  // raytracer.c:163-166
    const v3 ns = mul(n, 2.0f * __builtin_fabsf(dot(dd, n)));
    const v3 r = normalize(add(dd, ns));
    if constexpr (PB) {
        pb[it * 64] = make_float4(col.x, col.y, col.z, __int_as_float(m));
    } else {
        set3<MAXB>(cols, it, col);
        seti<MAXB>(mats, it, m);
    }
    const v3 kr = xyz(s.mats[3 * m + 2]);
    if (!(mag(kr) > 0.0f)) {  // raytracer.c:168
        L = it + 1;
        tail = false;
        return true;
    }
    if (it + 1 == bounces) {  // raytrace(.., BOUNCES) returns {0,0,0}: col += kr * 0
        L = it + 1;
        tail = true;
        return true;
    }
    o = ip;
    d = r;
    return false;
}

// fold: R_i = c_i + kr_i * R_{i+1}, deepest level first (raytracer.c:169-172)
template <int MAXB>
__device__ __forceinline__ v3 fold_path(const DScene& s, const v3 (&cols)[MAXB], const int (&mats)[MAXB], int L,
                                        bool tail) {
    v3 acc = mk(0.0f, 0.0f, 0.0f);
    bool have = false;
#pragma unroll
    for (int i = MAXB - 1; i >= 0; --i) {
        if (i < L) {
            if (!have) {
                acc = cols[i];
                if (tail) {
                    const v3 kr = xyz(s.mats[3 * mats[i] + 2]);
                    acc = mk(acc.x + kr.x * 0.0f, acc.y + kr.y * 0.0f, acc.z + kr.z * 0.0f);
                }
                have = true;
            } else {
                const v3 kr = xyz(s.mats[3 * mats[i] + 2]);
                acc = mk(cols[i].x + kr.x * acc.x, cols[i].y + kr.y * acc.y, cols[i].z + kr.z * acc.z);
            }
        }
    }
    return acc;
}

// fold_path over a path buffer (PB kernels): the same sums in the same order
template <int MAXB>
__device__ __forceinline__ v3 fold_pb(const DScene& s, const float4* __restrict__ pb, int L, bool tail) {
    v3 acc = mk(0.0f, 0.0f, 0.0f);
    bool have = false;
#pragma unroll
    for (int i = MAXB - 1; i >= 0; --i) {
        if (i < L) {
            const float4 e = pb[i * 64];
            const v3 ci = mk(e.x, e.y, e.z);
            const v3 kr = xyz(s.mats[3 * __float_as_int(e.w) + 2]);
            if (!have) {
                acc = ci;
                if (tail) acc = mk(acc.x + kr.x * 0.0f, acc.y + kr.y * 0.0f, acc.z + kr.z * 0.0f);
                have = true;
            } else {
                acc = mk(ci.x + kr.x * acc.x, ci.y + kr.y * acc.y, ci.z + kr.z * acc.z);
            }
        }
    }
    return acc;
}

// PB: 0 = levels in registers, 1 = path buffer in global memory (A.pathbuf), 2 = path buffer in dynamic LDS
// after the DYN wide stack (2 * wcap ints per lane): [wave][level][lane] float4, the L2 left to the scene
// (PK / TQ: after the path buffer, the waves' packed-triangle queues)
template <int MAXB, bool STRICT, bool COUNT, bool REG = true, int G = 1, int PB = 0, bool PK = false, bool TQ = false>
__device__ v3 trace_path(const KArgs& A, v3 o, v3 d, int* __restrict__ stk, Ctr& c, int& hit0, float& t0, int bh_pix,
                         unsigned q = 0, int* __restrict__ sstk = nullptr, int wcap = WSTACK) {
    v3 cols[MAXB];
    int mats[MAXB];
    float4* pb = nullptr;
    int* tq = nullptr;
    if constexpr (PB == 2) {
        extern __shared__ int lds_dyn[];
        float4* pb0 = (float4*)(lds_dyn + wstack_words(wcap, PK) * BLOCK);
        pb = pb0 + (size_t)((threadIdx.x >> 6) * MAXB) * 64 + (threadIdx.x & 63);
        if constexpr (TQ) tq = (int*)(pb0 + (size_t)BLOCK * MAXB) + (threadIdx.x >> 6) * TQ_WORDS;
    } else if constexpr (TQ) {  // (PB 0 / 1: the kernel's static queues)
        tq = tq_static();
    } else if constexpr (PB) {  // [wave][level][lane] (persistent grids: a wave's slot is its own for the launch)
        pb = A.pathbuf + ((size_t)(blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6)) * MAXB) * 64 + (threadIdx.x & 63);
    } else {
#pragma unroll
        for (int k = 0; k < MAXB; k++) {
            cols[k] = mk(0.0f, 0.0f, 0.0f);
            mats[k] = 0;
        }
    }
    int L = 0;
    bool tail = false;
    for (int it = 0; it < A.bounces; ++it) {
        if (path_step<MAXB, STRICT, COUNT, REG, G, PB != 0, PK, TQ>(A.s, A.bounces, it, o, d, cols, mats, L, tail, hit0,
                                                                t0, A.bounce_hit, bh_pix, stk, c, q, pb, sstk, wcap, tq))
            break;
    }
    if constexpr (PB != 0) return fold_pb<MAXB>(A.s, pb, L, tail);
    else return fold_path<MAXB>(A.s, cols, mats, L, tail);
}

__device__ __forceinline__ v3 clamp01(v3 c) {  // vec_constrain(col, 0, 1), vec.c:47-54
    return mk(fminf(fmaxf(c.x, 0.0f), 1.0f), fminf(fmaxf(c.y, 0.0f), 1.0f), fminf(fmaxf(c.z, 0.0f), 1.0f));
}

// image row of compact output row k (rt_frame: rows in blocks of row_block, blocks row_stride apart)
// (frame f of a batch with frame_shift: rows start at (row_offset + f * frame_shift) % row_stride)
__device__ __forceinline__ int image_row(const KArgs& A, int k, int frame = 0) {
    const int off = A.frame_shift ? (A.row_offset + frame * A.frame_shift) % A.row_stride : A.row_offset;
    return off + (k / A.row_block) * A.row_stride + k % A.row_block;
}

// one frame's camera constants (main.c:243-250)
struct Cam {
    v3 pos, ul, ix, iy;
};
// frame f of a batch (A.cams; BATCH kernels), or the launch's single camera (kernel arguments: a
// camera read from memory stays live in registers across the spp loop and costs the single-frame
// kernels spills, so they never read A.cams)
template <bool BATCH = false>
__device__ __forceinline__ Cam cam_of(const KArgs& A, int f) {
    if (!BATCH || !A.cams) return Cam{mk(A.pos[0], A.pos[1], A.pos[2]), mk(A.ul[0], A.ul[1], A.ul[2]),
                                      mk(A.ix[0], A.ix[1], A.ix[2]), mk(A.iy[0], A.iy[1], A.iy[2])};
    // f is wave-uniform: three vector loads, then every value moved to a scalar register (readfirstlane),
    // so the camera costs no vector registers while it stays live across the spp loop
    const float4* c4 = reinterpret_cast<const float4*>(A.cams) + 3 * f;
    const float4 a = c4[0], b = c4[1], e = c4[2];
    float c[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, e.x, e.y, e.z, e.w};
#pragma unroll
    for (int i = 0; i < 12; i++) c[i] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(c[i])));
    return Cam{mk(c[0], c[1], c[2]), mk(c[3], c[4], c[5]), mk(c[6], c[7], c[8]), mk(c[9], c[10], c[11])};
}
// primary direction, main.c:229-233: ((ul - pos) + inc_x * x) + inc_y * y
__device__ __forceinline__ v3 primary_dir(const Cam& C, float fx, float fy) {
    v3 d = sub(C.ul, C.pos);
    d = add(d, mul(C.ix, fx));
    d = add(d, mul(C.iy, fy));
    return d;
}
__device__ __forceinline__ v3 primary_dir(const KArgs& A, float fx, float fy) {
    return primary_dir(cam_of(A, 0), fx, fy);
}
// The same inside a multi-sample loop: the wave-uniform camera re-read from its scalar registers at every sample
// (an empty asm the compiler cannot look through), so that ul - pos, a loop invariant it would otherwise hoist into
// vector registers live across every sample's path, is formed per sample
__device__ __forceinline__ v3 primary_dir_sample(const Cam& C, float fx, float fy) {
    float p[12] = {C.pos.x, C.pos.y, C.pos.z, C.ul.x, C.ul.y, C.ul.z, C.ix.x, C.ix.y, C.ix.z, C.iy.x, C.iy.y, C.iy.z};
#pragma unroll
    for (int i = 0; i < 12; i++) __asm__ volatile("" : "+s"(p[i]));
    return primary_dir(Cam{mk(p[0], p[1], p[2]), mk(p[3], p[4], p[5]), mk(p[6], p[7], p[8]), mk(p[9], p[10], p[11])},
                       fx, fy);
}
// The lane's index in its wave, computed where it is used (v_mbcnt in an asm the compiler cannot hoist or keep): in the
// 4-wave kernels every register held across the walks costs a spill, and this one is two instructions to remake.
__device__ __forceinline__ unsigned lane_now() {
    unsigned l;
    __asm__ volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
// a lane's A.lanebuf slot ([block][lane]): the wave's slots from scalar registers, the lane's offset remade per use
template <bool LDS = false>
__device__ __forceinline__ float4* lane_slot(const KArgs& A) {
    const unsigned wave = (unsigned)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if constexpr (LDS) {  // (the PB = 2 kernels: the launch's slots after its LDS layout, KArgs::slot_off)
        extern __shared__ int lds_dyn[];
        return reinterpret_cast<float4*>(lds_dyn + A.slot_off) + wave * 64u + lane_now();
    }
    const unsigned gw = (unsigned)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * (BLOCK / 64))) + wave;
    return reinterpret_cast<float4*>(reinterpret_cast<char*>(A.lanebuf + (size_t)gw * 64) + lane_now() * 16u);
}

// the shadow-pool kernels' pixel (rt_shpool.hpp, RT_VARIANT_SHPOOL): every lane of the wave calls it
struct UCtr;
template <int MAXB, bool COUNT, bool SPP1, int SHP>
__device__ __forceinline__ void render_pixel_shp(const KArgs& A, const Cam& C, int frame, int x, int k, bool valid,
                                                 int* __restrict__ stk, Ctr& c, UCtr& u, int* __restrict__ sstk,
                                                 int wcap);
__device__ __forceinline__ void flush_u(const UCtr& u, unsigned long long* g);

// Pixel (x, compact row k) of frame `frame` of the launch (outputs at frame * frame_px).
// SPPM: 0 = either (the launch's spp decides at run time), 1 = a build for spp = 1 only (the stratified-sample loop
// compiled out, fewer live values around the path), 2 = a build for spp > 1 only (the corner ray compiled out: one
// inlined path; the host runs the SPPM = 1 builds for spp = 1). With A.lanebuf the running sum of a multi-sample pixel
// lives in the lane's slot of it across the samples, not in registers.
template <int MAXB, bool STRICT, bool COUNT, bool REG = true, int G = 1, int PB = 0, int SPPM = 0,
          bool TQ = false, bool PK = TQ>
__device__ __forceinline__ void render_pixel(const KArgs& A, const Cam& C, int frame, int x, int k,
                                             int* __restrict__ stk, Ctr& c, unsigned q = 0,
                                             int* __restrict__ sstk = nullptr, int wcap = WSTACK) {
    const int y = image_row(A, k, frame);
    if (y >= A.H) return;  // frame_shift: a rotated rank's compact rows past the image
    const int o = (int)((size_t)frame * A.frame_px + (size_t)k * A.W + x);  // (< 2^31: rt_render's bound)
    int hit0 = -1;
    float t0 = FMAX;
    v3 col;
    if (A.bounce_hit)
        for (int i = 0; i < A.bounces; i++) A.bounce_hit[(size_t)o * A.bounces + i] = -2;
    if (SPPM == 1 || (SPPM == 0 && A.spp <= 1)) {
        col = clamp01(trace_path<MAXB, STRICT, COUNT, REG, G, PB, PK, TQ>(A, C.pos, primary_dir(C, (float)x, (float)y),
                                                                          stk, c, hit0, t0, o, q, sstk, wcap));
    } else if (SPPM == 2) {  // stratified g x g sub-pixel grid, mean of clamped samples
        // the persistent kernels' multi-sample builds: the lane's A.lanebuf slot carries the running sum and the pixel
        // (x, compact row k) from sample to sample, so that no register stays live across a sample's path; hit / t of
        // the first sample are stored as soon as it returns (the host sets A.lanebuf for every k_persist launch and
        // guarantees W, n_rows <= 65535 for spp > 1)
        const int g = A.spp_grid;
        *lane_slot<PB == 2>(A) = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float((unsigned)x | ((unsigned)k << 16)));
        v3 acc = mk(0.0f, 0.0f, 0.0f);
        for (int s = 0; s < g * g; ++s) {
            __asm__ volatile("" ::: "memory");  // (read the slot back: no value forwarded in registers across the path)
            float4* lb = lane_slot<PB == 2>(A);
            const float4 e = *lb;
            const unsigned px = __float_as_uint(e.w);
            const int xs = (int)(px & 0xFFFFu), ks = (int)(px >> 16), ys = image_row(A, ks, frame);
            const int sj = s / g, si = s - sj * g;
            const float fx = (float)xs + ((float)si + 0.5f) / (float)g;
            const float fy = (float)ys + ((float)sj + 0.5f) / (float)g;
            const size_t os = (size_t)frame * A.frame_px + (size_t)ks * A.W + xs;
            int h;
            float tt;
            const v3 cs = clamp01(trace_path<MAXB, STRICT, COUNT, REG, G, PB, PK, TQ>(
                A, C.pos, primary_dir_sample(C, fx, fy), stk, c, h, tt, s == 0 ? (int)os : -1, q, sstk, wcap));
            __asm__ volatile("" ::: "memory");
            lb = lane_slot<PB == 2>(A);
            const float4 a = *lb;
            if (s == 0 && q == 0) {  // (the output index from the slot again, not held across the path)
                const unsigned pa = __float_as_uint(a.w);
                const size_t oa = (size_t)frame * A.frame_px + (size_t)(pa >> 16) * A.W + (pa & 0xFFFFu);
                if (A.hit) A.hit[oa] = h;
                if (A.t) A.t[oa] = tt;
            }
            acc = add(mk(a.x, a.y, a.z), cs);
            *lb = make_float4(acc.x, acc.y, acc.z, a.w);
        }
        const float nn = (float)(g * g);
        CTR_INC(c, pix, C_PIX);
        if (q != 0) return;
        __asm__ volatile("" ::: "memory");
        const unsigned pf = __float_as_uint(lane_slot<PB == 2>(A)->w);  // (the pixel from the slot: nothing held across the loop)
        store_px(A.rgb, A.bgra, (size_t)frame * A.frame_px + (size_t)(pf >> 16) * A.W + (pf & 0xFFFFu),
                 mk(acc.x / nn, acc.y / nn, acc.z / nn));
        return;
    } else {  // stratified g x g sub-pixel grid, mean of clamped samples
        const int g = A.spp_grid;
        v3 acc = mk(0.0f, 0.0f, 0.0f);
        for (int sj = 0; sj < g; ++sj)
            for (int si = 0; si < g; ++si) {
                const float fx = (float)x + ((float)si + 0.5f) / (float)g;
                const float fy = (float)y + ((float)sj + 0.5f) / (float)g;
                int h;
                float tt;
                v3 cs;
                cs = clamp01(trace_path<MAXB, STRICT, COUNT, REG, G, PB, PK, TQ>(
                        A, C.pos, primary_dir(C, fx, fy), stk, c, h, tt, si == 0 && sj == 0 ? o : -1, q, sstk, wcap));
                acc = add(acc, cs);
                if (si == 0 && sj == 0) {
                    hit0 = h;
                    t0 = tt;
                }
            }
        const float nn = (float)(g * g);
        col = mk(acc.x / nn, acc.y / nn, acc.z / nn);
    }
    CTR_INC(c, pix, C_PIX);
    if (q != 0) return;  // a group's pixel is written once
    const int oo = opaque(o);
    store_px(A.rgb, A.bgra, (size_t)oo, col);
    if (A.hit) A.hit[oo] = hit0;
    if (A.t) A.t[oo] = t0;
}

// ---------------------------------------------------------------- kernels
template <int MAXB, bool STRICT, bool COUNT>
__global__ __launch_bounds__(BLOCK) void k_tiles(KArgs A) {
    __shared__ int lds[STACK * BLOCK];
    int* stk = lds + threadIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (w & 1) * 8 + (lane & 7);
    const int k = blockIdx.y * 16 + (w >> 1) * 8 + (lane >> 3);
    Ctr c = {};
    if (x < A.W && k < A.n_rows) render_pixel<MAXB, STRICT, COUNT>(A, cam_of(A, 0), 0, x, k, stk, c);
    flush<COUNT>(c, A.counters);
}

// Persistent variant: each wave repeatedly takes the next 8x8 tile from a global counter
// (one returning atomic per wave per tile; microarch row "dequeue"). Tiles are dealt in row-major
// order of 8x8 blocks so that concurrently running waves trace neighbouring pixels (shared L1/L2
// lines for the upper BVH levels).
// OCC: waves per SIMD the register allocation must allow: 3 caps VGPRs at 168 (512 / 3 in 8-register
// granules; one register more halves nothing but drops a whole wave per SIMD), 4 at 128 (the LDS
// stack allows 4 workgroups per CU).
// The next (frame, tile) item of a persistent wave. Default: one counter over items t = (tile t / F of
// the dealing order, frame t % F). XCD-aware (A.region_off): the workgroups on XCD x (blockIdx % 8, the
// dispatcher's round-robin) drain spatial region x first — its rays touch a smaller part of the scene,
// which that XCD's own 4 MB L2 then holds — and then the other regions in turn (load balance); `reg` is
// the wave's current region offset from its home region.
__device__ __forceinline__ bool next_item(const KArgs& A, int lane, int& reg, int& frame, unsigned& tile) {
    const unsigned F = (unsigned)A.n_frames;
    if (!A.region_off) {
        unsigned t = 0;
        if (lane == 0) t = atomicAdd(A.work, 1u);
        t = __builtin_amdgcn_readfirstlane(__shfl(t, 0, 64));
        if (t >= (unsigned)A.n_tiles * F) return false;
        frame = (int)(t % F);
        tile = t / F;
        if (A.tile_order) tile = (unsigned)A.tile_order[tile];
        return true;
    }
    while (reg < 8) {
        const int r = (int)((blockIdx.x + (unsigned)reg) & 7u);
        const unsigned base = (unsigned)A.region_off[r], n = (unsigned)A.region_off[r + 1] - base;
        unsigned t = 0;
        if (lane == 0) t = atomicAdd(A.work + 16 * r, 1u);
        t = __builtin_amdgcn_readfirstlane(__shfl(t, 0, 64));
        if (t < n * F) {
            frame = (int)(t % F);
            tile = (unsigned)A.tile_order[base + t / F];
            return true;
        }
        ++reg;
    }
    return false;
}

// DYN: the wide walk's stack in dynamic LDS sized to the scene's wide depth (wstack_words ints per lane instead
// of STACK = 34) and the binary walks' (rare strict fallbacks) in global memory, so that more workgroups
// fit a CU's LDS: the kernels with OCC > 4 waves per SIMD.
template <int SHP> struct UCtrSel { using type = UCtr; };
template <> struct UCtrSel<0> { struct type {}; };
template <> struct UCtrSel<3> { struct type {}; };
template <int SHP> using UCtrOf = typename UCtrSel<SHP>::type;

template <int MAXB, bool STRICT, bool COUNT, bool REG = true, int OCC = 3, bool TRACE = false, bool BATCH = false,
          int PB = 0, bool DYN = false, bool SPP1 = false, int SHP = 0>
__global__ __attribute__((amdgpu_flat_work_group_size(1, BLOCK), amdgpu_waves_per_eu(OCC > 0 ? OCC : 1)))
void k_persist(KArgs A) {
    static_assert(PB != 2 || DYN, "an LDS path buffer lives in the DYN kernels' dynamic LDS");
    static_assert(SHP == 0 || SHP == 3 || PB == 2, "the shadow pool hands its rays over through the LDS path buffer");
    // SHP = 3: no pool; packed triangle tests (queues after the LDS path buffer with packed stack entries in the DYN
    // kernels, a static array in the others)
    int* stk;
    int* sstk = nullptr;
    int wcap = WSTACK;
    if constexpr (DYN) {
        extern __shared__ int lds_dyn[];
        stk = lds_dyn + threadIdx.x;
        sstk = A.gstack + (size_t)blockIdx.x * STACK * BLOCK + threadIdx.x;
        wcap = A.wcap;
    } else {
        __shared__ int lds[STACK * BLOCK];
        stk = lds + threadIdx.x;
    }
    const int lane = threadIdx.x & 63;
    Ctr c = {};
    if constexpr (COUNT) {
        c.hist = hist_lds<true>();
        if (threadIdx.x < 32) c.hist[threadIdx.x] = 0u;
        __syncthreads();
    }
    if constexpr (LDS_TOP) {  // the top nodes of the primary and the unit-direction views (wide_for's choices)
        if (A.s.wide.nodes) {
            float4* t = top_lds<true>();
            const DWide& P = A.s.prim.nodes ? A.s.prim : A.s.wide;
            const DWide& U = A.s.unit.nodes ? A.s.unit : A.s.wide;
            for (int i = threadIdx.x; i < 2 * NTOP * 5; i += BLOCK) {
                const DWide& W = i < NTOP * 5 ? P : U;
                const int r = i % (NTOP * 5);
                if (r < 5 * W.n) t[i] = W.nodes[r];
            }
            __syncthreads();
            c.top[0] = t;
            c.top[1] = t + NTOP * 5;
        }
    }
    constexpr bool EVM = !COUNT && !TRACE;  // (the tile trace reads the per-lane fallback counts)
    if constexpr (EVM) {
        c.evm = true;
        c.ev = ev_lds<true>();
        if (threadIdx.x < 16) c.ev[threadIdx.x] = 0u;
        __syncthreads();
    }
    UCtrOf<SHP> u = {};  // SHP: the wave-uniform ray counts (rt_shpool.hpp)
    if constexpr (SHP == 3) {  // the wave's packed-triangle queue starts clear
        if constexpr (DYN) {
            extern __shared__ int lds_dyn[];
            tq_clear((int*)((float4*)(lds_dyn + wstack_words(wcap, true) * BLOCK) + (size_t)BLOCK * MAXB) +
                     (threadIdx.x >> 6) * TQ_WORDS);
        } else {
            tq_clear(tq_static());
        }
    }
    // frame batches: dealt item t = (tile t / n_frames of the dealing order, frame t % n_frames), so the
    // expensive (central) tiles of every frame of the batch start first
    int reg = 0;
    for (;;) {
        int frame;
        unsigned tile;
        if (!next_item(A, lane, reg, frame, tile)) break;
        const int tx = (int)(tile % (unsigned)A.tiles_x), ty = (int)(tile / (unsigned)A.tiles_x);
        const unsigned ln = lane_now();  // (remade per tile rather than held, or spilled, across the walks)
        const int x = tx * 8 + (int)(ln & 7u), k = ty * 8 + (int)(ln >> 3);
        unsigned long long t0 = 0;
        const unsigned fb0 = c.fb, ws0 = c.ws, nd0 = c.chi + c.shi;
        if (TRACE || A.tile_cost) t0 = __builtin_amdgcn_s_memrealtime();
        if constexpr (SHP == 1 || SHP == 2)
            render_pixel_shp<MAXB, COUNT, SPP1, SHP>(A, cam_of<BATCH>(A, frame), frame, x, k, x < A.W && k < A.n_rows,
                                                     stk, c, u, sstk, wcap);
        else if (x < A.W && k < A.n_rows)
            render_pixel<MAXB, STRICT, COUNT, REG, 1, PB, SPP1 ? 1 : 2, SHP == 3, SHP == 3 && DYN>(
                A, cam_of<BATCH>(A, frame), frame, x, k, stk, c, 0u, sstk, wcap);
        if (A.tile_cost && lane == 0)  // the feedback's tile duration (single frames: tile = its 8x8 tile)
            A.tile_cost[tile] = (unsigned)(__builtin_amdgcn_s_memrealtime() - t0);
        if (TRACE) {  // {begin, end, wave | fallbacks << 32, wave steps | lane node visits << 32} (COUNT)
            const unsigned fb = wave_sum(c.fb - fb0), ws = wave_sum(c.ws - ws0), nv = wave_sum(c.chi + c.shi - nd0);
            if (lane == 0) {
                A.tile_trace[4 * tile] = t0;
                A.tile_trace[4 * tile + 1] = __builtin_amdgcn_s_memrealtime();
                A.tile_trace[4 * tile + 2] = (blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6)) | ((unsigned long long)fb << 32);
                A.tile_trace[4 * tile + 3] = ws | ((unsigned long long)nv << 32);
            }
        }
    }
    flush<COUNT>(c, A.counters);
    if constexpr (SHP == 1 || SHP == 2) flush_u(u, A.counters);
    if constexpr (EVM) {  // every wave of the workgroup leaves the tile loop and reaches this point
        __syncthreads();
        if (threadIdx.x < 16 && c.ev[threadIdx.x]) atomicAdd(A.counters + threadIdx.x, (unsigned long long)c.ev[threadIdx.x]);
    }
    if constexpr (COUNT) {  // every wave of the workgroup leaves the tile loop and reaches this point
        __syncthreads();
        if (threadIdx.x < 32 && c.hist[threadIdx.x]) atomicAdd(A.counters + C_HIST + threadIdx.x, (unsigned long long)c.hist[threadIdx.x]);
    }
}

}  // namespace rtd
