// rt_pool.hpp — k_pool: tile-local ray queues with dynamic fetch (ballot compaction of divergent rays).
//
// k_persist traces one pixel path per lane and runs a wave's 64 walks in lockstep: every closest-hit or shadow
// walk lasts as long as the wave's slowest lane, and lanes whose path has ended (a miss, kr = 0) or whose shadow
// ray was skipped (back-facing light) idle through the others' walks. Measured on the bench frame: SIMD efficiency
// of node steps 0.56. k_chain (round 2, removed) removed the idling by letting each lane run its
// own walks back to back, but mixed walk kinds and levels in a wave (per-step bookkeeping for both, less coherent
// node loads) and lost.
//
// k_pool keeps the walks of ONE kind and ONE level together, and moves the rays instead of the lanes: a
// workgroup (4 waves) owns a 16 x 16 pixel tile (wave w owns its 8 x 8 quadrant: owner thread t = pixel t), and
// every bounce level runs as two phases, separated by workgroup barriers:
//   closest phase: the owners of live paths append their pixel id to a workgroup queue in LDS (wave ballot +
//                  popcount + a 4-entry prefix: the queue is compact and in pixel order, so the first rays a
//                  wave takes are its own quadrant's), then the 4 waves trace the queue's rays with DYNAMIC
//                  FETCH: a lane whose walk ends takes the next queued ray as soon as `regroup` lanes of its
//                  wave are idle (one LDS atomic per refill for the wave, ranks by mbcnt), so a wave's walk no
//                  longer waits for its slowest lane while other rays are pending, and dead paths take no lane;
//   shadow phase:  the owners of hit points append (pixel, light) for every light past the back-face test
//                  (light-major: all of light 0's rays of the tile, then light 1's, ...; up to 4 lights per
//                  phase), traced the same way; occluded rays set their light's bit in the pixel's LDS word.
// Between phases the owners shade exactly as path_step does (raytracer.c:101-177), expression for expression:
// the closest hit's colour term, every light's Lambert/Blinn term with the shadow ray's visibility in light
// order, the reflection; each level's colour and material stay in the owner's registers and are folded
// deepest-first (the reference's summation order). Rays stay inside their 16 x 16 tile (coherence is kept:
// queue order = pixel order); paths never move between lanes mid-walk, so a ray's walk state (stack in LDS,
// [depth][lane], node record in registers) stays where it started.
//
// LDS per workgroup (dynamic): the wide stack (2 * wcap ints per lane), the tile's rays (o, d: 6 x 256 floats),
// closest results (orig, t, nd: 3 x 256; then the hit's normal and material, the owner's state across the shadow
// walks, so that only the walk's registers are live during a walk), the queue (4 x 256 ints), occlusion bits
// (256 ints), control words.
#pragma once
#include "rt_kernels.hpp"

namespace rtd {

// the rare strict walks (a zero direction component, an exact tie) out of line, so that their registers do not
// weigh on the walk loops; counters returned by value
struct StrictC {  // result of an out-of-line strict closest walk, counters returned by value
    int orig, nd;
    float best;
    unsigned chi, chl, cht, err;
};

template <bool COUNT>
__device__ __noinline__ StrictC strict_closest_ool(const DBvh B, v3 o, v3 d, int* __restrict__ bstk) {
    Ctr c = {};
    float best = FMAX;
    int hp = -1, nd = 0;
    bool tie = false;
    closest_walk<true, COUNT, true>(B, o, d, best, hp, nd, tie, bstk, c);
    return StrictC{hp >= 0 ? B.tri_orig[hp] : -1, nd, best, c.chi, c.chl, c.cht, c.err};
}

template <bool COUNT>
__device__ __noinline__ unsigned strict_visible_ool(const DBvh B, v3 o, v3 d, float ld2, int* __restrict__ bstk) {
    // bit 31: visible; bits 0..30: interior visits (COUNT; leaf / triangle counts are not kept)
    Ctr c = {};
    const bool v = visible_walk<true, COUNT, true>(B, o, d, ld2, bstk, c);
    return (v ? 0x80000000u : 0u) | (c.shi & 0x7FFFFFFFu);
}

constexpr int POOL_QL = 4;  // lights per shadow phase (queue capacity 256 x POOL_QL)
enum { PC_CNT = 0, PC_HEAD = 20, PC_ITEM = 21, PC_FRAME = 22, PC_N = 32 };

// LDS offsets (in 4-B words) of a k_pool workgroup
struct PoolLds {
    int* stk;    // [2 * wcap][256]
    float* ray;  // [6][256]: o.xyz, d.xyz (the shadow phase: o = the hit point)
    float* res;  // [4][256]: orig (int bits), best, nd (int bits); then the owner's n.xyz, material (int bits)
    int* q;      // [256 * POOL_QL]
    unsigned* occ;  // [256]
    int* ctl;    // [PC_N]
};
__host__ __device__ constexpr size_t pool_lds_bytes(int wcap) {
    return sizeof(int) * ((size_t)2 * wcap * BLOCK + 6 * BLOCK + 4 * BLOCK + POOL_QL * BLOCK + BLOCK + PC_N);
}

// Appends entry `e` of every thread with `want` to the workgroup queue at `base0` (thread order: wave order,
// then lane order); returns the number appended. Two barriers; the caller reads q only after both.
__device__ __forceinline__ int pool_append(const PoolLds& L, int slot, bool want, int e, int base0) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long m = __ballot(want);
    if (lane == 0) L.ctl[PC_CNT + 4 * slot + w] = __popcll(m);
    __syncthreads();
    int base = base0, total = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int c = L.ctl[PC_CNT + 4 * slot + i];
        base += i < w ? c : 0;
        total += c;
    }
    if (want) L.q[base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))] = e;
    return total;
}

// Dynamic fetch: when at least `refill` lanes of the wave are idle (r < 0) and the queue is not drained, the
// wave takes that many entries with one LDS atomic; returns this lane's new queue position (-1: none).
__device__ __forceinline__ int pool_fetch(const PoolLds& L, bool idle_me, int refill, int total, bool& drained) {
    const unsigned long long idle = __ballot(idle_me);
    const int n = __popcll(idle);
    if (drained || n == 0 || (n < refill && n < 64)) return -1;
    const int lane = threadIdx.x & 63;
    const int first = __builtin_ctzll(idle);
    int base = 0;
    if (lane == first) base = atomicAdd(&L.ctl[PC_HEAD], n);
    base = __shfl(base, first, 64);
    if (base + n >= total) drained = true;
    if (!idle_me) return -1;
    const int k = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(idle >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)idle, 0u));
    return k < total ? k : -1;
}

// The closest-hit rays of the queue (pixel ids): one wide-node step per loop iteration for every lane with a ray,
// refills in between. Results to L.res[.][pixel].
template <bool COUNT>
__device__ __forceinline__ void pool_closest(const DScene& s, const PoolLds& L, int total, int refill, int wcap,
                                             int* __restrict__ bstk, Ctr& c) {
    const DWide& W = s.wide;
    int r = -1;  // pixel of this lane's ray
    bool drained = false;
    v3 o = mk(0.0f, 0.0f, 0.0f), d = o;
    RayPre p = {};
    unsigned oct = 0;
    float best = FMAX;
    int hp = -1, nd = 0, sp = 0;
    bool tie = false;
    WNode N = {};
    for (;;) {
        const int k = pool_fetch(L, r < 0, refill, total, drained);
        if (k >= 0) {
            r = L.q[k];
            o = mk(L.ray[r], L.ray[BLOCK + r], L.ray[2 * BLOCK + r]);
            d = mk(L.ray[3 * BLOCK + r], L.ray[4 * BLOCK + r], L.ray[5 * BLOCK + r]);
            best = FMAX;
            hp = -1;
            nd = 0;
            tie = false;
            sp = 0;
            if (degenerate(d)) {  // the reference's 0/0 NaN slabs: strict walk from the start (out of line)
                c.fb++;
                const StrictC sr = strict_closest_ool<COUNT>(s.ref, o, d, bstk);
                if (COUNT) {
                    c.chi += sr.chi;
                    c.chl += sr.chl;
                    c.cht += sr.cht;
                    c.nb += 8 * sr.chi + sr.chl;
                }
                c.err += sr.err;
                L.res[r] = __int_as_float(sr.orig);
                L.res[BLOCK + r] = sr.best;
                L.res[2 * BLOCK + r] = __int_as_float(sr.nd);
                r = -1;
            } else {
                p = ray_pre(o, d);
                oct = (p.ix < 0.0f ? 1u : 0u) | (p.iy < 0.0f ? 2u : 0u) | (p.iz < 0.0f ? 4u : 0u);
                N = wload(W, 0);
            }
        }
        if (!__ballot(r >= 0)) {  // every lane idle: either the queue is drained or the fetched rays were all
            if (drained) break;   // resolved at once (strict fallbacks), and the next pass fetches again
            continue;
        }
        if (r >= 0) {  // closest_wide's step
            unsigned nh, th, imask, nl;
            int cb, tb;
            wide_node<COUNT>(N, p, oct, best * PRUNE_SLACK, nh, th, cb, tb, imask, nl);
            if (COUNT) {
                c.chi++;
                c.chl += nl;
                c.nb += 10;
                c.ws += first_active_lane();
            }
            const int next = wide_next(nh, cb, imask, oct, sp, L.stk + threadIdx.x, wcap);
            N = wload(W, next >= 0 ? next : 0);  // unconditional (rt_kernels.hpp closest_wide)
            while (th) {
                const int i = tb + __builtin_ctz(th);
                th &= th - 1u;
                int kk;
                const float tt = hit_triangle(o, d, W.tris + 3 * i, kk);
                if (COUNT) c.cht++;
                if (tt < best) {
                    best = tt;
                    nd = kk;
                    hp = i;
                    tie = false;
                } else if (tt == best && tt != FMAX) {
                    tie = true;
                }
            }
            if (next < 0) {
                if (next == -2) c.err++;
                int orig = hp >= 0 ? W.tri_orig[hp] : -1;
                if (tie) {  // exact tie: the reference keeps the first triangle found (bvh.c:331), strict re-walk
                    c.fb++;
                    const StrictC sr = strict_closest_ool<COUNT>(s.ref, o, d, bstk);
                    if (COUNT) {
                        c.chi += sr.chi;
                        c.chl += sr.chl;
                        c.cht += sr.cht;
                        c.nb += 8 * sr.chi + sr.chl;
                    }
                    c.err += sr.err;
                    orig = sr.orig;
                    nd = sr.nd;
                    best = sr.best;
                }
                L.res[r] = __int_as_float(orig);
                L.res[BLOCK + r] = best;
                L.res[2 * BLOCK + r] = __int_as_float(nd);
                r = -1;
            }
        }
    }
}

// The shadow rays of the queue (pixel | light << 8): the hit point in L.ray[0..2][pixel], the direction and
// distance recomputed from the light as path_step does; occluded rays set bit `light - j0` of L.occ[pixel].
template <bool COUNT>
__device__ __forceinline__ void pool_shadow(const DScene& s, const PoolLds& L, int total, int refill, int wcap,
                                            int j0, int* __restrict__ bstk, Ctr& c) {
    const DWide& W = s.wide;
    int r = -1;  // this lane's queue entry (pixel | light << 8)
    bool drained = false;
    v3 o = mk(0.0f, 0.0f, 0.0f), d = o;
    RayPre p = {};
    unsigned oct = 0;
    float best = FMAX, reach = 0.0f, ld2 = 0.0f;
    int sp = 0;
    WNode N = {};
    for (;;) {
        const int k = pool_fetch(L, r < 0, refill, total, drained);
        if (k >= 0) {
            r = L.q[k];
            const int px = r & 255, j = r >> 8;
            o = mk(L.ray[px], L.ray[BLOCK + px], L.ray[2 * BLOCK + px]);
            const v3 Lp = xyz(s.lights[2 * j]);  // light_v, raytracer.c:62-99 (as path_step)
            v3 l = sub(Lp, o);
            const float mg = mag(l);
            l = dvs(l, mg);
            const v3 tmp = sub(o, Lp);
            ld2 = dot(tmp, tmp);
            d = l;
            best = FMAX;
            sp = 0;
            if (degenerate(d)) {
                c.fb++;
                const unsigned sr = strict_visible_ool<COUNT>(s.ref, o, d, ld2, bstk);
                if (COUNT) {
                    c.shi += sr & 0x7FFFFFFFu;
                    c.nb += 8 * (sr & 0x7FFFFFFFu);
                }
                if ((sr >> 31) == 0u) atomicOr(&L.occ[px], 1u << (j - j0));
                r = -1;
            } else {
                p = ray_pre(o, d);
                oct = (p.ix < 0.0f ? 1u : 0u) | (p.iy < 0.0f ? 2u : 0u) | (p.iz < 0.0f ? 4u : 0u);
                reach = shadow_reach(o, ld2);
                N = wload(W, 0);
            }
        }
        if (!__ballot(r >= 0)) {  // every lane idle: either the queue is drained or the fetched rays were all
            if (drained) break;   // resolved at once (strict fallbacks), and the next pass fetches again
            continue;
        }
        if (r >= 0) {  // visible_wide's step
            unsigned nh, th, imask, nl;
            int cb, tb;
            wide_node<COUNT>(N, p, oct, fminf(best * PRUNE_SLACK, reach), nh, th, cb, tb, imask, nl, SHADOW_ORDER_XOR);
            if (COUNT) {
                c.shi++;
                c.shl += nl;
                c.nb += 10;
                c.ws += first_active_lane();
            }
            const int next = wide_next(nh, cb, imask, oct ^ SHADOW_ORDER_XOR, sp, L.stk + threadIdx.x, wcap);
            N = wload(W, next >= 0 ? next : 0);  // unconditional (rt_kernels.hpp closest_wide)
            bool occl = false;
            while (th) {
                const int i = tb + __builtin_ctz(th);
                th &= th - 1u;
                int kk;
                const float tt = hit_triangle(o, d, W.tris + 3 * i, kk);
                if (COUNT) c.sht++;
                if (tt < best) {
                    best = tt;
                    const v3 ip = add(o, mul(d, best));
                    const v3 oi = sub(o, ip);
                    if (ld2 > dot(oi, oi)) {  // bvh.c:283-290: an occluder nearer than the light
                        occl = true;
                        break;
                    }
                }
            }
            if (next == -2) c.err++;
            if (occl || next < 0) {
                if (occl) atomicOr(&L.occ[r & 255], 1u << ((r >> 8) - j0));
                r = -1;
            }
        }
    }
}

// OCC: waves per SIMD the register allocation must allow (4: <= 128 VGPRs).
template <int MAXB, bool COUNT, int OCC, bool BATCH>
__global__ __attribute__((amdgpu_flat_work_group_size(BLOCK, BLOCK), amdgpu_waves_per_eu(OCC))) void k_pool(KArgs A) {
    extern __shared__ int lds_dyn[];
    const int wcap = A.wcap;
    PoolLds L;
    L.stk = lds_dyn;
    L.ray = (float*)(lds_dyn + 2 * wcap * BLOCK);
    L.res = L.ray + 6 * BLOCK;
    L.q = (int*)(L.res + 4 * BLOCK);
    L.occ = (unsigned*)(L.q + POOL_QL * BLOCK);
    L.ctl = (int*)(L.occ + BLOCK);
    int* bstk = A.gstack + (size_t)blockIdx.x * STACK * BLOCK + threadIdx.x;
    const DScene& s = A.s;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const v3 amb = mk(s.amb_x, s.amb_y, s.amb_z);
    const int refill = A.regroup > 0 ? A.regroup : 16;
    const int nl = s.n_lights;
    Ctr c = {};
    int reg = 0;
    for (;;) {
        // ---- the workgroup's next (16 x 16 tile, frame): wave 0 deals, the others read it from LDS
        if (w == 0) {
            int frame = 0;
            unsigned tile = 0;
            const bool ok = next_item(A, lane, reg, frame, tile);
            if (lane == 0) {
                L.ctl[PC_ITEM] = ok ? (int)tile : -1;
                L.ctl[PC_FRAME] = frame;
            }
        }
        __syncthreads();
        const int item = L.ctl[PC_ITEM], frame = L.ctl[PC_FRAME];
        if (item < 0) break;
        const Cam C = cam_of<BATCH>(A, frame);
        const int x = (item % A.tiles_x) * 16 + (w & 1) * 8 + (lane & 7);
        const int k = (item / A.tiles_x) * 16 + (w >> 1) * 8 + (lane >> 3);
        const int y = k < A.n_rows ? image_row(A, k, frame) : A.H;
        const bool valid = x < A.W && k < A.n_rows && y < A.H;  // frame_shift: rows past the image are skipped
        const size_t po = (size_t)frame * A.frame_px + (size_t)k * A.W + x;
        if (valid && A.bounce_hit)
            for (int i = 0; i < A.bounces; i++) A.bounce_hit[po * (size_t)A.bounces + i] = -2;
        const int g = A.spp_grid;
        const int ns = A.spp <= 1 ? 1 : g * g;
        v3 acc = mk(0.0f, 0.0f, 0.0f);
        for (int si = 0; si < ns; ++si) {  // render_pixel (main.c:228-239) and its stratified samples
            v3 cols[MAXB];
            int mats[MAXB];
#pragma unroll
            for (int i = 0; i < MAXB; i++) {
                cols[i] = mk(0.0f, 0.0f, 0.0f);
                mats[i] = 0;
            }
            int Lv = 0;
            bool tail = false, alive = valid;
            if (valid) {  // the primary ray (o, d) into the tile's ray slots
                float fx = (float)x, fy = (float)y;
                if (A.spp > 1) {
                    fx = (float)x + ((float)(si % g) + 0.5f) / (float)g;
                    fy = (float)y + ((float)(si / g) + 0.5f) / (float)g;
                }
                const v3 dd = primary_dir(C, fx, fy);
                L.ray[t] = C.pos.x;
                L.ray[BLOCK + t] = C.pos.y;
                L.ray[2 * BLOCK + t] = C.pos.z;
                L.ray[3 * BLOCK + t] = dd.x;
                L.ray[4 * BLOCK + t] = dd.y;
                L.ray[5 * BLOCK + t] = dd.z;
            }
            for (int it = 0; it < A.bounces; ++it) {
                // ---- closest phase (raytrace's bvh_traverse, raytracer.c:129)
                if (alive) {
                    if (it == 0) c.prim++;
                    else c.refl++;
                }
                if (t == 0) L.ctl[PC_HEAD] = 0;
                const int nq = pool_append(L, 0, alive, t, 0);
                __syncthreads();
                if (nq == 0) break;  // (uniform) every path of the tile has ended
                pool_closest<COUNT>(s, L, nq, refill, wcap, bstk, c);
                __syncthreads();
                // ---- the hit (raytracer.c:130-147); its state goes to the pixel's LDS slots (ray[0..2] = ip,
                // res[0..3] = n, m), the shadow phase's back-face tests use it, the walkers only ray[0..2]
                bool shade = false;
                if (alive) {
                    const int orig = __float_as_int(L.res[t]);
                    const float best = L.res[BLOCK + t];
                    const int ndv = __float_as_int(L.res[2 * BLOCK + t]);
                    if (si == 0) {
                        if (it == 0) {
                            if (A.hit) A.hit[po] = orig;
                            if (A.t) A.t[po] = best;
                        }
                        if (A.bounce_hit) A.bounce_hit[po * (size_t)A.bounces + it] = orig;
                    }
                    if (orig < 0) {  // raytracer.c:132-135
                        set3<MAXB>(cols, it, mk(0.0f + amb.x, 0.0f + amb.y, 0.0f + amb.z));
                        Lv = it + 1;
                        tail = false;
                        alive = false;
                    } else {
                        c.hits++;
                        const v3 o = mk(L.ray[t], L.ray[BLOCK + t], L.ray[2 * BLOCK + t]);
                        const v3 d = mk(L.ray[3 * BLOCK + t], L.ray[4 * BLOCK + t], L.ray[5 * BLOCK + t]);
                        const v3 ip = add(o, mul(d, best));
                        const float4 sh0 = s.shade[2 * orig], sh1 = s.shade[2 * orig + 1];
                        const v3 n = ndv ? xyz(sh1) : xyz(sh0);
                        L.ray[t] = ip.x;  // the shadow rays' origin
                        L.ray[BLOCK + t] = ip.y;
                        L.ray[2 * BLOCK + t] = ip.z;
                        L.res[t] = n.x;
                        L.res[BLOCK + t] = n.y;
                        L.res[2 * BLOCK + t] = n.z;
                        L.res[3 * BLOCK + t] = sh0.w;  // material id (int bits)
                        shade = true;
                    }
                }
                v3 col = mk(0.0f, 0.0f, 0.0f);
                // ---- shadow phases, POOL_QL lights each (light_v, raytracer.c:149-160)
                for (int j0 = 0; j0 < nl; j0 += POOL_QL) {
                    const int jn = nl - j0 < POOL_QL ? nl - j0 : POOL_QL;
                    L.occ[t] = 0u;
                    if (t == 0) L.ctl[PC_HEAD] = 0;
                    int base = 0;
                    for (int j = 0; j < jn; j++) {
                        bool want = false;
                        if (shade) {
                            const v3 ip = mk(L.ray[t], L.ray[BLOCK + t], L.ray[2 * BLOCK + t]);
                            const v3 n = mk(L.res[t], L.res[BLOCK + t], L.res[2 * BLOCK + t]);
                            const v3 Lp = xyz(s.lights[2 * (j0 + j)]);
                            const v3 tmp2 = sub(Lp, ip);
                            if (dot(tmp2, n) < 0) c.skip++;
                            else {
                                c.shad++;
                                want = true;
                            }
                        }
                        base += pool_append(L, 1 + j, want, t | ((j0 + j) << 8), base);  // (one count slot per light)
                    }
                    __syncthreads();
                    if (base) pool_shadow<COUNT>(s, L, base, refill, wcap, j0, bstk, c);
                    __syncthreads();
                    if (shade) {  // every light's term in light order, V from the shadow ray (raytracer.c:21-33,157-159)
                        const v3 ip = mk(L.ray[t], L.ray[BLOCK + t], L.ray[2 * BLOCK + t]);
                        const v3 n = mk(L.res[t], L.res[BLOCK + t], L.res[2 * BLOCK + t]);
                        const int m = __float_as_int(L.res[3 * BLOCK + t]);
                        if (j0 == 0) {
                            const v3 kd0 = xyz(s.mats[3 * m + 1]);
                            col = mk(0.0f + kd0.x * amb.x, 0.0f + kd0.y * amb.y, 0.0f + kd0.z * amb.z);  // :144-146
                        }
                        const unsigned ob = L.occ[t];
                        const v3 d = mk(L.ray[3 * BLOCK + t], L.ray[4 * BLOCK + t], L.ray[5 * BLOCK + t]);
                        const v3 v = mul(d, -1.0f);
                        for (int j = 0; j < jn; j++) {
                            const v3 Lp = xyz(s.lights[2 * (j0 + j)]);
                            v3 l = sub(Lp, ip);
                            float mg = mag(l);
                            l = dvs(l, mg);
                            mg *= mg;
                            const v3 tmp2 = sub(Lp, ip);
                            const int V = dot(tmp2, n) < 0 ? 0 : ((ob >> j) & 1u) ? 0 : 1;
                            const v3 kl = xyz(s.lights[2 * (j0 + j) + 1]);
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
                    }
                    __syncthreads();  // occ / queue reused by the next light group
                }
                if (shade) {  // the reflection (raytracer.c:162-173)
                    const v3 n = mk(L.res[t], L.res[BLOCK + t], L.res[2 * BLOCK + t]);
                    const int m = __float_as_int(L.res[3 * BLOCK + t]);
                    if (nl == 0) {
                        const v3 kd0 = xyz(s.mats[3 * m + 1]);
                        col = mk(0.0f + kd0.x * amb.x, 0.0f + kd0.y * amb.y, 0.0f + kd0.z * amb.z);  // :144-146
                    }
                    const v3 d = mk(L.ray[3 * BLOCK + t], L.ray[4 * BLOCK + t], L.ray[5 * BLOCK + t]);
                    const v3 v = mul(d, -1.0f);
                    const v3 dd = mul(v, -1.0f);
                    const v3 ns = mul(n, 2.0f * __builtin_fabsf(dot(dd, n)));
                    const v3 r = normalize(add(dd, ns));
                    set3<MAXB>(cols, it, col);
                    seti<MAXB>(mats, it, m);
                    const v3 kr = xyz(s.mats[3 * m + 2]);
                    if (!(mag(kr) > 0.0f)) {
                        Lv = it + 1;
                        tail = false;
                        alive = false;
                    } else if (it + 1 == A.bounces) {  // raytrace(.., BOUNCES) returns {0,0,0}: col += kr * 0
                        Lv = it + 1;
                        tail = true;
                        alive = false;
                    } else {  // the next level's ray: o = the hit point (already in the slots), d = r
                        L.ray[3 * BLOCK + t] = r.x;
                        L.ray[4 * BLOCK + t] = r.y;
                        L.ray[5 * BLOCK + t] = r.z;
                    }
                }
            }
            if (valid) {
                const v3 cs = clamp01(fold_path<MAXB>(s, cols, mats, Lv, tail));
                acc = A.spp <= 1 ? cs : add(acc, cs);
            }
            __syncthreads();  // the slots are rewritten by the next sample
        }
        if (valid) {
            v3 col = acc;
            if (A.spp > 1) {
                const float nn = (float)(g * g);
                col = mk(acc.x / nn, acc.y / nn, acc.z / nn);
            }
            c.pix++;
            store_px(A.rgb, A.bgra, po, col);
        }
    }
    flush<COUNT>(c, A.counters);
}

}  // namespace rtd
