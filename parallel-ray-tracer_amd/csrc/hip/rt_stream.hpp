// rt_stream.hpp — k_stream (RT_VARIANT_STREAM): persistent waves whose lanes each trace one pixel's path at a time
// and take the next pixel of the wave's current 8x8 tile as soon as their path ends.
//
// k_persist runs a wave's 64 paths level by level in lockstep: at bounce level i only the lanes whose path reached it
// work, so the deep levels run with few active lanes (dragon, 20-frame batches: 33 % of all wave steps have 1-16 of
// 64 lanes active, most of them at levels 2-3 of both walk kinds; bench.py roofline.per_ray.wave_steps_by_kind_level).
// Here a lane whose path has ended (a miss, a material without reflection, or BOUNCES reached) folds and stores its
// pixel, and at the top of the next round takes the next pending pixel of the wave's tile; when the tile has none
// left the wave takes its next tile (rtd::next_item: the dealing order, XCD regions, frame batches). So every round
// -- one closest-hit walk per lane, then its level's shadow rays through the per-wave pool (rt_shpool.hpp), then the
// Lambert/Blinn terms -- runs with (nearly) every lane busy until the launch runs out of tiles. A wave's lanes hold
// pixels of one tile, or of two consecutive ones, at different levels of their paths. Nothing is workgroup-wide: no
// barrier.
//
// Bit-exactness: a path is the reference's recursion (raytracer.c:101-177) whatever lane runs it and whenever: the
// closest walk of level i (primary view at level 0, the unit-direction view above), the shadow rays from the pool,
// path_step's colour expressions in the reference's order, and the fold of the levels deepest-first (fold_pb).
#pragma once
#include "rt_shpool.hpp"

namespace rtd {

// frame f's camera for a lane (frames may differ between the lanes of a wave: per-lane loads, or the arguments)
__device__ __forceinline__ Cam cam_lane(const KArgs& A, int f) {
    if (!A.cams) return cam_of<false>(A, 0);
    const float4* c4 = reinterpret_cast<const float4*>(A.cams) + 3 * f;
    const float4 a = c4[0], b = c4[1], e = c4[2];
    return Cam{mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), mk(b.z, b.w, e.x), mk(e.y, e.z, e.w)};
}

// spp = 1 (the reference's pixel-corner ray). PB: the path levels in the LDS path buffer after the wide stack (DYN).
template <int MAXB, bool COUNT>
__global__ __attribute__((amdgpu_flat_work_group_size(1, BLOCK), amdgpu_waves_per_eu(4))) void k_stream(KArgs A) {
    extern __shared__ int lds_dyn[];
    const int lane = (int)(threadIdx.x & 63u);
    int* stk = lds_dyn + threadIdx.x;
    int* sstk = A.gstack + (size_t)blockIdx.x * STACK * BLOCK + threadIdx.x;
    const int wcap = A.wcap;
    float4* pb = (float4*)(lds_dyn + 2 * wcap * BLOCK) + (size_t)((threadIdx.x >> 6) * MAXB) * 64 + lane;
    float4* pbw = pb - lane;  // the wave's slots
    const DScene& s = A.s;
    const v3 amb = mk(s.amb_x, s.amb_y, s.amb_z);
    Ctr c = {};
    UCtr u = {};
    if constexpr (COUNT) {
        c.hist = hist_lds<true>();
        if (threadIdx.x < 32) c.hist[threadIdx.x] = 0u;
        __syncthreads();
    }
    // the wave's tile supply (wave-uniform): the pending pixels of the current tile, the dealing cursor
    int reg = 0;
    bool more = true;
    unsigned long long pend = 0ull;
    int ptile = 0, pframe = 0;
    // this lane's path: its pixel (output index), its level, its ray
    bool active = false;
    int it = 0, opix = 0;
    v3 o = mk(0.0f, 0.0f, 0.0f), d = o;
    for (;;) {
        // idle lanes take the next pending pixels: the k-th idle lane the k-th pending pixel, the tiles in dealing order
        unsigned long long idle = uni64(__ballot(!active));
        bool got = false;
        int gpix = 0, gtile = 0, gframe = 0;
        while (idle != 0ull) {
            if (pend == 0ull) {
                if (!more) break;
                int frame;
                unsigned tile;
                if (!next_item(A, lane, reg, frame, tile)) {
                    more = false;
                    break;
                }
                ptile = uni((int)tile);
                pframe = uni(frame);
                const int x = (ptile % A.tiles_x) * 8 + (lane & 7), k = (ptile / A.tiles_x) * 8 + (lane >> 3);
                pend = uni64(__ballot(x < A.W && k < A.n_rows && image_row(A, k, pframe) < A.H));
                u.pix += (unsigned)__builtin_popcountll(pend);
                continue;
            }
            const unsigned nav = (unsigned)__builtin_popcountll(pend), nid = (unsigned)__builtin_popcountll(idle);
            const unsigned rk = __builtin_amdgcn_mbcnt_hi((unsigned)(idle >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)idle, 0u));
            if (((idle >> lane) & 1ull) && rk < nav) {
                gpix = kth_bit(pend, rk);
                gtile = ptile;
                gframe = pframe;
                got = true;
            }
            const unsigned take = nav < nid ? nav : nid;
            pend = uni64(drop_low(pend, take));
            idle = uni64(drop_low(idle, take));
        }
        if (got) {  // the pixel's primary ray (main.c:228-239)
            const int x = (gtile % A.tiles_x) * 8 + (gpix & 7), k = (gtile / A.tiles_x) * 8 + (gpix >> 3);
            const int y = image_row(A, k, gframe);
            opix = (int)((size_t)gframe * A.frame_px + (size_t)k * A.W + x);
            const Cam C = cam_lane(A, gframe);
            o = C.pos;
            d = primary_dir(C, (float)x, (float)y);
            it = 0;
            active = true;
            if (A.bounce_hit)
                for (int i = 0; i < A.bounces; i++) A.bounce_hit[(size_t)opix * A.bounces + i] = -2;
        }
        const unsigned long long am = uni64(__ballot(active));
        if (am == 0ull) break;  // (no pixel pending and no tile left: idle lanes found nothing)
        u.prim += (unsigned)__builtin_popcountll(uni64(__ballot(active && it == 0)));
        u.refl += (unsigned)__builtin_popcountll(uni64(__ballot(active && it > 0)));
        if (COUNT) c.lvl = (unsigned)it;
        // one level of every active path: the closest hit (raytracer.c:101-147 as path_step)
        int hit = -1;
        bool nd_side = false, ends = false, tail = false;
        unsigned okm = 0;
        if (active) {
            float best;
            int nd;
            const int orig = closest<false, COUNT, true>(s, o, d, best, nd, stk, c, sstk, wcap, it > 0);
            if (it == 0) {
                if (A.hit) A.hit[opix] = orig;
                if (A.t) A.t[opix] = best;
            }
            if (A.bounce_hit) A.bounce_hit[(size_t)opix * A.bounces + it] = orig;
            if (orig < 0) {  // raytracer.c:132-135
                pb[it * 64] = make_float4(0.0f + amb.x, 0.0f + amb.y, 0.0f + amb.z, __int_as_float(0));
                ends = true;
            } else {
                hit = orig;
                nd_side = nd != 0;
                const v3 ip = add(o, mul(d, best));
                const v3 n = xyz(s.shade[2 * orig + (nd ? 1 : 0)]);
                for (int j = 0; j < s.n_lights; ++j) {  // light_v's back-face test (raytracer.c:66-67)
                    const v3 tmp2 = sub(xyz(s.lights[2 * j]), ip);
                    okm |= dot(tmp2, n) < 0 ? 0u : (1u << j);
                }
                pb[it * 64] = make_float4(ip.x, ip.y, ip.z, __uint_as_float(0u));
            }
        }
        const unsigned nh = popc_wave(hit >= 0);
        u.hits += nh;
        if (nh) {  // the shadow rays of every hit, whatever its level, as one pool
            u.skip += nh * (unsigned)s.n_lights;
            const unsigned sh0 = u.shad;
            shadow_pool<COUNT>(s, okm, pbw, it * 64 + lane, stk, sstk, wcap, A.regroup, c, u);
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
                const int V = (int)((vis >> j) & 1u);
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
                ends = true;
            } else if (it + 1 == A.bounces) {  // raytrace(.., BOUNCES) returns {0,0,0}: col += kr * 0
                ends = true;
                tail = true;
            } else {
                o = ip;
                d = r;
            }
        }
        if (ends) {  // the path's pixel: the levels folded deepest-first, clamped, stored; the lane is free again
            const v3 col = clamp01(fold_pb<MAXB>(s, pb, it + 1, tail));
            store_px(A.rgb, A.bgra, (size_t)opix, col);
            active = false;
        } else if (active) {
            ++it;
        }
    }
    flush<COUNT>(c, A.counters);
    flush_u(u, A.counters);
    if constexpr (COUNT) {  // every wave of the workgroup leaves the loop and reaches this point
        __syncthreads();
        if (threadIdx.x < 32 && c.hist[threadIdx.x]) atomicAdd(A.counters + C_HIST + threadIdx.x, (unsigned long long)c.hist[threadIdx.x]);
    }
}

}  // namespace rtd
