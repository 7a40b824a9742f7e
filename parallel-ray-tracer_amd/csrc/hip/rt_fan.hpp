// rt_fan.hpp — shadow fan-out: R lanes per pixel, one traces the path's closest-hit chain, the other
// R - 1 trace its shadow rays one bounce level behind.
//
// Why: a frame (or a frame's 1/N on N GPUs) ends when its slowest tile does, and a tile's time is the
// dependent chain of its pixels' traversals. Per bounce level the reference traces one closest-hit ray
// and one shadow ray per light (raytracer.c:149-173); on the bench frame a closest-hit walk takes 6.4
// wide-node visits and a shadow walk 13.4, so with 2 lights ~80 % of a path's chain is shadow walks —
// which nothing else in the path waits for: the reflection ray of level i + 1 needs only level i's hit.
// Here lane 0 of a pixel's group walks level i + 1's closest hit WHILE lanes 1..L walk level i's
// shadow rays (one light each), all in one unified walk loop (a lane's mode is data, so the wave does
// not serialise the two kinds). A path's chain becomes (levels + 1) x max(closest, shadow) visits
// instead of levels x (closest + L x shadow).
//
// Bit-exactness: every quantity is computed by the same expressions as path_step (rt_kernels.hpp):
// the shadow lane receives the level's hit point, normal, direction and material from lane 0 as bit
// copies (__shfl), forms  term = ((V * kl) * cr) / mg  — the reference's
// col + V*kl*cr/mg  (raytracer.c:157-159) minus the final add — and lane 0 adds the terms to the level's
// colour in light order. The unified walk is closest_wide / visible_wide with the mode as a lane flag;
// ties and zero direction components take the same strict walks.
#pragma once
#include "rt_coop.hpp"

namespace rtd {

// closest_wide (shadow = false) or visible_wide (shadow = true) in one loop. Closest: best, hp, nd, tie
// as closest_wide. Shadow: occ = the ray is occluded (visible_wide returned false).
template <bool COUNT>
__device__ __forceinline__ void walk_unified(const DWide& W, v3 o, v3 d, bool shadow, float ld2, float& best, int& hp,
                                             int& nd, bool& tie, bool& occ, int* __restrict__ stk, Ctr& c) {
    const RayPre p = ray_pre(o, d);
    const unsigned oct = (p.ix < 0.0f ? 1u : 0u) | (p.iy < 0.0f ? 2u : 0u) | (p.iz < 0.0f ? 4u : 0u);
    const float reach = shadow ? shadow_reach(o, ld2) : FMAX;
    best = FMAX;
    hp = -1;
    nd = 0;
    tie = false;
    occ = false;
    int sp = 0;
    WNode N = wload(W, 0);
    for (;;) {
        unsigned nh, th, imask, nl;
        int cb, tb;
        const float lim = shadow ? fminf(best * PRUNE_SLACK, reach) : best * PRUNE_SLACK;
        wide_node<COUNT>(N, p, oct, lim, nh, th, cb, tb, imask, nl);
        if (COUNT) {
            if (shadow) {
                c.shi++;
                c.shl += nl;
            } else {
                c.chi++;
                c.chl += nl;
            }
            c.nb += 10;
            c.ws += first_active_lane();
        }
        const int next = wide_next(nh, cb, imask, oct, sp, stk);
        N = wload(W, next >= 0 ? next : 0);  // unconditional (rt_kernels.hpp closest_wide)
        while (th) {
            const int i = tb + __builtin_ctz(th);
            th &= th - 1u;
            int k;
            const float tt = hit_triangle(o, d, W.tris + 3 * i, k);
            if (COUNT) {
                if (shadow) c.sht++;
                else c.cht++;
            }
            if (tt < best) {
                best = tt;
                nd = k;
                hp = i;
                tie = false;
                if (shadow) {
                    const v3 ip = add(o, mul(d, best));
                    const v3 oi = sub(o, ip);
                    if (ld2 > dot(oi, oi)) {
                        occ = true;
                        break;
                    }
                }
            } else if (tt == best && tt != FMAX) {
                tie = true;
            }
        }
        if (occ) break;
        if (next < 0) {
            if (next == -2) c.err++;
            break;
        }
    }
}

__device__ __forceinline__ float shfl_f(float v, int src) { return __shfl(v, src, 64); }
__device__ __forceinline__ v3 shfl3(v3 v, int src) { return mk(shfl_f(v.x, src), shfl_f(v.y, src), shfl_f(v.z, src)); }

// Persistent waves pulling TW x TH pixel tiles (GTile<R>: 64 / R pixels); lane = (pixel lane / R, role
// lane % R). Role 0 owns the pixel's path (path_step's state), role j in 1..R-1 the shadow ray toward
// light j - 1 (the host launches this kernel only for 1 <= lights <= R - 1).
template <int MAXB, bool COUNT, int R, int OCC = 3, bool TRACE = false, bool BATCH = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, BLOCK), amdgpu_waves_per_eu(OCC))) void k_fan(KArgs A) {
    __shared__ int lds[STACK * BLOCK];
    int* stk = lds + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const int role = lane % R, pi = lane / R;
    const int src = lane - role;  // __shfl source: the group's role-0 lane
    constexpr int TW = GTile<R>::TW, TH = GTile<R>::TH;
    const DScene& s = A.s;
    const v3 amb = mk(s.amb_x, s.amb_y, s.amb_z);
    const int lj = role - 1;  // this lane's light (shadow roles)
    const bool has_light = role > 0 && lj < s.n_lights;
    v3 Lp = mk(0.0f, 0.0f, 0.0f), kl = Lp;
    if (has_light) {
        Lp = xyz(s.lights[2 * lj]);
        kl = xyz(s.lights[2 * lj + 1]);
    }
    Ctr c = {};
    const unsigned items = (unsigned)A.n_tiles * (unsigned)A.n_frames;  // frame batches: as k_persist
    for (;;) {
        unsigned t = 0;
        if (lane == 0) t = atomicAdd(A.work, 1u);
        t = __builtin_amdgcn_readfirstlane(__shfl(t, 0, 64));
        if (t >= items) break;
        const int frame = (int)(t % (unsigned)A.n_frames);
        unsigned tile = t / (unsigned)A.n_frames;
        if (A.tile_order) tile = (unsigned)A.tile_order[tile];
        const Cam C = cam_of<BATCH>(A, frame);
        const int tx = (int)(tile % (unsigned)A.tiles_x), ty = (int)(tile / (unsigned)A.tiles_x);
        const int x = tx * TW + pi % TW, k = ty * TH + pi / TW;
        const int y = image_row(A, k, frame);
        const bool valid = x < A.W && k < A.n_rows && y < A.H;  // uniform in the group
        unsigned long long tr0 = 0;
        const unsigned fb0 = c.fb, ws0 = c.ws, nd0 = c.chi + c.shi;
        if (TRACE) tr0 = __builtin_amdgcn_s_memrealtime();
        const size_t po = (size_t)frame * A.frame_px + (size_t)k * A.W + x;
        if (valid && role == 0 && A.bounce_hit)
            for (int i = 0; i < A.bounces; i++) A.bounce_hit[po * (size_t)A.bounces + i] = -2;
        const int g = A.spp <= 1 ? 1 : A.spp_grid;
        v3 acc = mk(0.0f, 0.0f, 0.0f), col1 = acc;
        int hit0 = -1;
        float t0 = FMAX;
        for (int sj = 0; sj < g; ++sj)
            for (int si = 0; si < g; ++si) {
                // ---- role 0: the path (trace_path's state)
                const float fx = g == 1 ? (float)x : (float)x + ((float)si + 0.5f) / (float)g;
                const float fy = g == 1 ? (float)y : (float)y + ((float)sj + 0.5f) / (float)g;
                v3 o = C.pos, d = primary_dir(C, fx, fy);
                v3 cols[MAXB];
                int mats[MAXB];
#pragma unroll
                for (int q = 0; q < MAXB; q++) {
                    cols[q] = mk(0.0f, 0.0f, 0.0f);
                    mats[q] = 0;
                }
                int L = 0, h0 = -1;
                bool tail = false, alive = valid && role == 0;
                float tt0 = FMAX;
                const int bh_pix = (si == 0 && sj == 0) ? (int)po : -1;
                // ---- shadow roles: the pending ray of the previous level and its light factors
                bool pend = false;
                v3 sip = mk(0.0f, 0.0f, 0.0f), sl = sip, scr = sip;
                float sld2 = 0.0f, smg = 1.0f;
                int prev = -1;  // level whose light terms are in flight (role 0: to accumulate)
                for (int phase = 0;; ++phase) {
                    if (!__ballot(alive || pend || prev >= 0)) break;
                    const bool tr = alive || pend;
                    const bool shadow = role != 0;
                    const v3 ro = shadow ? sip : o, rd = shadow ? sl : d;
                    float best = FMAX;
                    int hp = -1, nd = 0;
                    bool tie = false, occ = false;
                    if (tr) {
                        if (shadow) c.shad++;
                        else if (phase == 0) c.prim++;
                        else c.refl++;
                    }
                    const bool degen = tr && degenerate(rd);
                    if (tr && !degen) walk_unified<COUNT>(s.wide, ro, rd, shadow, sld2, best, hp, nd, tie, occ, stk, c);
                    int orig = hp >= 0 ? s.wide.tri_orig[hp] : -1;
                    if (tr && (degen || (!shadow && tie))) {  // the reference's answer via its own walk
                        c.fb++;
                        if (shadow) {
                            occ = !visible_walk<true, COUNT, true>(s.ref, ro, rd, sld2, stk, c);
                        } else {
                            best = FMAX;
                            hp = -1;
                            nd = 0;
                            closest_walk<true, COUNT, true>(s.ref, ro, rd, best, hp, nd, tie, stk, c);
                            orig = hp >= 0 ? s.ref.tri_orig[hp] : -1;
                        }
                    }
                    // ---- shadow lanes: the light term of level `prev` (raytracer.c:157-159 without the add)
                    v3 term = mk(0.0f, 0.0f, 0.0f);
                    if (shadow && pend) {
                        const float fV = occ ? 0.0f : 1.0f;
                        term = mk(fV * kl.x * scr.x / smg, fV * kl.y * scr.y / smg, fV * kl.z * scr.z / smg);
                        pend = false;
                    } else if (shadow && has_light && prev >= 0) {  // back-facing (V = 0) at level prev
                        term = mk(0.0f * kl.x * scr.x / smg, 0.0f * kl.y * scr.y / smg, 0.0f * kl.z * scr.z / smg);
                    }
                    // ---- role 0: add level prev's light terms in light order (all lanes active here)
                    const int pv = __shfl(prev, src, 64);
                    v3 cp = mk(0.0f, 0.0f, 0.0f);
#pragma unroll
                    for (int q = 0; q < MAXB; q++)
                        if (q == pv) cp = cols[q];
                    for (int j = 0; j < s.n_lights; ++j) {
                        const v3 tj = shfl3(term, src + 1 + j);
                        cp.x = cp.x + tj.x;
                        cp.y = cp.y + tj.y;
                        cp.z = cp.z + tj.z;
                    }
                    if (role == 0 && pv >= 0) set3<MAXB>(cols, pv, cp);
                    // ---- role 0: the closest hit of level `phase` (path_step)
                    bool hl = false;
                    v3 hip = mk(0.0f, 0.0f, 0.0f), hn = hip, hd = hip;
                    int hm = 0;
                    if (alive) {
                        if (phase == 0) {
                            h0 = orig;
                            tt0 = best;
                        }
                        if (A.bounce_hit && bh_pix >= 0) A.bounce_hit[(size_t)bh_pix * A.bounces + phase] = orig;
                        if (orig < 0) {  // raytracer.c:132-135
                            set3<MAXB>(cols, phase, mk(0.0f + amb.x, 0.0f + amb.y, 0.0f + amb.z));
                            L = phase + 1;
                            tail = false;
                            alive = false;
                        } else {
                            c.hits++;
                            const v3 ip = add(o, mul(d, best));  // raytracer.c:137-138
                            const float4 sh0 = s.shade[2 * orig], sh1 = s.shade[2 * orig + 1];
                            const int m = __float_as_int(sh0.w);
                            const v3 n = nd ? xyz(sh1) : xyz(sh0);
                            const v3 kd = xyz(s.mats[3 * m + 1]), kr = xyz(s.mats[3 * m + 2]);
                            set3<MAXB>(cols, phase, mk(0.0f + kd.x * amb.x, 0.0f + kd.y * amb.y, 0.0f + kd.z * amb.z));
                            seti<MAXB>(mats, phase, m);
                            hl = true;
                            hip = ip;
                            hn = n;
                            hd = d;
                            hm = m;
                            const v3 v = mul(d, -1.0f);
                            const v3 dd = mul(v, -1.0f);  // raytracer.c:163-166
                            const v3 ns = mul(n, 2.0f * __builtin_fabsf(dot(dd, n)));
                            const v3 r = normalize(add(dd, ns));
                            if (!(mag(kr) > 0.0f)) {  // raytracer.c:168
                                L = phase + 1;
                                tail = false;
                                alive = false;
                            } else if (phase + 1 == A.bounces) {  // raytrace(.., BOUNCES) returns {0,0,0}
                                L = phase + 1;
                                tail = true;
                                alive = false;
                            } else {
                                o = ip;
                                d = r;
                            }
                        }
                    }
                    // ---- hand-off: level `phase`'s hit to the shadow lanes (all lanes active here)
                    const bool ghl = __shfl(hl ? 1 : 0, src, 64) != 0;
                    const v3 gip = shfl3(hip, src), gn = shfl3(hn, src), gd = shfl3(hd, src);
                    const int gm = __shfl(hm, src, 64);
                    prev = ghl ? phase : -1;
                    if (shadow && has_light && ghl) {  // light_v + lambert_blinn factors, raytracer.c:149-156
                        const v3 ks = xyz(s.mats[3 * gm]), kd = xyz(s.mats[3 * gm + 1]);
                        const v3 v = mul(gd, -1.0f);
                        v3 l = sub(Lp, gip);
                        float mg = mag(l);
                        l = dvs(l, mg);
                        mg *= mg;
                        const float ndl = dot(gn, l);
                        const v3 h = normalize(add(l, v));
                        const float coeff = fmaxf(0.0f, dot(gn, h));
                        scr = mk(kd.x * fmaxf(0.0f, ndl) + ks.x * coeff, kd.y * fmaxf(0.0f, ndl) + ks.y * coeff,
                                 kd.z * fmaxf(0.0f, ndl) + ks.z * coeff);
                        smg = mg;
                        const v3 tmp = sub(gip, Lp), tmp2 = sub(Lp, gip);
                        sld2 = dot(tmp, tmp);
                        if (dot(tmp2, gn) < 0) {
                            c.skip++;  // V = 0: term formed next phase without a walk
                        } else {
                            pend = true;
                            sip = gip;
                            sl = l;
                        }
                    }
                }
                if (role == 0 && valid) {
                    const v3 cs = clamp01(fold_path<MAXB>(s, cols, mats, L, tail));
                    acc = add(acc, cs);
                    if (si == 0 && sj == 0) {
                        hit0 = h0;
                        t0 = tt0;
                        col1 = cs;
                    }
                }
            }
        if (role == 0 && valid) {
            c.pix++;
            v3 col = col1;
            if (A.spp > 1) {
                const float nn = (float)(g * g);
                col = mk(acc.x / nn, acc.y / nn, acc.z / nn);
            }
            store_px(A.rgb, A.bgra, po, col);
            if (A.hit) A.hit[po] = hit0;
            if (A.t) A.t[po] = t0;
        }
        if (TRACE) {  // as k_persist's: {begin, end, wave | fallbacks << 32, wave steps | lane node visits << 32}
            const unsigned fb = wave_sum(c.fb - fb0), ws = wave_sum(c.ws - ws0), nv = wave_sum(c.chi + c.shi - nd0);
            if (lane == 0) {
                A.tile_trace[4 * tile] = tr0;
                A.tile_trace[4 * tile + 1] = __builtin_amdgcn_s_memrealtime();
                A.tile_trace[4 * tile + 2] = (blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6)) | ((unsigned long long)fb << 32);
                A.tile_trace[4 * tile + 3] = ws | ((unsigned long long)nv << 32);
            }
        }
    }
    flush<COUNT>(c, A.counters);
}

}  // namespace rtd
