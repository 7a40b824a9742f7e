// rt_chain.hpp — k_chain: one lane = one pixel's whole path, its walks run back to back.
//
// k_persist runs a tile's paths in lockstep by walk: every lane does level 0's closest-hit walk, then
// light 0's shadow walk, then light 1's, then level 1's closest walk ... and each of those walks lasts
// as long as its slowest lane. Measured per lane and per walk on the bench frame (round 2, one 1080p
// frame, a diagnostic build recording each walk's wide-node visits per pixel): 1.666 M wave
// steps for 59.98 M lane visits,
// SIMD efficiency 0.56; shadow walks are 69 % of the steps (2 lights through the knot). The paths of a
// tile differ little in LENGTH (lanes alive per level: 100 / 94 / 71 / 48 %, 0.92 of the tile's
// level-slots used), but a lane's walks differ a lot in COST, and lockstep pays the maximum of every walk.
//
// k_chain keeps the tile (one 8x8 pixel tile per wave, the same dealing as k_persist, so the rays of a
// wave stay neighbours) but lets every lane run its own chain of walks: closest-hit and shadow rays
// share ONE wide-BVH step loop (the same node test, a per-lane flag picks the leaf handling), and a
// lane whose walk ends moves to its next walk on its own — the wave pays the maximum over lanes of the
// SUM of each lane's walks instead of the sum of the maxima: 0.79x the wave steps on the same frame
// (SIMD efficiency 0.71), the slowest tile 738 -> 454 steps. Stage transitions (shading a hit, the
// light loop, the reflection, the fold, the next spp sample) are batched by ballot: lanes whose walk
// ended wait until `regroup` lanes are waiting (or no lane is walking), then all of them advance
// together, so the transition code runs with many lanes at once instead of once per finishing lane.
//
// Arithmetic is path_step / fold_pb / render_pixel's (rt_kernels.hpp), expression for expression, in
// the reference's order (raytracer.c:101-177, main.c:228-239): bit-exact to the other kernels. The rare
// strict re-walks (a zero direction component, an exact tie) are out of line.
//
// Measured (round 2, same box, tools/ab_variants.py, 16-frame batches, ms per frame): the step count
// drops as modelled (regroup 1: 1.316 M wave steps vs 1.660 M, SIMD efficiency 0.71; regroup 8: 0.65),
// but each step costs more than k_persist's: one loop serves both walk kinds (the closest walk's
// bookkeeping runs on shadow lanes too: ~460 instructions per step against ~340 for k_persist's mostly
// shadow steps on dragon), a wave mixes closest and shadow rays of different levels (less coherent node
// loads), and the transitions run ~10-20 passes per tile instead of one per walk. dragon 1.26 vs 0.92,
// car_boxed 1.52 vs 1.02: a variant (RT_VARIANT_CHAIN / CHAIN4) and a tuning candidate, not the default.
#pragma once
#include "rt_kernels.hpp"

namespace rtd {

struct StrictC {  // result of an out-of-line strict closest walk, counters returned by value
    int orig, nd;
    float best;
    unsigned chi, chl, cht, err;
};

template <bool COUNT>
__device__ __noinline__ StrictC chain_strict_closest(const DBvh B, v3 o, v3 d, int* __restrict__ bstk) {
    Ctr c = {};
    float best = FMAX;
    int hp = -1, nd = 0;
    bool tie = false;
    closest_walk<true, COUNT, true>(B, o, d, best, hp, nd, tie, bstk, c);
    return StrictC{hp >= 0 ? B.tri_orig[hp] : -1, nd, best, c.chi, c.chl, c.cht, c.err};
}

template <bool COUNT>
__device__ __noinline__ unsigned chain_strict_visible(const DBvh B, v3 o, v3 d, float ld2, int* __restrict__ bstk) {
    // bit 31: visible; bits 0..30: interior visits (COUNT; leaf / triangle counts are not kept)
    Ctr c = {};
    const bool v = visible_walk<true, COUNT, true>(B, o, d, ld2, bstk, c);
    return (v ? 0x80000000u : 0u) | (c.shi & 0x7FFFFFFFu);
}

// lane states
enum : int {
    CH_DONE = 0,
    CH_WALK_C = 1,   // closest-hit walk in progress
    CH_WALK_S = 2,   // shadow walk in progress
    CH_C_END = 3,    // closest walk finished (hp, best, nd, tie)
    CH_SAMPLE = 4,   // start sample `si` of the pixel (primary ray)
    CH_CLOSEST = 5,  // start a closest-hit walk for (o, d) at level `it`
    CH_LIGHT = 6,    // light `j` of the hit at level `it`
    CH_S_END = 7,    // shadow walk of light `j` finished (occ)
    CH_LEVEL = 8,    // all lights done: the level's colour, the reflection
    CH_PATH = 9,     // path ended: fold, clamp, next sample or the pixel
    CH_HIT = 10      // closest hit resolved: hp = original triangle (-1: miss), best, nd
};

// OCC: waves per SIMD the register allocation must allow (3: <= 168 VGPRs, 4: <= 128). LDS per workgroup
// (dynamic): the wide walk's stack, 2 * wcap ints per lane ([depth][lane], 64 distinct banks per wave),
// then the path buffer [wave][level][lane] float4 (each level's colour + material, read by the fold).
// The strict fallbacks' binary stacks live in global memory (A.gstack).
template <int MAXB, bool COUNT, int OCC, bool BATCH>
__global__ __attribute__((amdgpu_flat_work_group_size(1, BLOCK), amdgpu_waves_per_eu(OCC))) void k_chain(KArgs A) {
    extern __shared__ int lds_dyn[];
    const int wcap = A.wcap;
    int* stk = lds_dyn + threadIdx.x;
    float4* pb = (float4*)(lds_dyn + 2 * wcap * BLOCK) + (size_t)((threadIdx.x >> 6) * MAXB) * 64 + (threadIdx.x & 63);
    int* bstk = A.gstack + (size_t)blockIdx.x * STACK * BLOCK + threadIdx.x;
    const DScene& s = A.s;
    const DWide& W = s.wide;
    const int lane = threadIdx.x & 63;
    const v3 amb = mk(s.amb_x, s.amb_y, s.amb_z);
    const int regroup = A.regroup;
    Ctr c = {};
    int reg = 0;

    // ---- per-lane state (hot: the walk; cold: the path, touched only by the transitions)
    int ph = CH_DONE;
    int it = 0, j = 0, si = 0, L = 0;
    bool tail = false, occ = false, tie = false;
    int pxk = 0;  // pixel: x | compact row k << 16 (the output index and the image row follow from it)
    int frame = 0;
    v3 acc = mk(0.0f, 0.0f, 0.0f);
    v3 o = acc, d = acc, vin = acc, n = acc, col = acc;
    int m = 0;
    float ld2 = 0.0f, best = FMAX;
    int hp = -1, nd = 0, sp = 0, nxt = 0;
    Cam C = cam_of<false>(A, 0);

    for (;;) {
        // ---- the wave's next tile once every lane is done (one item = one 8x8 tile of one frame)
        if (!__ballot(ph != CH_DONE)) {
            unsigned tile;
            if (!next_item(A, lane, reg, frame, tile)) break;
            C = cam_of<BATCH>(A, frame);
            const int tx = (int)(tile % (unsigned)A.tiles_x), ty = (int)(tile / (unsigned)A.tiles_x);
            const int x = tx * 8 + (lane & 7), k = ty * 8 + (lane >> 3);
            const int y = k < A.n_rows ? image_row(A, k, frame) : A.H;
            if (x < A.W && k < A.n_rows && y < A.H) {  // frame_shift: compact rows past the image are skipped
                pxk = x | (k << 16);
                si = 0;
                acc = mk(0.0f, 0.0f, 0.0f);
                const size_t po = (size_t)frame * A.frame_px + (size_t)k * A.W + x;
                if (A.bounce_hit)
                    for (int i = 0; i < A.bounces; i++) A.bounce_hit[po * (size_t)A.bounces + i] = -2;
                if (A.hit) A.hit[po] = -1;
                if (A.t) A.t[po] = FMAX;
                ph = CH_SAMPLE;
            }
            continue;
        }
        // ---- stage transitions, batched: only when `regroup` lanes wait or nobody walks
        const unsigned long long waiting = __ballot(ph >= CH_C_END);
        const unsigned long long walking = __ballot(ph == CH_WALK_C || ph == CH_WALK_S);
        if (waiting && (!walking || __popcll(waiting) >= (unsigned)regroup)) {
            // One pass in pipeline order, each stage's code runs at most once per pass (the light loop once
            // per consecutive back-facing light): walk ends -> hits -> lights -> level end -> path end -> new
            // sample -> next closest-hit walk. A lane whose strict fallback resolves a hit at the last stage
            // keeps waiting for the next pass.
            const int px = pxk & 0xFFFF, pk = pxk >> 16;
            const size_t po = (size_t)frame * A.frame_px + (size_t)pk * A.W + px;
            if (ph == CH_C_END) {
                if (tie) {  // exact tie: the reference keeps the first triangle found (bvh.c:331)
                    c.fb++;
                    const StrictC r = chain_strict_closest<COUNT>(s.ref, o, d, bstk);
                    if (COUNT) {
                        c.chi += r.chi;
                        c.chl += r.chl;
                        c.cht += r.cht;
                        c.nb += 8 * r.chi + r.chl;
                    }
                    c.err += r.err;
                    hp = r.orig;
                    nd = r.nd;
                    best = r.best;
                } else {
                    hp = hp >= 0 ? W.tri_orig[hp] : -1;
                }
                ph = CH_HIT;
            }
            if (ph == CH_HIT) {  // raytracer.c:130-147
                if (si == 0) {
                    if (it == 0) {
                        if (A.hit) A.hit[po] = hp;
                        if (A.t) A.t[po] = best;
                    }
                    if (A.bounce_hit) A.bounce_hit[po * (size_t)A.bounces + it] = hp;
                }
                if (hp < 0) {  // raytracer.c:132-135
                    pb[it * 64] = make_float4(0.0f + amb.x, 0.0f + amb.y, 0.0f + amb.z, __int_as_float(0));
                    L = it + 1;
                    tail = false;
                    ph = CH_PATH;
                } else {
                    c.hits++;
                    vin = d;
                    o = add(o, mul(d, best));  // the hit point, raytracer.c:137-138
                    const float4 sh0 = s.shade[2 * hp], sh1 = s.shade[2 * hp + 1];
                    m = __float_as_int(sh0.w);
                    n = nd ? xyz(sh1) : xyz(sh0);
                    const v3 kd0 = xyz(s.mats[3 * m + 1]);
                    col = mk(0.0f + kd0.x * amb.x, 0.0f + kd0.y * amb.y, 0.0f + kd0.z * amb.z);  // :144-146
                    j = 0;
                    ph = CH_LIGHT;
                }
            }
            // the light loop (raytracer.c:149-160): a finished shadow walk's term, then the next light's shadow
            // ray (light_v, :62-99); back-facing lights and strict fallbacks resolve at once and loop
            while (ph == CH_S_END || ph == CH_LIGHT) {
                if (ph == CH_S_END) {  // lambert_blinn and the light's term (raytracer.c:21-33,157-159)
                    const v3 Lp = xyz(s.lights[2 * j]);
                    v3 l = sub(Lp, o);
                    float mg = mag(l);
                    l = dvs(l, mg);
                    mg *= mg;
                    const v3 v = mul(vin, -1.0f);
                    const v3 kl = xyz(s.lights[2 * j + 1]);
                    const v3 ks = xyz(s.mats[3 * m]), kd = xyz(s.mats[3 * m + 1]);
                    const float ndl = dot(n, l);
                    const v3 h = normalize(add(l, v));
                    const float coeff = fmaxf(0.0f, dot(n, h));
                    const v3 cr = mk(kd.x * fmaxf(0.0f, ndl) + ks.x * coeff, kd.y * fmaxf(0.0f, ndl) + ks.y * coeff,
                                     kd.z * fmaxf(0.0f, ndl) + ks.z * coeff);
                    const float fV = occ ? 0.0f : 1.0f;
                    col.x = col.x + fV * kl.x * cr.x / mg;
                    col.y = col.y + fV * kl.y * cr.y / mg;
                    col.z = col.z + fV * kl.z * cr.z / mg;
                    j++;
                }
                if (j >= s.n_lights) {
                    ph = CH_LEVEL;
                } else {
                    const v3 Lp = xyz(s.lights[2 * j]);
                    v3 l = sub(Lp, o);
                    const float mg = mag(l);
                    l = dvs(l, mg);
                    const v3 tmp = sub(o, Lp), tmp2 = sub(Lp, o);
                    ld2 = dot(tmp, tmp);
                    ph = CH_S_END;
                    if (dot(tmp2, n) < 0) {
                        c.skip++;
                        occ = true;  // V = 0
                    } else {
                        c.shad++;
                        if (degenerate(l)) {
                            c.fb++;
                            const unsigned r = chain_strict_visible<COUNT>(s.ref, o, l, ld2, bstk);
                            if (COUNT) {
                                c.shi += r & 0x7FFFFFFFu;
                                c.nb += 8 * (r & 0x7FFFFFFFu);
                            }
                            occ = (r >> 31) == 0u;
                        } else {  // the shadow walk: o = the hit point, d = l
                            d = l;
                            best = FMAX;
                            occ = false;
                            sp = 0;
                            nxt = 0;
                            ph = CH_WALK_S;
                        }
                    }
                }
            }
            if (ph == CH_LEVEL) {  // raytracer.c:162-173
                const v3 v = mul(vin, -1.0f);
                const v3 dd = mul(v, -1.0f);
                const v3 ns = mul(n, 2.0f * __builtin_fabsf(dot(dd, n)));
                const v3 r = normalize(add(dd, ns));
                pb[it * 64] = make_float4(col.x, col.y, col.z, __int_as_float(m));
                const v3 kr = xyz(s.mats[3 * m + 2]);
                if (!(mag(kr) > 0.0f)) {
                    L = it + 1;
                    tail = false;
                    ph = CH_PATH;
                } else if (it + 1 == A.bounces) {  // raytrace(.., BOUNCES) returns {0,0,0}: col += kr * 0
                    L = it + 1;
                    tail = true;
                    ph = CH_PATH;
                } else {
                    d = r;
                    it++;
                    c.refl++;
                    ph = CH_CLOSEST;
                }
            }
            if (ph == CH_PATH) {  // fold deepest-first, clamp; the next sample or the pixel
                const v3 cs = clamp01(fold_pb<MAXB>(s, pb, L, tail));
                if (A.spp <= 1) {
                    col = cs;
                    ph = CH_DONE;
                } else {
                    acc = add(acc, cs);
                    si++;
                    if (si < A.spp) {
                        ph = CH_SAMPLE;
                    } else {
                        const float nn = (float)(A.spp_grid * A.spp_grid);
                        col = mk(acc.x / nn, acc.y / nn, acc.z / nn);
                        ph = CH_DONE;
                    }
                }
                if (ph == CH_DONE) {
                    c.pix++;
                    store_px(A.rgb, A.bgra, po, col);
                }
            }
            if (ph == CH_SAMPLE) {  // render_pixel, main.c:228-239 (+ stratified sub-pixel samples)
                float fx = (float)px, fy = (float)image_row(A, pk, frame);
                if (A.spp > 1) {
                    const int g = A.spp_grid;
                    fx = fx + ((float)(si % g) + 0.5f) / (float)g;
                    fy = fy + ((float)(si / g) + 0.5f) / (float)g;
                }
                o = C.pos;
                d = primary_dir(C, fx, fy);
                it = 0;
                c.prim++;
                ph = CH_CLOSEST;
            }
            if (ph == CH_CLOSEST) {
                if (degenerate(d)) {  // the reference's 0/0 NaN slabs: strict walk from the start
                    c.fb++;
                    const StrictC r = chain_strict_closest<COUNT>(s.ref, o, d, bstk);
                    if (COUNT) {
                        c.chi += r.chi;
                        c.chl += r.chl;
                        c.cht += r.cht;
                        c.nb += 8 * r.chi + r.chl;
                    }
                    c.err += r.err;
                    hp = r.orig;
                    nd = r.nd;
                    best = r.best;
                    ph = CH_HIT;  // resolved in the next pass
                } else {
                    best = FMAX;
                    hp = -1;
                    nd = 0;
                    tie = false;
                    sp = 0;
                    nxt = 0;
                    ph = CH_WALK_C;
                }
            }
            continue;
        }
        // ---- the walks: wide-node steps of every walking lane (closest-hit and shadow walks together) until
        // `regroup` lanes wait for a transition or none walks. Only this loop is hot: the ray's reciprocals and
        // the node record are rebuilt on entry (a few instructions per lane per entry, against hundreds of
        // steps per tile), so nothing but the walk state is live across the transitions above.
        {
            const bool shw = ph == CH_WALK_S;
            RayPre p = {};
            unsigned oct = 0;
            float reach = 0.0f;
            WNode N = {};
            if (ph == CH_WALK_C || ph == CH_WALK_S) {
                p = ray_pre(o, d);
                oct = (p.ix < 0.0f ? 1u : 0u) | (p.iy < 0.0f ? 2u : 0u) | (p.iz < 0.0f ? 4u : 0u);
                if (shw) reach = shadow_reach(o, ld2);
                N = wload(W, nxt);
            }
            for (;;) {
                if (ph == CH_WALK_C || ph == CH_WALK_S) {
                    const float lim = shw ? fminf(best * PRUNE_SLACK, reach) : best * PRUNE_SLACK;  // as closest_wide / visible_wide
                    unsigned nh, th, imask, nl;
                    int cb, tb;
                    wide_node<COUNT>(N, p, oct, lim, nh, th, cb, tb, imask, nl);
                    if (COUNT) {
                        if (shw) {
                            c.shi++;
                            c.shl += nl;
                        } else {
                            c.chi++;
                            c.chl += nl;
                        }
                        c.nb += 10;
                        c.ws += first_active_lane();
                    }
                    const int next = wide_next(nh, cb, imask, oct, sp, stk, wcap);
                    nxt = next < 0 ? 0 : next;  // (a finished walk reloads the root: no branch)
                    N = wload(W, nxt);
                    bool end = next < 0;
                    if (next == -2) c.err++;
                    // leaf triangles, branch-free per triangle: the closest walk keeps the nearest (first found on
                    // ties, then flagged), the shadow walk stops at an occluder nearer than the light (bvh.c:283-290);
                    // a shadow lane's hp / nd / tie are dead (its hit was shaded before the walk)
                    while (th) {
                        const int i = tb + __builtin_ctz(th);
                        th &= th - 1u;
                        int k;
                        const float tt = hit_triangle(o, d, W.tris + 3 * i, k);
                        if (COUNT) {
                            if (shw) c.sht++;
                            else c.cht++;
                        }
                        const bool lt = tt < best;
                        const bool eq = tt == best && tt != FMAX;
                        best = lt ? tt : best;
                        hp = lt ? i : hp;
                        nd = lt ? k : nd;
                        tie = lt ? false : (tie || eq);
                        const v3 ip = add(o, mul(d, best));
                        const v3 oi = sub(o, ip);
                        occ = occ || (shw && lt && ld2 > dot(oi, oi));
                    }
                    end = end || (shw && occ);  // (occ of a closest walk is the last shadow walk's, unused)
                    if (end) ph = shw ? CH_S_END : CH_C_END;
                }
                const unsigned long long wk = __ballot(ph == CH_WALK_C || ph == CH_WALK_S);
                if (!wk || __popcll(__ballot(ph >= CH_C_END)) >= (unsigned)regroup) break;
            }
        }
    }
    flush<COUNT>(c, A.counters);
}

}  // namespace rtd
