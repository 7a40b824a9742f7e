// rt_wave.hpp — k_wave: the fast kernel as a persistent per-lane state machine.
//
// Why: with one thread per pixel running the whole recursion (k_persist), a wave idles on its slowest
// pixel at every stage (a miss ends a pixel after 1 ray, a reflective hit needs up to BOUNCES closest
// rays + one shadow ray per light each) and on the longest traversal of every ray. rocprof on the bench
// workload: ~20 % lane utilisation, 60 % of wave cycles waiting on memory at 3 waves/SIMD.
//
// How: every lane owns ONE ray at a time. The wave runs a single traversal loop (the only hot loop)
// over whatever rays its lanes hold - closest-hit and shadow rays share the loop - and leaves it only
// when fewer than `refill_below` lanes are still tracing. Then each finished lane advances its own
// path through the reference's stages (shade the hit, next light's shadow ray, reflection ray, fold +
// write the pixel, take the next pixel from a per-frame atomic counter) until it holds a new ray.
//
// Semantics are exactly those of rt_kernels.hpp's per-pixel path (same arithmetic in the same order;
// the strict reference walk is used for rays with a zero direction component and for closest hits
// ending on an exact tie). Pixels are dealt in 8x8 tiles (pixel id -> tile-major) so lanes that take
// consecutive ids trace neighbouring pixels.
#pragma once
#include "rt_kernels.hpp"

namespace rtd {

enum : int { PH_NONE = 0, PH_START, PH_CTRACE, PH_CDONE, PH_LIGHT, PH_STRACE, PH_SDONE, PH_REFLECT };

struct StrictHit {
    int og;
    int nd;
    float best;
};

// Rare paths (zero direction component, exact ties): kept out of line so that their registers do not
// inflate the traversal loop's allocation.
__device__ __noinline__ StrictHit strict_closest(const DBvh B, v3 o, v3 d, int* __restrict__ stk) {
    Ctr c = {};
    float best = FMAX;
    int hp = -1, nd = 0;
    bool tie = false;
    closest_walk<true, false>(B, o, d, best, hp, nd, tie, stk, c);
    return StrictHit{hp >= 0 ? B.tri_orig[hp] : -1, nd, best};
}

__device__ __noinline__ bool strict_visible(const DBvh B, v3 o, v3 d, float ld2, int* __restrict__ stk) {
    Ctr c = {};
    return visible_walk<true, false>(B, o, d, ld2, stk, c);
}

template <int MAXB>
__device__ __forceinline__ v3 get3(const v3 (&a)[MAXB], int i) {
    v3 r = a[0];
#pragma unroll
    for (int k = 1; k < MAXB; k++)
        if (k == i) r = a[k];
    return r;
}

template <int MAXB, bool COUNT>
__device__ __forceinline__ void wave_body(const KArgs& A, int* __restrict__ stk) {
    const DScene& s = A.s;
    const DBvh& acc = s.acc;
    const unsigned lane = threadIdx.x & 63;
    const unsigned n_ids = (unsigned)A.n_tiles * 64u;
    Ctr c = {};

    // ---- per-lane state
    int ph = PH_NONE;
    bool exhausted = false;
    int pix = 0;  // compact output index k*W + x
    int it = 0, j = 0, og = -1, nd = 0, hp = -1, sp = 0;
    bool tie = false, occl = false, tail = false;
    v3 o = mk(0, 0, 0), d = mk(0, 0, 0), din = mk(0, 0, 0), col = mk(0, 0, 0), cr = mk(0, 0, 0);
    float best = FMAX, ld2 = 0.0f, mg = 1.0f;
    RayPre p = {};
    v3 cols[MAXB];
    int mats[MAXB];
#pragma unroll
    for (int k = 0; k < MAXB; k++) {
        cols[k] = mk(0.0f, 0.0f, 0.0f);
        mats[k] = 0;
    }
    const v3 amb = mk(s.amb_x, s.amb_y, s.amb_z);

    for (;;) {
        // ================= advance: every lane not tracing moves its path forward =================
        for (;;) {
            // pixel fetch for idle lanes: one returning atomic per wave
            const unsigned long long need = __ballot(ph == PH_NONE && !exhausted);
            if (need) {
                unsigned base = 0;
                if (lane == (unsigned)__ffsll((long long)need) - 1) base = atomicAdd(A.work, (unsigned)__popcll(need));
                base = __shfl(base, __ffsll((long long)need) - 1, 64);
                if (ph == PH_NONE && !exhausted) {
                    const unsigned id = base + (unsigned)__popcll(need & ((1ull << lane) - 1ull));
                    if (id >= n_ids) {
                        exhausted = true;
                    } else {
                        const int tile = (int)(id >> 6), w = (int)(id & 63u);
                        const int x = (tile % A.tiles_x) * 8 + (w & 7), k = (tile / A.tiles_x) * 8 + (w >> 3);
                        if (x < A.W && k < A.n_rows) {
                            pix = k * A.W + x;
                            ph = PH_START;
                        }  // else: padding of an edge tile, stay NONE and fetch again
                    }
                }
            }
            const bool busy = ph != PH_NONE && ph != PH_CTRACE && ph != PH_STRACE;
            if (!__ballot(busy) && !__ballot(ph == PH_NONE && !exhausted)) break;
            if (!busy) continue;

            if (ph == PH_START) {  // render_pixel, main.c:228-239: primary ray
                const int k = pix / A.W, x = pix - k * A.W;
                const int y = image_row(A, k);
                o = mk(A.pos[0], A.pos[1], A.pos[2]);
                d = primary_dir(A, (float)x, (float)y);
                it = 0;
                tail = false;
                c.prim++;
                ph = PH_CTRACE;  // start closest ray (below)
            } else if (ph == PH_CDONE) {
                if (og == -2) {  // finished the fast walk: tie -> strict re-walk (bvh.c:331 first-found order)
                    if (tie) {
                        c.fb++;
                        const StrictHit h = strict_closest(s.ref, o, d, stk);
                        og = h.og;
                        nd = h.nd;
                        best = h.best;
                    } else {
                        og = hp >= 0 ? acc.tri_orig[hp] : -1;
                    }
                }
                if (it == 0) {
                    if (A.hit) A.hit[pix] = og;
                    if (A.t) A.t[pix] = best;
                }
                if (og < 0) {  // raytracer.c:132-135
                    set3<MAXB>(cols, it, mk(0.0f + amb.x, 0.0f + amb.y, 0.0f + amb.z));
                    const int L = it + 1;
                    // fold + clamp + write (below, shared with REFLECT's end)
                    v3 accum = mk(0.0f, 0.0f, 0.0f);
                    bool have = false;
#pragma unroll
                    for (int i = MAXB - 1; i >= 0; --i)
                        if (i < L) {
                            if (!have) {
                                accum = cols[i];
                                have = true;
                            } else {
                                const v3 kr = xyz(s.mats[3 * mats[i] + 2]);
                                accum = mk(cols[i].x + kr.x * accum.x, cols[i].y + kr.y * accum.y,
                                           cols[i].z + kr.z * accum.z);
                            }
                        }
                    const v3 cl = clamp01(accum);
                    store_px(A.rgb, A.bgra, (size_t)pix, cl);
                    c.pix++;
                    ph = PH_NONE;
                    continue;
                }
                c.hits++;
                o = add(o, mul(d, best));  // intersection, raytracer.c:137-138
                din = d;
                const int m = __float_as_int(s.shade[2 * og].w);
                seti<MAXB>(mats, it, m);
                const v3 kd = xyz(s.mats[3 * m + 1]);
                col = mk(0.0f + kd.x * amb.x, 0.0f + kd.y * amb.y, 0.0f + kd.z * amb.z);  // :144-146
                j = 0;
                ph = PH_LIGHT;
                continue;
            } else if (ph == PH_SDONE) {  // accumulate light j (raytracer.c:157-159)
                const v3 kl = xyz(s.lights[2 * j + 1]);
                const float fV = occl ? 0.0f : 1.0f;
                col.x = col.x + fV * kl.x * cr.x / mg;
                col.y = col.y + fV * kl.y * cr.y / mg;
                col.z = col.z + fV * kl.z * cr.z / mg;
                j++;
                ph = PH_LIGHT;
                continue;
            } else if (ph == PH_LIGHT) {  // raytracer.c:149-156 for light j, or the reflection
                if (j >= s.n_lights) {
                    ph = PH_REFLECT;
                    continue;
                }
                const int m = __float_as_int(s.shade[2 * og].w);
                const v3 n = xyz(s.shade[2 * og + nd]);
                const v3 ks = xyz(s.mats[3 * m]), kd = xyz(s.mats[3 * m + 1]);
                const v3 Lp = xyz(s.lights[2 * j]);
                const v3 v = mul(din, -1.0f);
                v3 l = sub(Lp, o);
                float mgl = mag(l);
                l = dvs(l, mgl);
                mgl *= mgl;
                const float ndl = dot(n, l);
                const v3 h = normalize(add(l, v));  // lambert_blinn, raytracer.c:21-33
                const float coeff = fmaxf(0.0f, dot(n, h));
                cr = mk(kd.x * fmaxf(0.0f, ndl) + ks.x * coeff, kd.y * fmaxf(0.0f, ndl) + ks.y * coeff,
                        kd.z * fmaxf(0.0f, ndl) + ks.z * coeff);
                mg = mgl;
                const v3 tmp = sub(o, Lp), tmp2 = sub(Lp, o);  // light_v, raytracer.c:62-74
                ld2 = dot(tmp, tmp);
                if (dot(tmp2, n) < 0) {
                    c.skip++;
                    occl = true;  // V = 0
                    ph = PH_SDONE;
                    continue;
                }
                c.shad++;
                if (degenerate(l)) {
                    c.fb++;
                    occl = !strict_visible(s.ref, o, l, ld2, stk);
                    ph = PH_SDONE;
                    continue;
                }
                d = l;
                p = ray_pre(o, d);
                best = FMAX;
                occl = false;
                sp = 1;
                stk[0] = acc.root;
                ph = PH_STRACE;
                continue;
            } else if (ph == PH_REFLECT) {  // raytracer.c:162-173
                const v3 n = xyz(s.shade[2 * og + nd]);
                const v3 dd = mul(mul(din, -1.0f), -1.0f);
                const v3 ns = mul(n, 2.0f * __builtin_fabsf(dot(dd, n)));
                const v3 r = normalize(add(dd, ns));
                set3<MAXB>(cols, it, col);
                const int m = __float_as_int(s.shade[2 * og].w);
                const v3 kr = xyz(s.mats[3 * m + 2]);
                const bool rec = mag(kr) > 0.0f;
                if (rec && it + 1 < A.bounces) {
                    it++;
                    d = r;
                    c.refl++;
                    ph = PH_CTRACE;  // start closest ray (below)
                } else {
                    tail = rec;  // raytrace(.., BOUNCES) returned {0,0,0}: col += kr * 0
                    const int L = it + 1;
                    v3 accum = mk(0.0f, 0.0f, 0.0f);
                    bool have = false;
#pragma unroll
                    for (int i = MAXB - 1; i >= 0; --i)
                        if (i < L) {
                            const v3 kri = xyz(s.mats[3 * mats[i] + 2]);
                            if (!have) {
                                accum = cols[i];
                                if (tail)
                                    accum = mk(accum.x + kri.x * 0.0f, accum.y + kri.y * 0.0f, accum.z + kri.z * 0.0f);
                                have = true;
                            } else {
                                accum = mk(cols[i].x + kri.x * accum.x, cols[i].y + kri.y * accum.y,
                                           cols[i].z + kri.z * accum.z);
                            }
                        }
                    const v3 cl = clamp01(accum);
                    store_px(A.rgb, A.bgra, (size_t)pix, cl);
                    c.pix++;
                    ph = PH_NONE;
                    continue;
                }
            }
            // ---- start a closest-hit ray (o, d): fast walk unless a direction component is zero
            if (ph == PH_CTRACE) {
                best = FMAX;
                hp = -1;
                nd = 0;
                tie = false;
                occl = false;
                if (degenerate(d)) {
                    c.fb++;
                    const StrictHit h = strict_closest(s.ref, o, d, stk);
                    og = h.og;
                    nd = h.nd;
                    best = h.best;
                    ph = PH_CDONE;
                } else {
                    og = -2;  // resolved at CDONE from hp
                    p = ray_pre(o, d);
                    sp = 1;
                    stk[0] = acc.root;
                }
            }
        }
        if (!__ballot(ph == PH_CTRACE || ph == PH_STRACE)) break;  // all lanes exhausted

        // ================= traversal: the hot loop, closest-hit and shadow rays together ============
        for (;;) {
            if (ph == PH_CTRACE || ph == PH_STRACE) {
                const bool shadow = ph == PH_STRACE;
                const int ref = stk[(--sp) * BLOCK];
                if (ref < 0) {
                    const int2 lf = acc.leaves[~ref];
                    if (COUNT) {
                        if (shadow) c.shl++;
                        else c.chl++;
                    }
                    for (int i = lf.x; i < lf.x + lf.y; ++i) {
                        int k;
                        const float tt = hit_triangle(o, d, acc.tris + 3 * i, k);
                        if (COUNT) {
                            if (shadow) c.sht++;
                            else c.cht++;
                        }
                        if (tt < best) {
                            best = tt;
                            if (!shadow) {  // a shadow ray must not clobber its hit's normal side
                                hp = i;
                                nd = k;
                                tie = false;
                            }
                            if (shadow) {  // bvh.c:283-290
                                const v3 ip = add(o, mul(d, best));
                                const v3 oi = sub(o, ip);
                                if (ld2 > dot(oi, oi)) {
                                    occl = true;
                                    break;
                                }
                            }
                        } else if (!shadow && tt == best && tt != FMAX) {
                            tie = true;
                        }
                    }
                } else {
                    if (COUNT) {
                        if (shadow) c.shi++;
                        else c.chi++;
                    }
                    const float4* N = acc.nodes + 4 * ref;
                    const float4 a = N[0], b = N[1], e = N[2], r = N[3];
                    int ni = __float_as_int(r.x), fi = __float_as_int(r.y);
                    float nt = box_fast(a.x, a.y, a.z, a.w, b.x, b.y, p);
                    float ft = box_fast(b.z, b.w, e.x, e.y, e.z, e.w, p);
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
                    if (sp + 2 > STACK) {
                        c.err++;
                        sp = 0;
                    } else {
                        const float lim = best * PRUNE_SLACK;
                        if (ft <= lim && ft != FMAX) stk[(sp++) * BLOCK] = fi;
                        if (nt <= lim && nt != FMAX) stk[(sp++) * BLOCK] = ni;
                    }
                }
                if (sp == 0 || (shadow && occl)) ph = shadow ? PH_SDONE : PH_CDONE;
            }
            const unsigned long long tr = __ballot(ph == PH_CTRACE || ph == PH_STRACE);
            if (!tr) break;
            if (__popcll(tr) < (unsigned)A.refill_below &&
                __ballot(ph == PH_CDONE || ph == PH_SDONE || (ph == PH_NONE && !exhausted)))
                break;
        }
    }
    flush<COUNT>(c, A.counters);
}

// k_wave: allocation left to the compiler (LDS caps residency at 4 workgroups = 4 waves/SIMD).
// k_wave4: register budget forced to 4 waves/SIMD (128 VGPRs); the compiler spills cold path state.
template <int MAXB, bool COUNT>
__global__ __launch_bounds__(BLOCK) void k_wave(KArgs A) {
    __shared__ int lds[STACK * BLOCK];
    wave_body<MAXB, COUNT>(A, lds + threadIdx.x);
}
template <int MAXB, bool COUNT>
__global__ __launch_bounds__(BLOCK, 4) void k_wave4(KArgs A) {
    __shared__ int lds[STACK * BLOCK];
    wave_body<MAXB, COUNT>(A, lds + threadIdx.x);
}

}  // namespace rtd
