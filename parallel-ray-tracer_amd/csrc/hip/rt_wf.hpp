// rt_wf.hpp — the wavefront pipeline (RT_KERNEL_WAVEFRONT): the per-pixel recursion split into stages that
// communicate through dense ray queues in HBM, so the traversal kernels stay lean.
//
// Why: one fused per-pixel kernel keeps the whole path state alive across every traversal (~150
// VGPRs) and needs a 34-deep LDS stack per lane: 3 waves/SIMD, 60 % of wave cycles waiting on the
// dependent node loads, ~20 % lane utilisation (rocprof, profiles/r1_*). Here the traversal kernels
// hold one ray per lane (origin, direction, reciprocals, best hit, stack pointer), keep the near child
// in a register (the LDS stack only holds deferred far children, <= BVH depth), and refill idle lanes
// with new rays from the queue whenever fewer than `refill_below` lanes are still tracing.
//
// Per frame, level i = 0 .. BOUNCES-1 (each a kernel on the context stream; counts stay on the device):
//   primary            camera rays of every pixel -> closest queue C0                 (main.c:228-233)
//   trace<closest>     C_i -> hit record per entry (t, triangle, normal side)       (bvh.c:317-358)
//   fallback<closest>  entries with a zero direction component / exact tie, strict walk
//   shade(i)           per hit: shadow ray per light past the back-face test -> S;
//                      reflection ray -> C_{i+1} while |kr| > 0 and i+1 < BOUNCES      (raytracer.c:132-173)
//   trace<shadow>      S -> visibility byte per (entry, light)                       (bvh.c:269-315)
//   fallback<shadow>
//   accum(i)           per hit: c_i = kd*amb + sum_j V_j*kl_j*cr_j/mag_j in light order (raytracer.c:144-160)
// fold                 per pixel: c_0 + kr_0*(c_1 + kr_1*(...)), clamp                 (raytracer.c:169-172)
// The arithmetic of every stage is rt_kernels.hpp's, operation for operation (bit-exact, tests).
#pragma once
#include "rt_kernels.hpp"

namespace rtd {

constexpr int WF_STACK = 26;  // acceleration BVH depth <= 24; only far children are stacked
constexpr int WF_BLOCK = 256;
constexpr int WF_MAXB = 8;    // per-pixel level records
enum { Q_C0 = 0, Q_C1 = 1, Q_S = 2, Q_F = 3, Q_WORK = 4, Q_FWORK = 5, Q_PIX = 6, Q_N = 8 };

struct WfArgs {
    DScene s;
    float pos[3], ul[3], ix[3], iy[3];
    int W, n_rows, row_offset, row_stride, tiles_x, n_tiles, bounces, level, cur;
    float4* cq[2];          // closest-ray queues (ping-pong): 2 float4 per entry: (o, pixel), (d, -)
    float4* sq;             // shadow-ray queue: (o, vis slot), (d, light_dist2)
    float4* hrec;           // per closest entry: (t, triangle, normal side, -)
    unsigned char* vis;     // per closest entry x light: 1 = light visible
    int* fq;                // fallback entries
    float4* lev;            // per pixel x WF_MAXB: (c_i, material id)
    int* plen;              // per pixel: levels | tail << 16
    float* rgb;
    int* hit;
    float* t;
    unsigned* q;            // Q_N counters
    unsigned long long* counters;
    int refill_below;
    int chunk_min, chunk_max;  // guided self-scheduling window bounds (entries per claim)
};
static_assert(sizeof(WfArgs) == 352, "kernel-argument layout changed (see rt_device.hpp)");



__device__ __forceinline__ void ray_store(float4* q, unsigned e, v3 o, v3 d, int tag, float w) {
    q[2 * e] = make_float4(o.x, o.y, o.z, __int_as_float(tag));
    q[2 * e + 1] = make_float4(d.x, d.y, d.z, w);
}

// wave-aggregated append: returns this lane's slot (lanes with !want get 0)
__device__ __forceinline__ unsigned wave_append(unsigned* cnt, bool want) {
    const unsigned long long m = __ballot(want);
    if (!m) return 0;
    const int leader = __ffsll((long long)m) - 1;
    unsigned base = 0;
    if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(cnt, (unsigned)__popcll(m));
    base = __shfl(base, leader, 64);
    return base + (unsigned)__popcll(m & ((1ull << (threadIdx.x & 63)) - 1ull));
}

// ---------------------------------------------------------------- primary rays
// Positional (no atomics): entry id = 8x8-tile-major pixel id, so a wave's 64 lanes trace one tile.
// Ids that fall outside a partial edge tile carry pixel -1 and are skipped by every stage.
__global__ __launch_bounds__(WF_BLOCK) void k_wf_primary(WfArgs A) {
    const unsigned n_ids = (unsigned)A.n_tiles * 64u;
    if (blockIdx.x == 0 && threadIdx.x == 0) A.q[Q_C0] = n_ids;
    const Cam K{mk(A.pos[0], A.pos[1], A.pos[2]), mk(A.ul[0], A.ul[1], A.ul[2]), mk(A.ix[0], A.ix[1], A.ix[2]),
                mk(A.iy[0], A.iy[1], A.iy[2])};
    Ctr c = {};
    for (unsigned id = blockIdx.x * WF_BLOCK + threadIdx.x; id < n_ids; id += gridDim.x * WF_BLOCK) {
        const int tile = (int)(id >> 6), w = (int)(id & 63u);
        const int x = (tile % A.tiles_x) * 8 + (w & 7), k = (tile / A.tiles_x) * 8 + (w >> 3);
        const bool ok = x < A.W && k < A.n_rows;
        const int y = A.row_offset + k * A.row_stride;
        ray_store(A.cq[0], id, mk(A.pos[0], A.pos[1], A.pos[2]), primary_dir(K, (float)x, (float)y),
                  ok ? k * A.W + x : -1, 0.0f);
        if (ok) c.prim++;
    }
    flush<false>(c, A.counters);
}

// Block-aggregated append: every thread of the (256-thread) workgroup calls it with its item count;
// ONE global atomic per workgroup (a single queue counter saturates at ~88 dequeues/us,
// MI355X_MICROARCH.md "dequeue"). Returns the thread's first slot.
__device__ __forceinline__ unsigned block_alloc(unsigned cnt, unsigned* gcnt, unsigned* s /* __shared__ [5] */) {
    const unsigned lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    unsigned x = cnt;  // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = __shfl_up(x, (unsigned)o, 64);
        if (lane >= (unsigned)o) x += y;
    }
    if (lane == 63) s[w] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t0 = s[0], t1 = s[1], t2 = s[2], t3 = s[3], tot = t0 + t1 + t2 + t3;
        const unsigned base = tot ? atomicAdd(gcnt, tot) : 0u;
        s[0] = base;
        s[1] = base + t0;
        s[2] = base + t0 + t1;
        s[3] = base + t0 + t1 + t2;
    }
    __syncthreads();
    const unsigned r = s[w] + x - cnt;
    __syncthreads();
    return r;
}

// ---------------------------------------------------------------- traversal (fast walk)
// One ray per lane, dynamic fetch from the queue. Near child kept in `cur`; far children on the stack.
template <bool SHADOW, bool COUNT>
__global__ __launch_bounds__(WF_BLOCK) void k_wf_trace(WfArgs A) {
    __shared__ int lds[WF_STACK * WF_BLOCK];
    int* __restrict__ stk = lds + threadIdx.x;
    const DBvh B = A.s.acc;
    const float4* __restrict__ q = SHADOW ? A.sq : A.cq[A.cur];
    const unsigned n = SHADOW ? A.q[Q_S] : A.q[A.cur];
    unsigned* work = &A.q[Q_WORK];
    if (blockIdx.x == 0 && threadIdx.x == 0) A.q[Q_FWORK] = 0;  // for the fallback kernel that follows
    Ctr c = {};
    bool act = false, tie = false;
    unsigned e = 0;
    int slot = 0, cur = 0, sp = 0, hp = -1, nd = 0;
    float best = FMAX, ld2 = 0.0f;
    v3 o = mk(0, 0, 0), d = mk(0, 0, 0);
    RayPre p = {};
    // Guided self-scheduling: the wave claims a window of queue entries with ONE atomic, sized to the
    // remaining work (rem / (2 * waves), 64..2048 entries), and refills its idle lanes from the window
    // without further atomics. Wave-uniform state.
    const unsigned lane = threadIdx.x & 63u;
    const unsigned nwaves = gridDim.x * (WF_BLOCK / 64);
    unsigned wnext = 0, wend = 0;
    bool drained = false;
    for (;;) {
        // ---- refill idle lanes from the wave's window
        for (;;) {
            const unsigned long long need = __ballot(!act);
            if (!need || drained) break;
            if (wnext >= wend) {
                unsigned start = 0, chunk = 0;
                if (lane == 0) {
                    const unsigned taken = __atomic_load_n(work, __ATOMIC_RELAXED);
                    const unsigned rem = taken < n ? n - taken : 0u;
                    chunk = min((unsigned)A.chunk_max, max((unsigned)A.chunk_min, rem / (2u * nwaves)));
                    start = atomicAdd(work, chunk);
                }
                start = __shfl(start, 0, 64);
                chunk = __shfl(chunk, 0, 64);
                if (start >= n) {
                    drained = true;
                    break;
                }
                wnext = start;
                wend = min(start + chunk, n);
            }
            const unsigned take = min((unsigned)__popcll(need), wend - wnext);
            const unsigned rank = (unsigned)__popcll(need & ((1ull << lane) - 1ull));
            if (!act && rank < take) {
                e = wnext + rank;
                const float4 a = q[2 * e], b = q[2 * e + 1];
                o = mk(a.x, a.y, a.z);
                d = mk(b.x, b.y, b.z);
                slot = __float_as_int(a.w);
                ld2 = b.w;
                if (!SHADOW && slot < 0) {
                    // padding entry of a partial edge tile: nothing to trace
                } else if (degenerate(d)) {  // NaN-slab semantics: strict walk (fallback kernel)
                    A.fq[atomicAdd(&A.q[Q_F], 1u)] = (int)e;
                    c.fb++;
                } else {
                    p = ray_pre(o, d);
                    best = FMAX;
                    hp = -1;
                    nd = 0;
                    tie = false;
                    sp = 0;
                    cur = B.root;
                    act = true;
                }
            }
            wnext += take;
        }
        if (!__ballot(act)) break;  // queue drained, every lane idle
        // ---- traverse until too few lanes remain busy
        for (;;) {
            if (act) {
                bool done = false;
                if (cur < 0) {  // leaf
                    const int2 lf = B.leaves[~cur];
                    if (COUNT) {
                        if (SHADOW) c.shl++;
                        else c.chl++;
                    }
                    for (int i = lf.x; i < lf.x + lf.y; ++i) {
                        int k;
                        const float tt = hit_triangle(o, d, B.tris + 3 * i, k);
                        if (COUNT) {
                            if (SHADOW) c.sht++;
                            else c.cht++;
                        }
                        if (tt < best) {
                            best = tt;
                            if (SHADOW) {  // bvh.c:283-290
                                const v3 ip = add(o, mul(d, best));
                                const v3 oi = sub(o, ip);
                                if (ld2 > dot(oi, oi)) {
                                    done = true;  // occluded
                                    break;
                                }
                            } else {
                                hp = i;
                                nd = k;
                                tie = false;
                            }
                        } else if (!SHADOW && tt == best && tt != FMAX) {
                            tie = true;
                        }
                    }
                    if (done) {
                        A.vis[slot] = 0;
                    } else if (sp > 0) {
                        cur = stk[(--sp) * WF_BLOCK];
                    } else {
                        done = true;
                        if (SHADOW) A.vis[slot] = 1;
                    }
                } else {
                    if (COUNT) {
                        if (SHADOW) c.shi++;
                        else c.chi++;
                    }
                    const float4* N = B.nodes + 4 * cur;
                    const float4 a = N[0], b = N[1], ee = N[2], r = N[3];
                    int ni = __float_as_int(r.x), fi = __float_as_int(r.y);
                    float nt = box_fast(a.x, a.y, a.z, a.w, b.x, b.y, p);
                    float ft = box_fast(b.z, b.w, ee.x, ee.y, ee.z, ee.w, p);
                    const float lim = best * PRUNE_SLACK;
                    const bool hn = ni != EMPTY_REF && nt != FMAX && nt <= lim;
                    const bool hf = fi != EMPTY_REF && ft != FMAX && ft <= lim;
                    if (hn && hf) {
                        if (ft < nt) {
                            const int ti = ni;
                            ni = fi;
                            fi = ti;
                        }
                        if (sp >= WF_STACK) {
                            c.err++;
                            done = true;
                        } else {
                            stk[(sp++) * WF_BLOCK] = fi;
                            cur = ni;
                        }
                    } else if (hn) {
                        cur = ni;
                    } else if (hf) {
                        cur = fi;
                    } else if (sp > 0) {
                        cur = stk[(--sp) * WF_BLOCK];
                    } else {
                        done = true;
                        if (SHADOW) A.vis[slot] = 1;
                    }
                }
                if (done) {
                    act = false;
                    if (!SHADOW) {
                        A.hrec[e] = make_float4(best, __int_as_float(hp >= 0 ? B.tri_orig[hp] : -1),
                                                __int_as_float(nd), 0.0f);
                        if (tie) {  // first-found order decides the winner (bvh.c:331): strict re-walk
                            A.fq[atomicAdd(&A.q[Q_F], 1u)] = (int)e;
                            c.fb++;
                        }
                    }
                }
            }
            const unsigned long long tr = __ballot(act);
            if (!tr) break;
            if (__popcll(tr) < (unsigned)A.refill_below && !drained) break;
        }
    }
    flush<COUNT>(c, A.counters);
}

// ---------------------------------------------------------------- strict fallbacks (rare)
template <bool SHADOW>
__global__ __launch_bounds__(WF_BLOCK) void k_wf_fallback(WfArgs A) {
    __shared__ int lds[STACK * WF_BLOCK];
    int* __restrict__ stk = lds + threadIdx.x;
    const unsigned n = A.q[Q_F];
    const float4* __restrict__ q = SHADOW ? A.sq : A.cq[A.cur];
    if (blockIdx.x == 0 && threadIdx.x == 0 && !SHADOW) {  // counters the shade kernel appends to
        A.q[1 - A.cur] = 0;
        A.q[Q_S] = 0;
    }
    for (unsigned i = blockIdx.x * WF_BLOCK + threadIdx.x; i < n; i += gridDim.x * WF_BLOCK) {
        const unsigned e = (unsigned)A.fq[i];
        const float4 a = q[2 * e], b = q[2 * e + 1];
        const v3 o = mk(a.x, a.y, a.z), d = mk(b.x, b.y, b.z);
        Ctr c = {};
        if (SHADOW) {
            A.vis[__float_as_int(a.w)] = visible_walk<true, false>(A.s.ref, o, d, b.w, stk, c) ? 1 : 0;
        } else {
            float best = FMAX;
            int hp = -1, nd = 0;
            bool tie = false;
            closest_walk<true, false>(A.s.ref, o, d, best, hp, nd, tie, stk, c);
            A.hrec[e] = make_float4(best, __int_as_float(hp >= 0 ? A.s.ref.tri_orig[hp] : -1), __int_as_float(nd), 0.0f);
        }
    }
}

// ---------------------------------------------------------------- shading stages
// The light loop of raytrace (raytracer.c:149-160) split in two passes over the same hits: shade emits
// the shadow rays, accum adds the terms once visibility is known. Both recompute l, |l|, cr from the hit
// with identical operations, so the bits are the same as computing them once.
struct LightTerm {
    v3 l, cr, kl;
    float mg, ld2;
    bool front;  // (L - P) . n >= 0: a shadow ray is traced (light_v, raytracer.c:66-67)
};

__device__ __forceinline__ LightTerm light_term(const DScene& s, int j, v3 ip, v3 n, v3 v, v3 ks, v3 kd) {
    LightTerm T;
    const v3 Lp = xyz(s.lights[2 * j]);
    T.kl = xyz(s.lights[2 * j + 1]);
    v3 l = sub(Lp, ip);
    float mg = mag(l);
    l = dvs(l, mg);
    mg *= mg;
    const float ndl = dot(n, l);
    const v3 h = normalize(add(l, v));
    const float coeff = fmaxf(0.0f, dot(n, h));
    T.cr = mk(kd.x * fmaxf(0.0f, ndl) + ks.x * coeff, kd.y * fmaxf(0.0f, ndl) + ks.y * coeff,
              kd.z * fmaxf(0.0f, ndl) + ks.z * coeff);
    T.l = l;
    T.mg = mg;
    const v3 tmp = sub(ip, Lp), tmp2 = sub(Lp, ip);
    T.ld2 = dot(tmp, tmp);
    T.front = !(dot(tmp2, n) < 0);
    return T;
}

__global__ __launch_bounds__(WF_BLOCK) void k_wf_shade(WfArgs A) {
    const DScene& s = A.s;
    const unsigned n = A.q[A.cur];
    const int nxt = 1 - A.cur, L = s.n_lights;
    const v3 amb = mk(s.amb_x, s.amb_y, s.amb_z);
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // the next trace kernel's work counter, fallback count
        A.q[Q_WORK] = 0;
        A.q[Q_F] = 0;
    }
    __shared__ unsigned s_alloc[4];
    Ctr c = {};
    const unsigned stride = gridDim.x * WF_BLOCK;
    for (unsigned e0 = blockIdx.x * WF_BLOCK; e0 < n; e0 += stride) {  // uniform per workgroup
        const unsigned e = e0 + threadIdx.x;
        bool hit = false, refl = false;
        v3 ip = mk(0, 0, 0), r = mk(0, 0, 0), nrm = mk(0, 0, 0), v = mk(0, 0, 0), ks = v, kd = v;
        int pix = -1, og = -1;
        if (e < n) pix = __float_as_int(A.cq[A.cur][2 * e].w);
        if (pix >= 0) {
            const float4 a = A.cq[A.cur][2 * e], b = A.cq[A.cur][2 * e + 1], h = A.hrec[e];
            const v3 o = mk(a.x, a.y, a.z), d = mk(b.x, b.y, b.z);
            og = __float_as_int(h.y);
            const float best = h.x;
            const int nd = __float_as_int(h.z);
            if (A.level == 0) {
                if (A.hit) A.hit[pix] = og;
                if (A.t) A.t[pix] = best;
            }
            float4* lv = A.lev + (size_t)pix * WF_MAXB + A.level;
            if (og < 0) {  // raytracer.c:132-135
                *lv = make_float4(0.0f + amb.x, 0.0f + amb.y, 0.0f + amb.z, 0.0f);
                A.plen[pix] = A.level + 1;
            } else {
                hit = true;
                c.hits++;
                ip = add(o, mul(d, best));
                const float4 sh0 = s.shade[2 * og];
                const int m = __float_as_int(sh0.w);
                nrm = xyz(s.shade[2 * og + nd]);
                ks = xyz(s.mats[3 * m]);
                kd = xyz(s.mats[3 * m + 1]);
                const v3 kr = xyz(s.mats[3 * m + 2]);
                v = mul(d, -1.0f);
                lv->w = __int_as_float(m);
                const v3 dd = mul(v, -1.0f);  // raytracer.c:163-166
                const v3 ns = mul(nrm, 2.0f * __builtin_fabsf(dot(dd, nrm)));
                r = normalize(add(dd, ns));
                const bool rec = mag(kr) > 0.0f;
                refl = rec && A.level + 1 < A.bounces;
                if (!refl) A.plen[pix] = (A.level + 1) | (rec ? (1 << 16) : 0);
                for (int j = 0; j < L; j++) A.vis[(size_t)e * L + j] = 0;
            }
        }
        // shadow rays past the back-face test (raytracer.c:66-67), then their queue slots
        unsigned emask = 0;
        if (hit)
            for (int j = 0; j < L; j++) {
                if (light_term(s, j, ip, nrm, v, ks, kd).front) {
                    emask |= 1u << j;
                    c.shad++;
                } else {
                    c.skip++;
                }
            }
        unsigned slot = block_alloc((unsigned)__popc(emask), &A.q[Q_S], s_alloc);
        for (int j = 0; emask >> j; j++)
            if ((emask >> j) & 1u) {
                const LightTerm T = light_term(s, j, ip, nrm, v, ks, kd);
                ray_store(A.sq, slot++, ip, T.l, (int)(e * L + j), T.ld2);
            }
        const unsigned rslot = block_alloc(refl ? 1u : 0u, &A.q[nxt], s_alloc);
        if (refl) {
            ray_store(A.cq[nxt], rslot, ip, r, pix, 0.0f);
            c.refl++;
        }
    }
    flush<false>(c, A.counters);
}

__global__ __launch_bounds__(WF_BLOCK) void k_wf_accum(WfArgs A) {
    const DScene& s = A.s;
    const unsigned n = A.q[A.cur];
    const int L = s.n_lights;
    const v3 amb = mk(s.amb_x, s.amb_y, s.amb_z);
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // next level's trace kernel
        A.q[Q_WORK] = 0;
        A.q[Q_F] = 0;
    }
    for (unsigned e = blockIdx.x * WF_BLOCK + threadIdx.x; e < n; e += gridDim.x * WF_BLOCK) {
        const float4 a = A.cq[A.cur][2 * e];
        const int pix = __float_as_int(a.w);
        if (pix < 0) continue;  // padding entry of a partial edge tile
        const float4 h = A.hrec[e];
        const int og = __float_as_int(h.y);
        if (og < 0) continue;
        const float4 b = A.cq[A.cur][2 * e + 1];
        const v3 o = mk(a.x, a.y, a.z), d = mk(b.x, b.y, b.z);
        const int nd = __float_as_int(h.z);
        const v3 ip = add(o, mul(d, h.x));
        const int m = __float_as_int(s.shade[2 * og].w);
        const v3 nrm = xyz(s.shade[2 * og + nd]);
        const v3 ks = xyz(s.mats[3 * m]), kd = xyz(s.mats[3 * m + 1]);
        v3 col = mk(0.0f + kd.x * amb.x, 0.0f + kd.y * amb.y, 0.0f + kd.z * amb.z);  // raytracer.c:144-146
        const v3 v = mul(d, -1.0f);
        for (int j = 0; j < L; j++) {  // raytracer.c:149-160, light order
            const LightTerm T = light_term(s, j, ip, nrm, v, ks, kd);
            const float fV = (float)A.vis[(size_t)e * L + j];
            col.x = col.x + fV * T.kl.x * T.cr.x / T.mg;
            col.y = col.y + fV * T.kl.y * T.cr.y / T.mg;
            col.z = col.z + fV * T.kl.z * T.cr.z / T.mg;
        }
        float4* lv = A.lev + (size_t)pix * WF_MAXB + A.level;
        const float mw = lv->w;
        *lv = make_float4(col.x, col.y, col.z, mw);
    }
}

// fold: R_i = c_i + kr_i * R_{i+1}, deepest level first (raytracer.c:169-172), then vec_constrain
__global__ __launch_bounds__(WF_BLOCK) void k_wf_fold(WfArgs A) {
    const DScene& s = A.s;
    const unsigned npx = (unsigned)A.W * (unsigned)A.n_rows;
    Ctr c = {};
    for (unsigned pix = blockIdx.x * WF_BLOCK + threadIdx.x; pix < npx; pix += gridDim.x * WF_BLOCK) {
        const int pl = A.plen[pix];
        const int L = pl & 0xffff;
        const bool tail = (pl >> 16) != 0;
        const float4* lv = A.lev + (size_t)pix * WF_MAXB;
        float4 f = lv[L - 1];
        v3 acc = mk(f.x, f.y, f.z);
        if (tail) {
            const v3 kr = xyz(s.mats[3 * __float_as_int(f.w) + 2]);
            acc = mk(acc.x + kr.x * 0.0f, acc.y + kr.y * 0.0f, acc.z + kr.z * 0.0f);
        }
        for (int i = L - 2; i >= 0; --i) {
            f = lv[i];
            const v3 kr = xyz(s.mats[3 * __float_as_int(f.w) + 2]);
            acc = mk(f.x + kr.x * acc.x, f.y + kr.y * acc.y, f.z + kr.z * acc.z);
        }
        const v3 cl = clamp01(acc);
        A.rgb[3 * (size_t)pix] = cl.x;
        A.rgb[3 * (size_t)pix + 1] = cl.y;
        A.rgb[3 * (size_t)pix + 2] = cl.z;
        c.pix++;
    }
    flush<false>(c, A.counters);
}

}  // namespace rtd
