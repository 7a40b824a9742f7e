// rt_relay.hpp — the relay kernel: one workgroup of 1 + lights waves per 8x8 pixel tile; wave 0 walks the
// tile's closest-hit chains, wave j walks every level's shadow rays toward light j - 1 as soon as wave 0 has
// published that level's hits (LDS hand-off, no barriers inside a tile).
//
// Why: a single frame (the drop-in seam, cpu/src/main.c:171-185 — one render_frame per timed iteration) lasts
// as long as its slowest tile, and a tile's time is its dependent chain of walks: per bounce level one
// closest-hit walk and then one shadow walk per light (raytracer.c:137-173), every walk in lockstep over the
// tile's 64 lanes. Only the reflection ray of level i + 1 depends on level i, and only on its hit — not on the
// shadow rays — so here the light waves trace level i's shadow rays WHILE the path wave traces level i + 1:
// the chain becomes about (levels + 1) x max(closest, shadow) walks instead of levels x (closest + lights x
// shadow). Unlike k_fan (rt_fan.hpp: the same fan-out over the lanes of ONE wave, whose mixed walk kinds cost
// ~3.5 us per step), every wave here walks one kind of ray over 64 coherent lanes, k_persist's step; unlike
// k_coop it adds no work per ray. The hybrid launch (rt_hip.hip launch_hybrid) sends a frame's costliest
// tiles here while k_persist renders the rest; RT_VARIANT_RELAY runs a whole frame through it (tests).
//
// Bit-exactness: every value is path_step's (rt_kernels.hpp) expression on the same operands: the path wave
// hands each level's hit point, normal, direction and material over as bit copies (LDS); a light wave forms
// the light's term  ((V * kl) * cr) / mg  (raytracer.c:157-159 without the add; back-facing lights with
// V = 0, as the reference) and the path wave adds the terms to the level's ambient colour in light order,
// then folds deepest-first (fold_path). Same walks (closest / visible: fast walk, strict re-walks), same
// counters.
//
// Hand-off protocol (per tile, LDS control block RelayCtl): the path wave writes level i's records and the
// mask of lanes holding one, then releases `pub` = i + 1; after its last level it releases `fin`. Light wave j
// acquires `pub` > i (or `fin` and re-reads `pub`), traces level i, writes its terms and releases
// `done[j]` = i + 1. The path wave acquires every `done[j]` == levels before it resolves. Every wait is a
// bounded spin (s_sleep between polls): all waves of a workgroup are resident together, so the producer always
// progresses; a spin that ever ran out would count an error (rt_get_stats fails) instead of hanging the GPU.
#pragma once
#include "rt_kernels.hpp"

namespace rtd {

constexpr int RELAY_MAXL = 7;  // lights: 1 + lights waves <= 8 (512 threads)

struct RelayCtl {
    int item;                  // the workgroup's current tile (-1: none left)
    int pub;                   // levels the path wave has published
    int fin;                   // 1: `pub` is final
    unsigned lsteps;           // TRACE: the light waves' wave steps of the tile (COUNT)
    int done[RELAY_MAXL + 1];  // levels light wave j has finished
    unsigned long long hm[8];  // per level: the lanes holding a hit record
};
static_assert(sizeof(RelayCtl) % 16 == 0, "records after the control block stay 16-B aligned");

// dynamic LDS of k_relay: the wide walks' stacks (2 * wcap ints per lane, [depth][256] banks of 4 waves), the
// control block, per level 3 float4 records per lane, per level and light one float4 term per lane
__host__ __device__ inline size_t relay_stack_ints(int waves, int wcap) {
    return (size_t)((waves + 3) / 4) * 2 * (size_t)wcap * BLOCK;
}
__host__ __device__ inline size_t relay_lds_bytes(int maxb, int lights, int wcap) {
    return sizeof(int) * relay_stack_ints(1 + lights, wcap) + sizeof(RelayCtl) +
           sizeof(float4) * 64 * (size_t)maxb * (3 + (size_t)lights);
}

constexpr unsigned RELAY_SPIN_MAX = 1u << 22;  // polls (s_sleep 2 each: > 0.5 s) before a wait gives up

__device__ __forceinline__ int lds_acquire(int* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// One 8x8 tile per workgroup iteration; tiles dealt from A.work over A.tile_order (single frames, spp = 1; the
// host launches it for 1 <= lights <= RELAY_MAXL with 64 * (1 + lights) threads and relay_lds_bytes of LDS).
// TRACE (diagnostics, PRT_TILE_TRACE): per tile {begin, end, workgroup, path wave steps | light waves' steps << 32}
template <int MAXB, bool COUNT, bool TRACE = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 64 * (1 + RELAY_MAXL)), amdgpu_waves_per_eu(3)))
void k_relay(KArgs A) {
    extern __shared__ int lds_dyn[];
    const DScene& s = A.s;
    const int nl = s.n_lights, wc = A.wcap;
    const int w = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    int* stk = lds_dyn + (size_t)(w >> 2) * 2 * wc * BLOCK + (threadIdx.x & 255);
    // the strict re-walks' stacks: gstack slots of 256 lanes (host: grid <= 4 x CUs)
    int* sstk = A.gstack + ((size_t)blockIdx.x * 2 + (threadIdx.x >> 8)) * STACK * BLOCK + (threadIdx.x & 255);
    RelayCtl* ctl = (RelayCtl*)(lds_dyn + relay_stack_ints(1 + nl, wc));
    float4* rec = (float4*)(ctl + 1);  // [level][3][64]: (ip, m), (n, -), (d, -)
    float4* trm = rec + MAXB * 3 * 64;  // [level][light][64]: the light's term
    const Cam C = cam_of(A, 0);
    const v3 amb = mk(s.amb_x, s.amb_y, s.amb_z);
    Ctr c = {};
    for (;;) {
        if (threadIdx.x == 0) {
            const unsigned t = atomicAdd(A.work, 1u);
            ctl->item = t < (unsigned)A.n_tiles ? (A.tile_order ? A.tile_order[t] : (int)t) : -1;
            ctl->pub = 0;
            ctl->fin = 0;
            ctl->lsteps = 0;
            for (int j = 0; j <= RELAY_MAXL; j++) ctl->done[j] = 0;
        }
        __syncthreads();
        const int tile = ctl->item;
        if (tile < 0) break;
        unsigned long long tr0 = 0;
        const unsigned ws0 = c.ws;
        if (TRACE) tr0 = __builtin_amdgcn_s_memrealtime();
        const int tx = tile % A.tiles_x, ty = tile / A.tiles_x;
        const int x = tx * 8 + (lane & 7), k = ty * 8 + (lane >> 3);
        const int y = image_row(A, k);
        const bool valid = x < A.W && k < A.n_rows && y < A.H;
        const size_t po = (size_t)k * A.W + x;
        if (w == 0) {
            // ---- the path wave: closest-hit chains (path_step without the light loop), records per level
            if (valid && A.bounce_hit)
                for (int i = 0; i < A.bounces; i++) A.bounce_hit[po * (size_t)A.bounces + i] = -2;
            v3 o = C.pos, d = primary_dir(C, (float)x, (float)y);
            v3 cols[MAXB];
            int mats[MAXB];
#pragma unroll
            for (int q = 0; q < MAXB; q++) {
                cols[q] = mk(0.0f, 0.0f, 0.0f);
                mats[q] = 0;
            }
            int Lv = 0, hit0 = -1;
            float t0 = FMAX;
            unsigned hitlev = 0;  // levels with a hit (their light terms are added)
            bool tail = false, alive = valid;
            int lev = 0;
            for (int it = 0; it < A.bounces; ++it) {
                if (!__ballot(alive)) break;
                bool has = false;
                if (alive) {
                    if (it == 0) c.prim++;
                    else c.refl++;
                    float best;
                    int nd;
                    const int orig = closest<false, COUNT>(s, o, d, best, nd, stk, c, sstk, wc, it > 0);
                    if (it == 0) {
                        hit0 = orig;
                        t0 = best;
                    }
                    if (A.bounce_hit) A.bounce_hit[po * (size_t)A.bounces + it] = orig;
                    if (orig < 0) {  // raytracer.c:132-135
                        set3<MAXB>(cols, it, mk(0.0f + amb.x, 0.0f + amb.y, 0.0f + amb.z));
                        Lv = it + 1;
                        tail = false;
                        alive = false;
                    } else {
                        c.hits++;
                        const v3 ip = add(o, mul(d, best));  // raytracer.c:137-138
                        const float4 sh0 = s.shade[2 * orig], sh1 = s.shade[2 * orig + 1];
                        const int m = __float_as_int(sh0.w);
                        const v3 n = nd ? xyz(sh1) : xyz(sh0);
                        const v3 kd0 = xyz(s.mats[3 * m + 1]);
                        set3<MAXB>(cols, it, mk(0.0f + kd0.x * amb.x, 0.0f + kd0.y * amb.y, 0.0f + kd0.z * amb.z));
                        seti<MAXB>(mats, it, m);
                        has = true;
                        hitlev |= 1u << it;
                        rec[(it * 3 + 0) * 64 + lane] = make_float4(ip.x, ip.y, ip.z, __int_as_float(m));
                        rec[(it * 3 + 1) * 64 + lane] = make_float4(n.x, n.y, n.z, 0.0f);
                        rec[(it * 3 + 2) * 64 + lane] = make_float4(d.x, d.y, d.z, 0.0f);
                        const v3 v = mul(d, -1.0f);
                        const v3 dd = mul(v, -1.0f);  // raytracer.c:163-166
                        const v3 ns = mul(n, 2.0f * __builtin_fabsf(dot(dd, n)));
                        const v3 r = normalize(add(dd, ns));
                        const v3 kr = xyz(s.mats[3 * m + 2]);
                        if (!(mag(kr) > 0.0f)) {  // raytracer.c:168
                            Lv = it + 1;
                            tail = false;
                            alive = false;
                        } else if (it + 1 == A.bounces) {  // raytrace(.., BOUNCES) returns {0,0,0}: col += kr * 0
                            Lv = it + 1;
                            tail = true;
                            alive = false;
                        } else {
                            o = ip;
                            d = r;
                        }
                    }
                }
                const unsigned long long hm = __ballot(has);
                if (lane == 0) ctl->hm[it] = hm;
                lev = it + 1;
                if (lane == 0) lds_release(&ctl->pub, lev);
            }
            if (lane == 0) lds_release(&ctl->fin, 1);
            // ---- resolve: every light wave done with every published level, then the terms in light order
            for (int j = 0; j < nl; j++) {
                unsigned spin = 0;
                while (lds_acquire(&ctl->done[j]) < lev) {
                    if (++spin > RELAY_SPIN_MAX) {
                        c.err++;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
            }
            if (valid) {
#pragma unroll
                for (int q = 0; q < MAXB; q++) {
                    if ((hitlev >> q) & 1u) {
                        v3 cq = cols[q];
                        for (int j = 0; j < nl; j++) {  // col = col + V*kl*cr/mg, raytracer.c:157-159, light order
                            const float4 tj = trm[(q * nl + j) * 64 + lane];
                            cq.x = cq.x + tj.x;
                            cq.y = cq.y + tj.y;
                            cq.z = cq.z + tj.z;
                        }
                        cols[q] = cq;
                    }
                }
                const v3 col = clamp01(fold_path<MAXB>(s, cols, mats, Lv, tail));
                c.pix++;
                store_px(A.rgb, A.bgra, po, col);
                if (A.hit) A.hit[po] = hit0;
                if (A.t) A.t[po] = t0;
            }
        } else if (w <= nl) {
            // ---- light wave j: level i's shadow ray toward light j and its term, as soon as level i is published
            const int j = w - 1;
            const v3 Lp = xyz(s.lights[2 * j]), kl = xyz(s.lights[2 * j + 1]);
            for (int i = 0;; ++i) {
                int p = 0;
                unsigned spin = 0;
                for (;;) {
                    p = lds_acquire(&ctl->pub);
                    if (p > i) break;
                    if (lds_acquire(&ctl->fin)) {
                        p = lds_acquire(&ctl->pub);
                        break;
                    }
                    if (++spin > RELAY_SPIN_MAX) {
                        c.err++;
                        p = -1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (p <= i) break;
                if ((ctl->hm[i] >> lane) & 1ull) {
                    const float4 r0 = rec[(i * 3 + 0) * 64 + lane], r1 = rec[(i * 3 + 1) * 64 + lane],
                                 r2 = rec[(i * 3 + 2) * 64 + lane];
                    const v3 ip = xyz(r0), n = xyz(r1), d = xyz(r2);
                    const int m = __float_as_int(r0.w);
                    const v3 v = mul(d, -1.0f);  // raytracer.c:147
                    v3 l = sub(Lp, ip);           // light_v, raytracer.c:62-99
                    float mg = mag(l);
                    l = dvs(l, mg);
                    mg *= mg;
                    const v3 tmp = sub(ip, Lp), tmp2 = sub(Lp, ip);
                    const float ld2 = dot(tmp, tmp);
                    int V;
                    if (dot(tmp2, n) < 0) {
                        V = 0;
                        c.skip++;
                    } else {
                        c.shad++;
                        V = visible<false, COUNT>(s, ip, l, ld2, stk, c, sstk, wc) ? 1 : 0;
                    }
                    const v3 ks = xyz(s.mats[3 * m]), kd = xyz(s.mats[3 * m + 1]);
                    const float ndl = dot(n, l);
                    const v3 h = normalize(add(l, v));  // lambert_blinn, raytracer.c:21-33
                    const float coeff = fmaxf(0.0f, dot(n, h));
                    const v3 cr = mk(kd.x * fmaxf(0.0f, ndl) + ks.x * coeff, kd.y * fmaxf(0.0f, ndl) + ks.y * coeff,
                                     kd.z * fmaxf(0.0f, ndl) + ks.z * coeff);
                    const float fV = (float)V;
                    trm[(i * nl + j) * 64 + lane] =
                        make_float4(fV * kl.x * cr.x / mg, fV * kl.y * cr.y / mg, fV * kl.z * cr.z / mg, 0.0f);
                }
                if (lane == 0) lds_release(&ctl->done[j], i + 1);
            }
        }
        if (TRACE && w > 0 && w <= nl) {
            const unsigned ws = wave_sum(c.ws - ws0);
            if (lane == 0) atomicAdd(&ctl->lsteps, ws);
        }
        __syncthreads();  // the tile's LDS is read by everyone before the next tile resets it
        if (TRACE && w == 0) {
            const unsigned ws = wave_sum(c.ws - ws0);
            if (lane == 0) {
                A.tile_trace[4 * tile] = tr0;
                A.tile_trace[4 * tile + 1] = __builtin_amdgcn_s_memrealtime();
                A.tile_trace[4 * tile + 2] = blockIdx.x;
                A.tile_trace[4 * tile + 3] = ws | ((unsigned long long)ctl->lsteps << 32);
            }
        }
    }
    flush<COUNT>(c, A.counters);
}

}  // namespace rtd
