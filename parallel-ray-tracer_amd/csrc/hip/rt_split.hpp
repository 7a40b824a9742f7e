// rt_split.hpp — the per-pixel recursion in three tile-coherent kernels (RT_KERNEL_FAST with >= 3 lights;
// PRT_SPLIT=0/1 forces either way).
//
// k_persist runs a tile's whole chain — per bounce level one closest-hit walk and one shadow walk per
// light — in one wave, so the frame ends when the slowest tile's chain does (PRT_TILE_TRACE: up to
// ~1.9 ms of a ~2 ms frame, while waves are busy ~55 % of it). Shadow walks are two thirds of that
// chain and depend on nothing but their level's hit point, so they move out of it:
//   k_split_closest : persistent tiles trace the closest-hit chain (primary + reflection rays) and
//                     record per level the hit point, normal, direction, material and the lights past
//                     light_v's back-face test; one batch per (tile, level, light) with any such lane;
//   k_split_shadow  : persistent waves take those batches — the tile's 64 lanes toward one light, the
//                     coherence of k_persist's shadow phase — and write one visibility byte per lane;
//   k_split_resolve : per pixel, the reference's per-light accumulation in light order with those bytes
//                     (raytracer.c:149-160, the same expressions as path_step), the fold, the clamp.
// Every per-pixel operation is path_step's, only moved: results are k_persist's bit for bit. Kernel
// boundaries order the hand-offs (no fences, no waiting inside a kernel). spp == 1, lights <= 32.
// Frame batches (BATCH, rt_render_frames): the closest kernel deals (frame, tile) items like k_persist
// (rtd::next_item: XCD-aware regions, every frame's central tiles first); a record slot is
// item * 64 + lane with item = frame * n_tiles + tile, so the three kernels cover the whole batch.
#pragma once
#include "rt_kernels.hpp"

namespace rtd {

constexpr unsigned SPLIT_TAIL = 1u << 8, SPLIT_MISS = 1u << 9;  // path info: L | flags
// KArgs::work slots (separate 128-B lines, past next_item's 8 region counters at 16 r)
constexpr int SPLIT_BATCH_AT = 160, SPLIT_TAKE_AT = 192;

// per (level, slot) record: f4[0] = ip, light mask (bits); f4[1] = n, material (bits); f4[2] = d, 0
__device__ __forceinline__ size_t srec_at(const KArgs& A, int it, size_t slot) {
    return ((size_t)it * A.nslots + slot) * 3;
}

template <int MAXB, bool COUNT, bool BATCH = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, BLOCK), amdgpu_waves_per_eu(3))) void k_split_closest(KArgs A) {
    __shared__ int lds[STACK * BLOCK];
    int* stk = lds + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const DScene& s = A.s;
    Ctr c = {};
    int reg = 0;
    for (;;) {
        int frame;
        unsigned tile;
        if (!next_item(A, lane, reg, frame, tile)) break;
        const int x = (int)(tile % (unsigned)A.tiles_x) * 8 + (lane & 7);
        const int k = (int)(tile / (unsigned)A.tiles_x) * 8 + (lane >> 3);
        const unsigned item = (unsigned)frame * (unsigned)A.n_tiles + tile;
        const size_t slot = (size_t)item * 64 + lane;
        unsigned info = 0;
        unsigned masks[MAXB];
#pragma unroll
        for (int q = 0; q < MAXB; q++) masks[q] = 0;
        const int y = image_row(A, k, frame);
        if (x < A.W && k < A.n_rows && y < A.H) {
            c.pix++;
            const size_t px = (size_t)frame * A.frame_px + (size_t)k * A.W + x;
            const Cam C = cam_of<BATCH>(A, frame);
            v3 o = C.pos;
            v3 d = primary_dir(C, (float)x, (float)y);
            if (A.bounce_hit)
                for (int i = 0; i < A.bounces; i++) A.bounce_hit[px * A.bounces + i] = -2;
            for (int it = 0; it < A.bounces; ++it) {
                float best;
                int nd;
                if (it == 0) c.prim++;
                else c.refl++;
                const int orig = closest<false, COUNT, true, true>(s, o, d, best, nd, stk, c, nullptr, WSTACK, it > 0);
                if (it == 0) {
                    if (A.hit) A.hit[px] = orig;
                    if (A.t) A.t[px] = best;
                }
                if (A.bounce_hit) A.bounce_hit[px * A.bounces + it] = orig;
                if (orig < 0) {  // raytracer.c:132-135
                    info = (unsigned)(it + 1) | SPLIT_MISS;
                    break;
                }
                c.hits++;
                const v3 ip = add(o, mul(d, best));  // raytracer.c:137-138
                const float4 sh0 = s.shade[2 * orig], sh1 = s.shade[2 * orig + 1];
                const int m = __float_as_int(sh0.w);
                const v3 n = nd ? xyz(sh1) : xyz(sh0);
                unsigned mask = 0;
                for (int j = 0; j < s.n_lights; ++j) {  // light_v's back-face test, raytracer.c:66-67
                    const v3 tmp2 = sub(xyz(s.lights[2 * j]), ip);
                    if (dot(tmp2, n) < 0) {
                        c.skip++;
                    } else {
                        c.shad++;
                        mask |= 1u << j;
                    }
                }
                set_u<MAXB>(masks, it, mask);
                float4* R = A.srec + srec_at(A, it, slot);
                R[0] = make_float4(ip.x, ip.y, ip.z, __uint_as_float(mask));
                R[1] = make_float4(n.x, n.y, n.z, __int_as_float(m));
                R[2] = make_float4(d.x, d.y, d.z, 0.0f);
                const v3 kr = xyz(s.mats[3 * m + 2]);
                const v3 v = mul(d, -1.0f);
                const v3 dd = mul(v, -1.0f);  // raytracer.c:163-166
                const v3 ns = mul(n, 2.0f * __builtin_fabsf(dot(dd, n)));
                const v3 r = normalize(add(dd, ns));
                if (!(mag(kr) > 0.0f)) {  // raytracer.c:168
                    info = (unsigned)(it + 1);
                    break;
                }
                if (it + 1 == A.bounces) {
                    info = (unsigned)(it + 1) | SPLIT_TAIL;
                    break;
                }
                o = ip;
                d = r;
            }
        }
        A.spinfo[slot] = info;
        // one shadow batch per (level, light) that any lane of the tile needs
        for (int it = 0; it < A.bounces; ++it) {
            const unsigned mk_ = get_u<MAXB>(masks, it);
            for (int j = 0; j < A.s.n_lights; ++j) {
                const unsigned long long any = __ballot((mk_ >> j) & 1u);
                if (any && lane == 0) {
                    const unsigned at = atomicAdd(A.work + SPLIT_BATCH_AT, 1u);
                    A.sbatch[at] = (item << 8) | ((unsigned)it << 5) | (unsigned)j;
                }
            }
        }
    }
    flush<COUNT>(c, A.counters);
}

template <bool COUNT>
__global__ __attribute__((amdgpu_flat_work_group_size(1, BLOCK))) void k_split_shadow(KArgs A) {
    __shared__ int lds[STACK * BLOCK];
    int* stk = lds + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const unsigned nb = A.work[SPLIT_BATCH_AT];  // written by k_split_closest: visible at this launch
    Ctr c = {};
    for (;;) {
        unsigned b = 0;
        if (lane == 0) b = atomicAdd(A.work + SPLIT_TAKE_AT, 1u);
        b = __shfl(b, 0, 64);
        if (b >= nb) break;
        const unsigned e = A.sbatch[b];
        const unsigned item = e >> 8, it = (e >> 5) & 7u, j = e & 31u;
        const size_t slot = (size_t)item * 64 + lane;
        const float4 f0 = A.srec[srec_at(A, (int)it, slot)];
        if ((__float_as_uint(f0.w) >> j) & 1u) {  // light_v past the back-face test, raytracer.c:72-74
            const v3 ip = xyz(f0), Lp = xyz(A.s.lights[2 * j]);
            v3 l = sub(Lp, ip);  // raytracer.c:150-153
            const float mg = mag(l);
            l = dvs(l, mg);
            const v3 tmp = sub(ip, Lp);
            const bool V = visible<false, COUNT, true, true>(A.s, ip, l, dot(tmp, tmp), stk, c);
            A.svis[((size_t)it * A.s.n_lights + j) * A.nslots + slot] = V ? 1 : 0;
        }
    }
    flush<COUNT>(c, A.counters);
}

template <int MAXB>
__global__ __launch_bounds__(256) void k_split_resolve(KArgs A) {
    const size_t slot = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= A.nslots) return;
    const unsigned info = A.spinfo[slot];
    const int L = (int)(info & 0xFFu);
    if (!L) return;  // outside the frame
    const unsigned item = (unsigned)(slot >> 6), lane = (unsigned)(slot & 63);
    const unsigned frame = item / (unsigned)A.n_tiles, tile = item % (unsigned)A.n_tiles;
    const int x = (int)(tile % (unsigned)A.tiles_x) * 8 + (int)(lane & 7u);
    const int k = (int)(tile / (unsigned)A.tiles_x) * 8 + (int)(lane >> 3);
    const DScene& s = A.s;
    const v3 amb = mk(s.amb_x, s.amb_y, s.amb_z);
    v3 cols[MAXB];
    int mats[MAXB];
#pragma unroll
    for (int q = 0; q < MAXB; q++) {
        cols[q] = mk(0.0f, 0.0f, 0.0f);
        mats[q] = 0;
    }
    for (int it = 0; it < L; ++it) {
        if (it == L - 1 && (info & SPLIT_MISS)) {  // raytracer.c:132-135
            set3<MAXB>(cols, it, mk(0.0f + amb.x, 0.0f + amb.y, 0.0f + amb.z));
            break;
        }
        const float4* R = A.srec + srec_at(A, it, slot);
        const float4 f0 = R[0], f1 = R[1], f2 = R[2];
        const v3 ip = xyz(f0), n = xyz(f1), d = xyz(f2);
        const unsigned mask = __float_as_uint(f0.w);
        const int m = __float_as_int(f1.w);
        const v3 ks = xyz(s.mats[3 * m]), kd = xyz(s.mats[3 * m + 1]);
        v3 col = mk(0.0f + kd.x * amb.x, 0.0f + kd.y * amb.y, 0.0f + kd.z * amb.z);  // :144-146
        const v3 v = mul(d, -1.0f);                                                      // :147
        for (int j = 0; j < s.n_lights; ++j) {                                           // :149-160
            const v3 Lp = xyz(s.lights[2 * j]), kl = xyz(s.lights[2 * j + 1]);
            v3 l = sub(Lp, ip);
            float mg = mag(l);
            l = dvs(l, mg);
            mg *= mg;
            const float ndl = dot(n, l);
            const v3 h = normalize(add(l, v));  // lambert_blinn, raytracer.c:21-33
            const float coeff = fmaxf(0.0f, dot(n, h));
            const v3 cr = mk(kd.x * fmaxf(0.0f, ndl) + ks.x * coeff, kd.y * fmaxf(0.0f, ndl) + ks.y * coeff,
                             kd.z * fmaxf(0.0f, ndl) + ks.z * coeff);
            const int V = ((mask >> j) & 1u) ? (int)A.svis[((size_t)it * s.n_lights + j) * A.nslots + slot] : 0;
            const float fV = (float)V;
            col.x = col.x + fV * kl.x * cr.x / mg;
            col.y = col.y + fV * kl.y * cr.y / mg;
            col.z = col.z + fV * kl.z * cr.z / mg;
        }
        set3<MAXB>(cols, it, col);
        seti<MAXB>(mats, it, m);
    }
    const v3 col = clamp01(fold_path<MAXB>(s, cols, mats, L, (info & SPLIT_TAIL) != 0));
    store_px(A.rgb, A.bgra, (size_t)frame * A.frame_px + (size_t)k * A.W + x, col);
}

}  // namespace rtd
