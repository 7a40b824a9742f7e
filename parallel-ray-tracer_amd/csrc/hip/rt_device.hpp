// rt_device.hpp — device-side data layout and the exact-arithmetic primitives of the hot path.
//
// Everything here is written for CDNA4 (gfx950, wave64) and compiled with -ffp-contract=off,
// no fast-math and IEEE-correct fp32 division / sqrt, so that each primitive rounds exactly like the
// reference's C (cpu/src/vec.c, raytracer.c, bvh.c) compiled strict (SURVEY §8c "O-strict").
#pragma once
#include <hip/hip_runtime.h>

namespace rtd {

constexpr float EPS = 1e-3f;             // EPSILON, cpu/src/raytracer.c:19
constexpr float FMAX = 3.402823466e+38f; // FLT_MAX
constexpr int EMPTY_REF = (int)0x80000000; // empty child (bvh_t child == 0 && tr_len == 0): never pushed

// ---------------------------------------------------------------- device scene (HBM layout)
// nodes   : one 64-B record per INTERIOR reference node (child-pair layout): both child boxes +
//           both child refs, loaded with 4 x global_load_dwordx4 per visit.
//             f4[0] = lo0.x lo0.y lo0.z hi0.x   f4[1] = hi0.y hi0.z lo1.x lo1.y
//             f4[2] = lo1.z hi1.x hi1.y hi1.z   f4[3] = ref0 ref1 (int bits) 0 0
//           ref >= 0: interior record index; ref < 0: leaf ~ref; EMPTY_REF: empty node.
// leaves  : int2 (first, count) into the leaf-ordered triangle arrays (= bvh_t tr_idx, tr_len)
// tris    : 48 B per leaf-ordered triangle: v0, e1 = v1 - v0, e2 = v2 - v0, n = e1 x e2
//             f4[0] = v0.x v0.y v0.z e1.x  f4[1] = e1.y e1.z e2.x e2.y  f4[2] = e2.z n.x n.y n.z
//           (the reference recomputes e1, e2, n per test, raytracer.c:36-38; same roundings)
// tri_orig: leaf position -> original triangle index (= tri_idx)
// shade   : 32 B per ORIGINAL triangle: f4[0] = norm[0].xyz, material id (int bits); f4[1] = norm[1].xyz, 0
// mats    : 48 B per distinct (ks, kd, kr): f4[0] = ks, f4[1] = kd, f4[2] = kr
// lights  : 32 B per light: f4[0] = pos, f4[1] = kl
// One BVH in device layout. A scene carries two: `ref`, the reference's own bvh_build output
// (traversed by the strict walk, in the reference's order), and `acc`, the acceleration BVH the fast
// walk uses (binned SAH by default; may alias `ref`). Triangle planes are stored per BVH in its leaf order.
struct DBvh {
    const float4* __restrict__ nodes;
    const int2* __restrict__ leaves;
    const float4* __restrict__ tris;
    const int* __restrict__ tri_orig;
    int root;
};

// The fast walk's 8-wide quantised BVH (rt_wide.cpp; replaces `acc` when present). 80-B nodes:
//   f4[0] = p.x p.y p.z | bits: e.x, e.y, e.z (signed bytes), imask (bytes 0..3)
//   f4[1] = child_base, tri_base, meta[0..3], meta[4..7]
//   f4[2] = the x planes, f4[3] = y, f4[4] = z: word j = bytes qlo[2j], qhi[2j], qlo[2j+1], qhi[2j+1]
// child box plane = fmaf(2^e, 1024 + q, p) (exact product, one rounding; the bias makes 1024 + q an f16 integer whose
// bits are 0x6400 | q, rt_kernels.hpp fma_half); slot s holds the child in octant s
// of the node (bit 0 = +x, 1 = +y, 2 = +z). imask bit s: slot s is an interior node, at
// child_base + popc(imask & (2^s - 1)); otherwise meta[s] = count << 5 | offset: triangles
// tri_base + offset .. + count - 1 (count 1..4; meta 0 = empty slot).
struct DWide {
    const float4* __restrict__ nodes;  // nullptr: no wide view (the fast walk uses `acc`)
    const float4* __restrict__ tris;   // 48-B triangle records in wide-leaf order
    const int* __restrict__ tri_orig;  // wide-leaf position -> original triangle index
    int n;                             // wide nodes (the LDS staging of the top levels copies min(n, NTOP) of them)
};

struct DScene {
    DBvh ref, acc;
    DWide wide;
    const float4* __restrict__ shade;
    const float4* __restrict__ mats;
    const float4* __restrict__ lights;
    int n_lights;
    float amb_x, amb_y, amb_z;
    // every face coordinate of the reference tree's child boxes, per axis, sorted: [n_face[0] x][n_face[1] y]
    // [n_face[2] z] (rt_hip.hip upload; nullable): a ray with a zero direction component whose origin lies on no face
    // of that axis divides no 0 by 0 in the reference's slab test, which then culls nothing the ordinary test keeps,
    // so it may take the fast walk (rt_kernels.hpp degenerate_ok)
    int n_face[3];
    const float* __restrict__ faces;
    // the reference tree's paths (rt_hip.hip build_view): [n_tris: original triangle -> its leaf][leaf -> the record
    // holding its box]; a record's parent is its 4th float4's z (-1: the root). rt_kernels.hpp ref_reaches
    const int* __restrict__ ref_path;
    int n_tris;
    int pad_path;
    // the fast walk's view for unit-length directions (reflection and shadow rays): `wide` without the triangles
    // no such ray can hit — hit_triangle culls |det| < EPS and |det| <= |n| |d| (rt_hip.hip unit_view); nodes ==
    // nullptr: `wide` serves every ray
    DWide unit;
    // the view for this launch's primary rays: `wide` without the triangles no direction of length <= PRIMARY_D can
    // hit (the host sets it only when every primary direction of the frame is that short); nullptr: `wide`
    DWide prim;
};

struct KArgs {
    DScene s;
    float pos[3], ul[3], ix[3], iy[3];
    int W, H, row_offset, row_stride, n_rows, bounces, spp, spp_grid;
    float* rgb;
    int* hit;
    float* t;
    int* bounce_hit;               // nullable: [n_rows][W][bounces] per-level closest hit (-1 miss, -2 unreached)
    unsigned long long* counters;  // RT_NCOUNT slots (rt_stats order)
    unsigned int* work;            // persistent-kernel tile / pixel counter
    int n_tiles, tiles_x;
    int regroup;                   // shadow pool: idle lanes of a wave that trigger a refill (rt_frame.regroup)
    unsigned long long* tile_trace;  // diagnostics (PRT_TILE_TRACE): per-tile timeline (rt_kernels.hpp)
    const int* tile_order;           // nullable: k-th dealt tile = tile_order[k] (default: row-major)
    // frame batches (rt_render_frames): n_frames frames of the same shape, frame f's camera at
    // cams[12 f .. 12 f + 11] (pos, ul, inc_x, inc_y; nullable when n_frames == 1: the fields above),
    // its outputs at pixel offset f * frame_px (frame_px = n_rows * W)
    const float* cams;
    int n_frames;
    int row_block;  // rows in blocks of row_block (>= 1): image row of compact row k = image_row()
    unsigned long long frame_px;
    // PB kernels: each level's colour + material of a lane's path, [wave][level][lane] (rt_kernels.hpp)
    float4* pathbuf;
    // DYN kernels: the wide walk's stack in dynamic LDS (wcap 2-int entries per lane = the scene's wide
    // depth), the binary walks' stacks in global memory (gstack: [block][STACK][256] ints)
    int* gstack;
    int wcap;
    int frame_shift;  // rt_frame.frame_shift: frame f's rows start at (row_offset + f * frame_shift) % row_stride
    // XCD-aware dealing (nullable): tile_order holds 8 spatial regions' tiles, region r at
    // [region_off[r], region_off[r + 1]); workgroup b (on XCD b % 8) drains region b % 8 first
    const int* region_off;
    // nullable: the frame quantised on the fly (rt_outputs.bgra), one packed B|G<<8|R<<16|255<<24 per pixel
    unsigned* bgra;
    // spp > 1 (the persistent kernels' multi-sample builds): one float4 per resident lane, [block][lane], holding the
    // pixel's running sum of clamped samples across the sample loop, so that no register stays live across a sample's
    // path (at the 4-wave kernels' 128-VGPR cap such values spilled inside the walks)
    float4* lanebuf;
    // spp > 1 in the kernels with an LDS path buffer (PB = 2): the same slots in dynamic LDS instead, [wave][lane] from
    // int offset slot_off (the host appends them to the launch's LDS layout), so that the per-sample sums never leave
    // the CU (64 spp at 4K: 530 M slot updates per frame)
    int slot_off;
    // single frames under the default rule's feedback (RT_VARIANT_HYBRID, rt_feedback.hpp; nullable): every 8x8 tile's
    // duration in s_memrealtime ticks (k_persist: stored; k_coop: the maximum of its tiles', scaled, by atomic max), from
    // which the next frame's tile lists are built on the device
    unsigned* tile_cost;
    // nullable: the number of tiles to deal, in device memory (k_coop over a list whose length the device built)
    const int* n_tiles_dev;
    int tiles_x8;  // 8x8 tiles per row of the frame (k_coop's tile_cost index)
    int pad_fb;
};

// Kernel arguments are laid out by the host compiler and read by the device compiler: both passes must
// agree on every offset (an LDS pointer, 32-bit on gfx950 but 64-bit on the host, once shifted every
// later field and hung a kernel). Pinned sizes catch such drift at compile time in whichever pass
// disagrees; never put address-space-qualified pointers in these structs.
static_assert(sizeof(DWide) == 32 && sizeof(DScene) == 256 && sizeof(KArgs) == 520,
              "kernel-argument layout changed: update the pinned sizes only after checking both passes agree");

// ---------------------------------------------------------------- vec_t arithmetic (cpu/src/vec.c)
struct v3 {
    float x, y, z;
};
__device__ __forceinline__ v3 mk(float x, float y, float z) { return v3{x, y, z}; }
__device__ __forceinline__ v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 mul(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ v3 dvs(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float mag(v3 a) { return __builtin_sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
__device__ __forceinline__ v3 cross(v3 a, v3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ v3 normalize(v3 a) { return dvs(a, mag(a)); }
__device__ __forceinline__ v3 xyz(float4 f) { return mk(f.x, f.y, f.z); }

// One finished pixel (o = frame-relative output index) to the frame's outputs: the f32 vec_t pixel
// (main.c:39) and/or its BMP quantisation vec_to_bgra (cpu/src/bmp_writer.c:88-95; as k_bgra, but in
// the frame's top-down row order), so that a quantised frame never takes a second pass over HBM.
__device__ __forceinline__ void store_px(float* __restrict__ rgb, unsigned* __restrict__ bgra, size_t o, v3 col) {
    if (rgb) {
        rgb[3 * o] = col.x;
        rgb[3 * o + 1] = col.y;
        rgb[3 * o + 2] = col.z;
    }
    if (bgra) {
        const unsigned r = (unsigned char)(col.x * 255.0f), g = (unsigned char)(col.y * 255.0f),
                       b = (unsigned char)(col.z * 255.0f);
        bgra[o] = b | (g << 8) | (r << 16) | (255u << 24);
    }
}

// ---------------------------------------------------------------- ray-triangle (raytracer.c:35-59)
// v0, e1, e2, n precomputed on the host with the reference's own roundings.
// The correctly rounded 1.0f / x for |x| <= 2^125: v_rcp_f32 (1 ulp) and one FMA correction (Markstein) give
// IEEE division's bits there -- checked for EVERY normal float of both signs on the GPU (tools/rcp/
// rcp_exhaustive.hip: the only mismatches are |x| >= 2^126, denormal results) -- in 3 instructions instead of
// the division's scale / fmas / fixup sequence; above 2^125 the division itself. Used by the closest walks'
// triangle tests (FAST_RCP): same box, dragon 0.801 vs 0.803 ms per frame, car_boxed 0.870 vs 0.882, sportscar
// 1.328 vs 1.332; in the shadow walks too it cost dragon 2.5 % (profiles/r2l/ab_fast_reciprocal*.txt). Also
// ray_pre's 1/d of every walk: dragon 0.796 vs 0.803, car_boxed 0.864 vs 0.871.
__device__ __forceinline__ float rcp_ieee(float x) {
    if (__builtin_fabsf(x) > 0x1p125f) return 1.0f / x;
    const float r = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
}
template <bool FAST_RCP = false>
__device__ __forceinline__ float hit_triangle_v(v3 o, v3 d, float4 a, float4 b, float4 c, int& nd) {
    const v3 v0 = mk(a.x, a.y, a.z), e1 = mk(a.w, b.x, b.y), e2 = mk(b.z, b.w, c.x), n = mk(c.y, c.z, c.w);
    const float det = -dot(d, n);
    nd = det < 0.0f;
    if (__builtin_fabsf(det) < EPS) return FMAX;
    const float inv = FAST_RCP ? rcp_ieee(det) : 1.0f / det;
    const v3 ao = sub(o, v0);
    const v3 dao = cross(ao, d);
    const float u = dot(e2, dao) * inv;
    const float v = -dot(e1, dao) * inv;
    const float t = dot(ao, n) * inv;
    if (t > EPS && u >= 0.0f && v >= 0.0f && (u + v) <= 1.0f) return t;
    return FMAX;
}
template <bool FAST_RCP = false>
__device__ __forceinline__ float hit_triangle(v3 o, v3 d, const float4* __restrict__ tri, int& nd) {
    return hit_triangle_v<FAST_RCP>(o, d, tri[0], tri[1], tri[2], nd);
}

// ---------------------------------------------------------------- exact slab test (bvh.c:48-59)
__device__ __forceinline__ float box_exact(v3 lo, v3 hi, v3 o, v3 d) {
    float tx1 = (lo.x - o.x) / d.x, tx2 = (hi.x - o.x) / d.x;
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    float ty1 = (lo.y - o.y) / d.y, ty2 = (hi.y - o.y) / d.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2));
    tmax = fminf(tmax, fmaxf(ty1, ty2));
    float tz1 = (lo.z - o.z) / d.z, tz2 = (hi.z - o.z) / d.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2));
    tmax = fminf(tmax, fmaxf(tz1, tz2));
    return (tmax >= tmin && tmax > 0) ? tmin : FMAX;
}
// box_exact's entry (bit for bit: the same operations) and the slab's exit in `out` (the tie re-walk's cut)
__device__ __forceinline__ float box_exact_out(v3 lo, v3 hi, v3 o, v3 d, float& out) {
    float tx1 = (lo.x - o.x) / d.x, tx2 = (hi.x - o.x) / d.x;
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    float ty1 = (lo.y - o.y) / d.y, ty2 = (hi.y - o.y) / d.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2));
    tmax = fminf(tmax, fmaxf(ty1, ty2));
    float tz1 = (lo.z - o.z) / d.z, tz2 = (hi.z - o.z) / d.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2));
    tmax = fminf(tmax, fmaxf(tz1, tz2));
    out = tmax;
    return (tmax >= tmin && tmax > 0) ? tmin : FMAX;
}

// ---------------------------------------------------------------- reciprocal slab test (fast kernel)
// t = lo * inv - o * inv via one FMA per plane; tmax widened by 2 ulp so that the test never rejects
// a box the exact test accepts (culling/order only; triangle tests stay exact).
struct RayPre {
    float ix, iy, iz, ox, oy, oz;  // 1/d and o/d (as o * (1/d))
};
// A zero direction component would give inf * 0 = NaN planes (and a NaN-swallowing fminf/fmaxf
// could then reject a box the ray passes through): such components are replaced by +1e-20, for which
// the slab degenerates to [-huge, +huge] (ray inside) or a same-signed huge pair (ray outside).
__device__ __forceinline__ float safe_dir(float x) { return __builtin_fabsf(x) < 1e-20f ? 1e-20f : x; }
__device__ __forceinline__ RayPre ray_pre(v3 o, v3 d) {
    RayPre p;
    p.ix = rcp_ieee(safe_dir(d.x));
    p.iy = rcp_ieee(safe_dir(d.y));
    p.iz = rcp_ieee(safe_dir(d.z));
    p.ox = o.x * p.ix;
    p.oy = o.y * p.iy;
    p.oz = o.z * p.iz;
    return p;
}
__device__ __forceinline__ float box_fast(float lx, float ly, float lz, float hx, float hy, float hz,
                                          const RayPre& p) {
    const float tx1 = __builtin_fmaf(lx, p.ix, -p.ox), tx2 = __builtin_fmaf(hx, p.ix, -p.ox);
    const float ty1 = __builtin_fmaf(ly, p.iy, -p.oy), ty2 = __builtin_fmaf(hy, p.iy, -p.oy);
    const float tz1 = __builtin_fmaf(lz, p.iz, -p.oz), tz2 = __builtin_fmaf(hz, p.iz, -p.oz);
    const float tmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    const float tmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2)) * 1.00000024f;
    return (tmax >= tmin && tmax > 0) ? tmin : FMAX;
}

}  // namespace rtd
