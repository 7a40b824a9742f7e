// rt_build.hpp — GPU-side build of the fast walk's BVH: PLOC (Meister & Bittner, "Parallel
// Locally-Ordered Clustering for Bounding Volume Hierarchy Construction", TVCG 2018) over Morton-sorted
// triangle centroids, on the device.
//
//   1. k_prim_boxes   triangle boxes and the centroid bounds (wave min/max, one ordered-int atomic per wave)
//   2. k_morton       30-bit Morton code of each centroid in the centroid bounds
//   3. radix sort     (hipcub) of (code, triangle): clusters start as the sorted leaves
//   4. PLOC rounds    k_nn: every cluster's nearest neighbour (smallest merged surface area) within +-R
//                     positions of the sorted cluster array; mutually nearest pairs merge into a new node
//                     (k_flags, scans, k_merge: node ids by prefix sum, so the tree is deterministic), the
//                     survivors are compacted (k_compact) — until one cluster is left
// The binary tree (children, boxes) goes back to the host, where rt_hip.hip lays it out as a reference-layout
// BVH (children consecutive, leaf triangles in depth-first order so that every subtree's triangles are one
// range) and the 8-wide collapse + outward quantisation (rt_wide.cpp) runs as for the host-built tree. Any
// conservative BVH renders the same bits (the fast walk returns the minimum t over all triangles, ties
// re-walked strictly), so the tree only changes speed.
#pragma once
#include <hip/hip_runtime.h>

namespace rtb {

constexpr int PLOC_R = 32;      // default neighbourhood radius (rt_scene.ploc_radius); 8 / 16 / 32 / 64 measured, DESIGN.md
constexpr int PLOC_R_MAX = 64;

__device__ __forceinline__ int f2o(float f) {  // float -> int with the same order (for atomicMin / atomicMax)
    const int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float o2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7FFFFFFF); }

// v: 9 floats per triangle (the reference's coords[3]); cb: 6 ordered ints (centroid min xyz, max xyz)
__global__ __launch_bounds__(256) void k_prim_boxes(const float* __restrict__ v, int n, float4* __restrict__ lo,
                                                    float4* __restrict__ hi, int* __restrict__ cb) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float c[3] = {INFINITY, INFINITY, INFINITY}, C[3] = {-INFINITY, -INFINITY, -INFINITY};
    if (i < n) {
        const float* p = v + 9 * (size_t)i;
        float l[3], h[3];
        for (int a = 0; a < 3; a++) {
            l[a] = fminf(fminf(p[a], p[3 + a]), p[6 + a]);
            h[a] = fmaxf(fmaxf(p[a], p[3 + a]), p[6 + a]);
            c[a] = C[a] = 0.5f * (l[a] + h[a]);
        }
        lo[i] = make_float4(l[0], l[1], l[2], 0.0f);
        hi[i] = make_float4(h[0], h[1], h[2], 0.0f);
    }
    for (int a = 0; a < 3; a++) {
        for (int off = 32; off > 0; off >>= 1) {
            c[a] = fminf(c[a], __shfl_xor(c[a], off, 64));
            C[a] = fmaxf(C[a], __shfl_xor(C[a], off, 64));
        }
    }
    if ((threadIdx.x & 63) == 0)
        for (int a = 0; a < 3; a++) {
            atomicMin(cb + a, f2o(c[a]));
            atomicMax(cb + 3 + a, f2o(C[a]));
        }
}

__device__ __forceinline__ unsigned expand10(unsigned v) {  // 10 bits -> every third bit of 30
    v &= 1023u;
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__global__ __launch_bounds__(256) void k_morton(const float4* __restrict__ lo, const float4* __restrict__ hi, int n,
                                                const int* __restrict__ cb, unsigned* __restrict__ keys,
                                                int* __restrict__ vals) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 l = lo[i], h = hi[i];
    const float c[3] = {0.5f * (l.x + h.x), 0.5f * (l.y + h.y), 0.5f * (l.z + h.z)};
    unsigned q[3];
    for (int a = 0; a < 3; a++) {
        const float mn = o2f(cb[a]), ext = o2f(cb[3 + a]) - mn;
        const float u = ext > 0.0f ? (c[a] - mn) / ext : 0.5f;
        q[a] = (unsigned)fminf(fmaxf(u * 1024.0f, 0.0f), 1023.0f);
    }
    keys[i] = (expand10(q[0]) << 2) | (expand10(q[1]) << 1) | expand10(q[2]);
    vals[i] = i;
}

// leaves: node k = sorted triangle sorted[k]; the clusters start as the leaves in Morton order
__global__ __launch_bounds__(256) void k_leaves(const int* __restrict__ sorted, const float4* __restrict__ plo,
                                                const float4* __restrict__ phi, int n, float4* __restrict__ nlo,
                                                float4* __restrict__ nhi, int* __restrict__ C) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const int t = sorted[k];
    nlo[k] = plo[t];
    nhi[k] = phi[t];
    C[k] = k;
}

__device__ __forceinline__ float merged_area(float4 alo, float4 ahi, float4 blo, float4 bhi) {
    const float dx = fmaxf(ahi.x, bhi.x) - fminf(alo.x, blo.x), dy = fmaxf(ahi.y, bhi.y) - fminf(alo.y, blo.y),
                dz = fmaxf(ahi.z, bhi.z) - fminf(alo.z, blo.z);
    return dx * dy + dy * dz + dz * dx;
}

// nearest neighbour of cluster i among positions [i - R, i + R] (the smallest merged area; ties: the lower
// position). Each block stages its clusters' boxes plus a halo of R on either side in LDS.
__global__ __launch_bounds__(256) void k_nn(const int* __restrict__ C, int m, const float4* __restrict__ nlo,
                                            const float4* __restrict__ nhi, int* __restrict__ nn, int R) {
    __shared__ float4 slo[256 + 2 * PLOC_R_MAX], shi[256 + 2 * PLOC_R_MAX];
    const int base = blockIdx.x * 256 - R;
    for (int s = threadIdx.x; s < 256 + 2 * R; s += 256) {
        const int j = base + s;
        if (j >= 0 && j < m) {
            const int c = C[j];
            slo[s] = nlo[c];
            shi[s] = nhi[c];
        }
    }
    __syncthreads();
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const int si = threadIdx.x + R;
    const float4 alo = slo[si], ahi = shi[si];
    float best = INFINITY;
    int bj = -1;
    const int j0 = i - R < 0 ? 0 : i - R, j1 = i + R >= m ? m - 1 : i + R;
    for (int j = j0; j <= j1; j++) {
        if (j == i) continue;
        const float a = merged_area(alo, ahi, slo[j - base], shi[j - base]);
        if (a < best) {
            best = a;
            bj = j;
        }
    }
    nn[i] = bj;
}

// mflag[i]: i merges with its mutual nearest neighbour nn[i] > i (i keeps the new node);
// keep[i]: i survives the round (it is not the higher partner of a merged pair)
__global__ __launch_bounds__(256) void k_flags(const int* __restrict__ nn, int m, int* __restrict__ mflag,
                                               int* __restrict__ keep) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int j = nn[i];
    const bool mutual = j >= 0 && nn[j] == i;
    mflag[i] = mutual && i < j;
    keep[i] = !(mutual && i > j);
}

// node id base + moff[i] = union of C[i] and C[nn[i]]; children of internal node id at left / right[id - n]
__global__ __launch_bounds__(256) void k_merge(int* __restrict__ C, const int* __restrict__ nn,
                                               const int* __restrict__ mflag, const int* __restrict__ moff, int m,
                                               int n, int base, float4* __restrict__ nlo, float4* __restrict__ nhi,
                                               int* __restrict__ left, int* __restrict__ right) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m || !mflag[i]) return;
    const int a = C[i], b = C[nn[i]], id = base + moff[i];
    const float4 alo = nlo[a], ahi = nhi[a], blo = nlo[b], bhi = nhi[b];
    nlo[id] = make_float4(fminf(alo.x, blo.x), fminf(alo.y, blo.y), fminf(alo.z, blo.z), 0.0f);
    nhi[id] = make_float4(fmaxf(ahi.x, bhi.x), fmaxf(ahi.y, bhi.y), fmaxf(ahi.z, bhi.z), 0.0f);
    left[id - n] = a;
    right[id - n] = b;
    C[i] = id;
}

__global__ __launch_bounds__(256) void k_compact(const int* __restrict__ C, const int* __restrict__ keep,
                                                 const int* __restrict__ koff, int m, int* __restrict__ C2) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m && keep[i]) C2[koff[i]] = C[i];
}

}  // namespace rtb
