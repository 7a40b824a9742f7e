// Checks on the GPU what rt_kernels.hpp's node test relies on (no reference data: plain IEEE arithmetic):
//   1. v_perm_b32(word, 0x64646464, 0x00050004 / 0x00070006) turns plane bytes q0, q1 (q2, q3) of a node word into two
//      f16 halves 0x6400 | q = 1024 + q (exact: f16 has an 11-bit significand);
//   2. v_fma_mix_f32 with an f16 source (low or high half) equals fmaf((float)(1024 + q), k, a) bit for bit, for every
//      q in 0..255 and 2^24 (k, a) pairs per q: random normal floats of all exponents and signs, and +-0, +-inf, NaN,
//      denormals, huge / tiny magnitudes.
// Prints the mismatch counts; exit status 0 iff both are 0. usage: tools/mix/mix_check (built by `make mix_check`)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

__device__ __forceinline__ float mix_lo(unsigned h2, float k, float a) {
    float r;
    __asm__("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h2), "v"(k), "v"(a));
    return r;
}
__device__ __forceinline__ float mix_hi(unsigned h2, float k, float a) {
    float r;
    __asm__("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h2), "v"(k), "v"(a));
    return r;
}
__device__ __forceinline__ unsigned hash(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ float special(unsigned h, unsigned r) {
    switch (h & 15u) {
        case 0: return 0.0f;
        case 1: return -0.0f;
        case 2: return __uint_as_float(0x7f800000u);
        case 3: return __uint_as_float(0xff800000u);
        case 4: return __uint_as_float(0x00000001u | (r & 0x807fffffu));  // denormal
        case 5: return __uint_as_float(0x7f000000u | (r & 0x807fffffu));  // huge
        default: return __uint_as_float(r & 0xff7fffffu | 0x00800000u);   // a normal of any exponent and sign
    }
}
__global__ void check(unsigned long long* bad_perm, unsigned long long* bad_mix, unsigned seed) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned q0 = i & 255u, q1 = (i >> 8) & 255u, q2 = hash(i) & 255u, q3 = hash(i * 7u) & 255u;
    const unsigned word = q0 | (q1 << 8) | (q2 << 16) | (q3 << 24);
    const unsigned lo2 = __builtin_amdgcn_perm(word, 0x64646464u, 0x00050004u);
    const unsigned hi2 = __builtin_amdgcn_perm(word, 0x64646464u, 0x00070006u);
    if (lo2 != ((0x6400u | q0) | ((0x6400u | q1) << 16)) || hi2 != ((0x6400u | q2) | ((0x6400u | q3) << 16)))
        atomicAdd(bad_perm, 1ull);
    unsigned long long bad = 0;
    for (int j = 0; j < 64; j++) {
        const unsigned h1 = hash(i * 131u + (unsigned)j * 977u + seed), h2 = hash(h1 ^ 0x9e3779b9u);
        const float k = (h1 >> 28) == 0 ? special(h1 >> 4, h2) : __uint_as_float((h2 & 0x80000000u) | (((h1 >> 8) % 254u + 1u) << 23) | (h2 & 0x7fffffu));
        const float a = (h2 >> 28) == 0 ? special(h2 >> 4, h1) : __uint_as_float((h1 & 0x80000000u) | (((h2 >> 8) % 254u + 1u) << 23) | (h1 & 0x7fffffu));
        const float want0 = __builtin_fmaf((float)(1024u + q0), k, a), want1 = __builtin_fmaf((float)(1024u + q1), k, a);
        const float got0 = mix_lo(lo2, k, a), got1 = mix_hi(lo2, k, a);
        const bool nan_ok0 = want0 != want0 && got0 != got0, nan_ok1 = want1 != want1 && got1 != got1;
        if (__float_as_uint(got0) != __float_as_uint(want0) && !nan_ok0) bad++;
        if (__float_as_uint(got1) != __float_as_uint(want1) && !nan_ok1) bad++;
    }
    if (bad) atomicAdd(bad_mix, bad);
}

int main() {
    unsigned long long *d = nullptr, h[2] = {0, 0};
    if (hipMalloc((void**)&d, 16) != hipSuccess) return 2;
    (void)hipMemset(d, 0, 16);
    const int blocks = 1 << 14, threads = 256;  // 2^22 threads x 64 pairs x 2 halves = 2^29 comparisons per pass
    for (unsigned pass = 0; pass < 4; pass++) check<<<blocks, threads>>>(d, d + 1, pass * 0x51ed27u);
    if (hipMemcpy(h, d, 16, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    std::printf("perm mismatches %llu, fma_mix mismatches %llu (of %llu comparisons)\n", h[0], h[1],
                4ull * blocks * threads * 128ull);
    return h[0] || h[1] ? 1 : 0;
}
