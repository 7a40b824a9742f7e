// Exhaustive check (every finite normal float, both signs) that rcp_ieee(x) -- v_rcp_f32 plus one FMA
// Newton-Markstein correction -- equals the correctly rounded 1.0f / x (the reference's division in
// hit_triangle, raytracer.c:35-59). Reports the mismatches per exponent range. Test infrastructure only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float rcp_fast(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}

__global__ void k(uint32_t base, unsigned long long* bad, uint32_t* first, unsigned* hist) {
    const uint32_t i = base + blockIdx.x * 256u + threadIdx.x;
    const uint32_t bits = i;
    const uint32_t ex = (bits >> 23) & 0xFF;
    if (ex == 0 || ex == 0xFF) return;  // denormals, inf/nan: outside the kernel's |det| >= EPS range
    const float x = __uint_as_float(bits);
    const float a = 1.0f / x, b = rcp_fast(x);
    if (__float_as_uint(a) != __float_as_uint(b)) {
        const unsigned long long n = atomicAdd(bad, 1ull);
        atomicAdd(hist + ex, 1u);
        if (n < 16) first[n] = bits;
    }
}

int main() {
    unsigned long long* bad;
    uint32_t* first;
    unsigned* hist;
    hipMalloc(&bad, 8);
    hipMalloc(&first, 64);
    hipMalloc(&hist, 256 * 4);
    hipMemset(bad, 0, 8);
    hipMemset(first, 0, 64);
    hipMemset(hist, 0, 1024);
    const uint32_t chunk = 1u << 28;
    for (uint64_t b = 0; b < (1ull << 32); b += chunk) k<<<chunk / 256, 256>>>((uint32_t)b, bad, first, hist);
    if (hipDeviceSynchronize() != hipSuccess) { printf("hip error\n"); return 2; }
    unsigned long long nb;
    uint32_t f[16];
    unsigned h[256];
    hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(f, first, 64, hipMemcpyDeviceToHost);
    hipMemcpy(h, hist, 1024, hipMemcpyDeviceToHost);
    printf("mismatches %llu of all normal floats (both signs)\n", nb);
    for (int i = 0; i < 16 && i < (int)nb; i++) printf("  0x%08x %g\n", f[i], (double)*(float*)&f[i]);
    for (int e = 0; e < 256; e++) if (h[e]) printf("  exponent field %d: %u\n", e, h[e]);
    return nb ? 1 : 0;
}
