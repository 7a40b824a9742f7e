// rt_output.hpp — the frame's output stage on the device: multi-GPU row gather and BMP quantisation.
#pragma once
#include <hip/hip_runtime.h>

namespace rtd {

// Compact rows of one context's frame (row k = image row off + (k / block) * stride + k % block, rt_frame)
// into the full frame. One thread per float4 of a row would need W % 4 == 0; rows are f32 x 3, so one
// thread per pixel.
__global__ __launch_bounds__(256) void k_unshuffle(const float* __restrict__ src, const int* __restrict__ src_hit,
                                                   float* __restrict__ dst, int* __restrict__ dst_hit, int W,
                                                   int off, int stride, int rows, int block) {
    const size_t n = (size_t)W * rows;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t k = i / W, x = i % W;
        const size_t o = ((size_t)off + (k / block) * stride + k % block) * W + x;
        dst[3 * o] = src[3 * i];
        dst[3 * o + 1] = src[3 * i + 1];
        dst[3 * o + 2] = src[3 * i + 2];
        if (dst_hit) dst_hit[o] = src_hit[i];
    }
}

// vec_to_bgra + bottom-up rows (cpu/src/bmp_writer.c:88-95,131-143): (uint8_t)(c * 255.0f) truncates
// toward zero exactly like the reference's C conversion (the product rounds once in f32 first).
__global__ __launch_bounds__(256) void k_bgra(const float* __restrict__ rgb, unsigned* __restrict__ out, int W, int H) {
    const size_t n = (size_t)W * H;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t y = i / W, x = i % W;
        const float* p = rgb + 3 * i;
        const unsigned r = (unsigned char)(p[0] * 255.0f), g = (unsigned char)(p[1] * 255.0f),
                       b = (unsigned char)(p[2] * 255.0f);
        out[(size_t)(H - 1 - y) * W + x] = b | (g << 8) | (r << 16) | (255u << 24);
    }
}

}  // namespace rtd
