// rt_output.hpp — the frame's output stage on the device: multi-GPU row gather and BMP quantisation.
#pragma once
#include <hip/hip_runtime.h>

namespace rtd {

// Compact frames of one rank, [frames][rows][W][words] 32-bit words per pixel (3: f32 rgb, 1: BGRA8 or a
// hit index), into full frames [frames][H][W][words]: compact row k of frame f is image row
// start_f + (k / block) * stride + k % block with start_f = (off + f * shift) % stride when the rows rotate
// (rt_frame.frame_shift), else off; rows at or past H (a rotated rank's padding) are skipped.
__global__ __launch_bounds__(256) void k_unshuffle_frames(const unsigned* __restrict__ src, unsigned* __restrict__ dst,
                                                          int W, int H, int frames, int rows, int off, int stride,
                                                          int block, int shift, int words) {
    const size_t per = (size_t)rows * W, n = per * frames;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t f = i / per, r = i % per, k = r / W, x = r % W;
        const size_t start = shift ? ((size_t)off + f * shift) % stride : (size_t)off;
        const size_t y = start + (k / block) * stride + k % block;
        if (y >= (size_t)H) continue;
        const size_t o = (f * H + y) * W + x;
        for (int e = 0; e < words; e++) dst[o * words + e] = src[i * words + e];
    }
}

// Pixels of gathered frames that no rank's part wrote: the root fills the frames with a value no render writes
// (BGRA8: alpha 0 -- vec_to_bgra always writes 255; f32: NaN -- every pixel is clamped to [0, 1]) before the first
// gather of a layout, and counts what is left afterwards (rt_comm_gather's coverage check).
__global__ __launch_bounds__(256) void k_count_unwritten(const unsigned* __restrict__ px, size_t n, int words,
                                                         unsigned long long* __restrict__ count) {
    unsigned c = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        if (words == 1) c += (px[i] >> 24) != 255u ? 1u : 0u;
        else c += (px[3 * i] == 0xFFFFFFFFu || px[3 * i + 1] == 0xFFFFFFFFu || px[3 * i + 2] == 0xFFFFFFFFu) ? 1u : 0u;
    }
    if (c) atomicAdd(count, (unsigned long long)c);
}

// top-down BGRA8 rows -> the BMP file's bottom-up order (cpu/src/bmp_writer.c:131-143)
__global__ __launch_bounds__(256) void k_flip_rows(const unsigned* __restrict__ in, unsigned* __restrict__ out, int W, int H) {
    const size_t n = (size_t)W * H;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t y = i / W, x = i % W;
        out[(size_t)(H - 1 - y) * W + x] = in[i];
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
