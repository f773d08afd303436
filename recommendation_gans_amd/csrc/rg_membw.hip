// STREAM-style copy on the device: the achievable HBM ceiling that bench.py reports beside
// the 8 TB/s nominal peak (SURVEY §8d "measure a STREAM-copy ceiling on the box and report
// both").  Grid-stride float4 copy, 8 loads in flight per thread, XCD-spread blocks.
#include "rg_common.h"

namespace rg {

namespace {

constexpr int kCopyThreads = 256, kCopyUnroll = 8;

__global__ __launch_bounds__(kCopyThreads) void stream_copy_kernel(float4 *__restrict__ dst,
                                                                   const float4 *__restrict__ src, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * kCopyThreads * kCopyUnroll;
    for (int64_t base = (int64_t)blockIdx.x * kCopyThreads * kCopyUnroll + threadIdx.x; base < n; base += stride) {
        float4 v[kCopyUnroll];
#pragma unroll
        for (int u = 0; u < kCopyUnroll; ++u) {
            const int64_t i = base + (int64_t)u * kCopyThreads;
            if (i < n) v[u] = src[i];
        }
#pragma unroll
        for (int u = 0; u < kCopyUnroll; ++u) {
            const int64_t i = base + (int64_t)u * kCopyThreads;
            if (i < n) dst[i] = v[u];
        }
    }
}

}  // namespace

}  // namespace rg

extern "C" int rg_stream_copy(void *stream, float *dst, const float *src, int64_t n_float4) {
    if (!dst || !src || n_float4 < 0 || (reinterpret_cast<uintptr_t>(dst) & 15) || (reinterpret_cast<uintptr_t>(src) & 15))
        return rg::fail_arg("rg_stream_copy: bad argument (16-B aligned buffers of n_float4 float4)");
    const int64_t per_block = (int64_t)rg::kCopyThreads * rg::kCopyUnroll;
    int64_t blocks = (n_float4 + per_block - 1) / per_block;
    const int64_t cap = 8 * (int64_t)rg::num_cus();   // a few waves of blocks per CU, grid-stride beyond
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(rg::stream_copy_kernel, dim3((unsigned)blocks), dim3(rg::kCopyThreads), 0, (hipStream_t)stream,
                       reinterpret_cast<float4 *>(dst), reinterpret_cast<const float4 *>(src), n_float4);
    return rg::check_launch("rg_stream_copy");
}
