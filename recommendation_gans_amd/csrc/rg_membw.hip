// STREAM-style copy on the device: the achievable HBM ceiling that bench.py reports beside
// the 8 TB/s nominal peak (SURVEY §8d "measure a STREAM-copy ceiling on the box and report
// both").  One grid over the buffer, 4 float4 per thread, nontemporal loads and stores
// (measured on the box: 6.31 TB/s at 1 GiB; plain loads / stores 5.69, 8 per thread 4.3-4.4).
#include <algorithm>

#include "rg_common.h"

namespace rg {

namespace {

constexpr int kCopyThreads = 256;
typedef float v4f __attribute__((ext_vector_type(4)));

template <int PER, bool NT>
__global__ __launch_bounds__(kCopyThreads) void stream_copy_kernel(v4f *__restrict__ dst,
                                                                   const v4f *__restrict__ src, int64_t n) {
    const int64_t base = (int64_t)blockIdx.x * kCopyThreads * PER + threadIdx.x;
    v4f v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int64_t i = base + (int64_t)u * kCopyThreads;
        if (i < n) v[u] = NT ? __builtin_nontemporal_load(src + i) : src[i];
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int64_t i = base + (int64_t)u * kCopyThreads;
        if (i < n) {
            if (NT) __builtin_nontemporal_store(v[u], dst + i);
            else dst[i] = v[u];
        }
    }
}

template <int PER, bool NT>
void launch_copy(hipStream_t st, v4f *dst, const v4f *src, int64_t n) {
    const int64_t per_block = (int64_t)kCopyThreads * PER;
    const int64_t blocks = std::max<int64_t>(1, (n + per_block - 1) / per_block);
    hipLaunchKernelGGL((stream_copy_kernel<PER, NT>), dim3((unsigned)blocks), dim3(kCopyThreads), 0, st, dst, src, n);
}

}  // namespace

}  // namespace rg

extern "C" int rg_stream_copy(void *stream, float *dst, const float *src, int64_t n_float4) {
    if (!dst || !src || n_float4 < 0 || (reinterpret_cast<uintptr_t>(dst) & 15) || (reinterpret_cast<uintptr_t>(src) & 15))
        return rg::fail_arg("rg_stream_copy: bad argument (16-B aligned buffers of n_float4 float4)");
    if (n_float4 > ((int64_t)1 << 40)) return rg::fail_arg("rg_stream_copy: buffer too large");
    rg::launch_copy<4, true>((hipStream_t)stream, reinterpret_cast<rg::v4f *>(dst),
                             reinterpret_cast<const rg::v4f *>(src), n_float4);
    return rg::check_launch("rg_stream_copy");
}
