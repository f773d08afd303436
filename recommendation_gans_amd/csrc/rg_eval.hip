// Top-k item ranking for the evaluation metrics (spotlight/evaluation.py:108-185,
// 192-213, 278-353: precision/recall@k, hit ratio and MAP@k read only the first k
// entries of each user's ranking, argsort(-scores)).
//
// One workgroup per user row: every thread keeps a sorted top-K of its strided slice
// of the row in registers (insertion, K <= kTopkMax), the 256 lists are merged in LDS
// by a tree of pairwise merges, and the row's k best item ids are written in rank
// order.  Order: higher score first, then the lower item id (numpy's default argsort
// leaves the order of equal scores unspecified; for distinct scores the ranking is
// the reference's).  Only users x k ids leave the device instead of the users x items
// score block.
#include <climits>

#include "rg_common.h"

namespace rg {
namespace {

constexpr int kTopkThreads = 256;
constexpr int kTopkMax = 32;

__device__ __forceinline__ bool topk_better(float a, int ia, float b, int ib) {
    return a > b || (a == b && ia < ib);
}

template <int K>
__global__ __launch_bounds__(kTopkThreads) void topk_kernel(const float *__restrict__ scores, int64_t cols, int64_t ld,
                                                            int k, int32_t *__restrict__ out) {
    __shared__ float sv[kTopkThreads * K];
    __shared__ int si[kTopkThreads * K];
    const int tid = threadIdx.x;
    const float *row = scores + (int64_t)blockIdx.x * ld;
    float v[K];
    int ix[K];
#pragma unroll
    for (int j = 0; j < K; ++j) { v[j] = -INFINITY; ix[j] = INT_MAX; }
    for (int64_t c = tid; c < cols; c += kTopkThreads) {
        float x = row[c];
        int xi = (int)c;
        if (x != x) x = -INFINITY;                       // NaN ranks last
        if (!topk_better(x, xi, v[K - 1], ix[K - 1])) continue;
        // insert: carry the displaced element down the sorted list (static indices only)
#pragma unroll
        for (int j = 0; j < K; ++j) {
            if (topk_better(x, xi, v[j], ix[j])) {
                const float tv = v[j];
                const int ti = ix[j];
                v[j] = x;
                ix[j] = xi;
                x = tv;
                xi = ti;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < K; ++j) { sv[tid * K + j] = v[j]; si[tid * K + j] = ix[j]; }
    __syncthreads();
    // tree merge: at stride s, thread t (t % 2s == 0) merges lists t and t + s into t
    for (int s = 1; s < kTopkThreads; s <<= 1) {
        if ((tid & (2 * s - 1)) == 0) {
            const float *av = sv + tid * K, *bv = sv + (tid + s) * K;
            const int *ai = si + tid * K, *bi = si + (tid + s) * K;
            float mv[K];
            int mi[K];
            int p = 0, q = 0;
            for (int j = 0; j < k; ++j) {
                const bool take_a = topk_better(av[p], ai[p], bv[q], bi[q]);
                mv[j] = take_a ? av[p] : bv[q];
                mi[j] = take_a ? ai[p] : bi[q];
                p += take_a ? 1 : 0;
                q += take_a ? 0 : 1;
            }
            for (int j = 0; j < k; ++j) { sv[tid * K + j] = mv[j]; si[tid * K + j] = mi[j]; }
        }
        __syncthreads();
    }
    if (tid < k) out[(int64_t)blockIdx.x * k + tid] = si[tid];
}

}  // namespace
}  // namespace rg

using namespace rg;

extern "C" int rg_topk_rows(void *stream, const float *scores, int64_t rows, int64_t cols, int64_t ld, int32_t k,
                            int32_t *out_idx) {
    if (!scores || !out_idx) return fail_arg("rg_topk_rows: null argument");
    if (rows < 0 || cols < 1 || ld < cols) return fail_arg("rg_topk_rows: bad shape");
    if (k < 1 || k > kTopkMax || k > cols) return fail_arg("rg_topk_rows: k must be in [1, min(32, cols)]");
    if (cols > INT_MAX) return fail_arg("rg_topk_rows: cols must fit int32");
    if (rows == 0) return RG_OK;
    if (rows > INT_MAX) return fail_arg("rg_topk_rows: too many rows for one launch");
    const dim3 grid((unsigned)rows), block(kTopkThreads);
    const hipStream_t s = (hipStream_t)stream;
    if (k <= 8)
        hipLaunchKernelGGL((topk_kernel<8>), grid, block, 0, s, scores, cols, ld, k, out_idx);
    else if (k <= 16)
        hipLaunchKernelGGL((topk_kernel<16>), grid, block, 0, s, scores, cols, ld, k, out_idx);
    else
        hipLaunchKernelGGL((topk_kernel<32>), grid, block, 0, s, scores, cols, ld, k, out_idx);
    return check_launch("rg_topk_rows");
}
