// fp32 GEMM on the gfx950 matrix cores (v_mfma_f32_32x32x2_f32, exact f32 fma
// chains) with the fused epilogues the cGAN step needs (rg_gemm.hip).
//
//   C[m][n] = sum_k A(m, k) * B(n, k)
//
// A is given K-major (A[m * lda + k]) or M-major (A[k * lda + m]); likewise B
// (B[n * ldb + k] or B[k * ldb + n]).  Leading dimensions, M/N of a contiguous
// dimension and K are multiples of 4 and base pointers are 16-B aligned (the
// launcher checks), so a float4 is either wholly inside or wholly outside.
#pragma once
#include <algorithm>

#include "rg_common.h"

namespace rg {

enum GemmEpi {
    kEpiStore = 0,    // C = post(acc + bias[n])                   (splits == 1)
    kEpiPartial = 1,  // C + z * M * N  <- acc (split-K partial, row stride N)
    kEpiOpt = 2,      // in-place optimizer update of P[m][n] with g = acc + hits
    kEpiArgmax = 3,   // per (row, column tile, head segment) argmax of tanh(acc + bias[n])
};

enum GemmPost {
    kPostNone = 0,
    kPostTanh = 1,       // tanh(v)
    kPostTanhGrad = 2,   // v * (1 - T[m][n]^2), column sums per row tile into colsum
    kPostLreluGrad = 3,  // v * (U[m][n] > 0 ? 1 : 0.2) * (Mult ? Mult[m][n] : 1)
};

constexpr int kGemmBM = 128, kGemmBN = 128, kGemmBK = 32;

struct GemmDesc {
    const float *A = nullptr;
    int64_t lda = 0;
    bool a_kmajor = true;
    const float *B = nullptr;
    int64_t ldb = 0;
    bool b_kmajor = true;
    int64_t M = 0, N = 0, K = 0;
    int splits = 1;           // > 1 only with kEpiPartial
    float clamp_b = 0.0f;     // > 0: B operand clamped to [-clamp_b, clamp_b] on load
    int epi = kEpiStore;
    // store / partial
    float *C = nullptr;
    int64_t ldc = 0;
    const float *bias = nullptr;
    int post = kPostNone;
    const float *T = nullptr;     // tanh-grad operand / lrelu-grad U
    int64_t ldt = 0;
    const float *Mult = nullptr;  // lrelu-grad multiplier (dropout), same stride as T
    float *colsum = nullptr;      // tanh-grad: colsum[row_tile * N + n]
    // optimizer epilogue: P (and its state) [m][n] with row stride ldp
    float *P = nullptr, *Ms = nullptr, *Vs = nullptr;
    int64_t ldp = 0;
    rg_opt_t opt{};
    float clamp_p = 0.0f;         // > 0: p clamped before its update (the D step's clip)
    // sparse extra rows of the gradient: hit h adds hit_src[hit_row[h] * hit_ld + m] to
    // column hit_col[h] (hits sorted by column, then row)
    const int32_t *hit_col = nullptr, *hit_row = nullptr;
    const int32_t *hit_tile_off = nullptr;   // [column tiles + 1]: hits of tile t are [off[t], off[t+1])
    int32_t n_hits = 0;
    const float *hit_src = nullptr;
    int64_t hit_ld = 0;
    // argmax: heads of `seg` columns; amax[(m * n_tiles + tile) * 2 + s] = (value, index)
    int64_t seg = 0;
    float2 *amax = nullptr;
};

int gemm(hipStream_t stream, const GemmDesc &d);

// C[m][n] = sum_{z < splits} part[z][m][n] (in split order) + bias[n]
int reduce_partials(hipStream_t stream, const float *part, int splits, int64_t M, int64_t N, float *C, int64_t ldc,
                    const float *bias);

__host__ __device__ inline int64_t gemm_tiles_n(int64_t N) { return (N + kGemmBN - 1) / kGemmBN; }
__host__ __device__ inline int64_t gemm_tiles_m(int64_t M) { return (M + kGemmBM - 1) / kGemmBM; }

}  // namespace rg
