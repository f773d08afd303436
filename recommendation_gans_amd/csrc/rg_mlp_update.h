// The NCF / NeuMF MLP update (reduce the pair kernel's per-workgroup weight-gradient partials,
// then the optimizer in place), one 64-parameter block at a time, shared by the stand-alone
// ncf_update_kernel (16 waves per workgroup) and the fused tail launch of the NCF step
// (mf_back_kernel's extra workgroups, 4 waves): either way the partials are summed as 16 fixed
// slices (four chains each), combined in slice order -- the same bits for any wave count.
#pragma once
#include "rg_common.h"

namespace rg {

constexpr int kMlpSlices = 16;

struct MlpUpdArgs {
    float *mlp, *m, *v;       // flat parameters and optimizer state (m / v may be null)
    const float *wpart;       // [nparts][P]
    int nparts, P;
    rg_opt_t opt;
    int mode;                 // 0: reduce + update; 1: reduce into grad[0, P) (data parallel)
    float *grad;
};

// one 64-parameter block: NW waves (NW divides kMlpSlices), `red` = LDS [kMlpSlices][64]
template <int NW>
__device__ __forceinline__ void mlp_update_block(const MlpUpdArgs &u, int64_t blk, float (*red)[64]) {
    static_assert(kMlpSlices % NW == 0, "slices per wave");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t e = blk * 64 + lane;
    const int q = (u.nparts + kMlpSlices - 1) / kMlpSlices;
#pragma unroll
    for (int r = 0; r < kMlpSlices / NW; ++r) {
        const int slice = wave + r * NW, k0 = slice * q, k1 = min(u.nparts, k0 + q);
        float g = 0.0f;
        if (e < u.P) {
            float c[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            int k = k0;
            // batches of 16 partials: every load of a batch in flight before the (unchanged)
            // four-chain sums consume them
            for (; k + 16 <= k1; k += 16) {
                float v[16];
#pragma unroll
                for (int t = 0; t < 16; ++t) v[t] = u.wpart[(int64_t)(k + t) * u.P + e];
#pragma unroll
                for (int t = 0; t < 16; ++t) c[t & 3] += v[t];
            }
            for (; k + 4 <= k1; k += 4) {
#pragma unroll
                for (int j = 0; j < 4; ++j) c[j] += u.wpart[(int64_t)(k + j) * u.P + e];
            }
            for (; k < k1; ++k) c[0] += u.wpart[(int64_t)k * u.P + e];
            g = (c[0] + c[1]) + (c[2] + c[3]);
        }
        red[slice][lane] = g;
    }
    __syncthreads();
    if (wave != 0 || e >= u.P) return;
    float g = red[0][lane];
#pragma unroll
    for (int w = 1; w < kMlpSlices; ++w) g += red[w][lane];
    if (u.mode == 1) {
        u.grad[e] = g;
        return;
    }
    float mm = u.m ? u.m[e] : 0.0f, vv = u.v ? u.v[e] : 0.0f;
    const float p = opt_update(u.opt, u.mlp[e], g, mm, vv);
    u.mlp[e] = p;
    if (u.m) u.m[e] = mm;
    if (u.v) u.v[e] = vv;
}

}  // namespace rg
