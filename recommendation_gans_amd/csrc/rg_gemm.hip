// fp32 GEMM on gfx950 MFMA (see rg_gemm.h).
//
// Block tile 128 x 128, K step 32, 256 threads = 4 waves in a 2 x 2 grid of 64 x 64
// wave tiles, each 2 x 2 v_mfma_f32_32x32x2_f32 accumulators (64 AGPR/VGPR).
// Operands are staged through LDS; the next step's global loads are in flight (in
// registers) while the current step's 64 MFMAs per wave issue.  One LDS stage and two
// barriers per K step (33.8 KB, <= 168 registers: 3 workgroups per CU) for every
// epilogue but the argmax, which keeps two stages (one barrier per step) for its LDS
// tile: at 2 workgroups per CU the lock-stepped workgroups of a CU left the matrix
// cores idle through each other's epilogues (cGAN 144k -> 166k slates/s).  K-major operands sit in LDS as [row][k] (stride 36 floats, 4 * odd
// mod 64: the ds_read_b128 lane groups of a 32-row column read are conflict-free);
// M/N-major operands as [k][row] (stride 132), read with ds_read_b32 across
// consecutive rows (conflict-free).
//
// K order inside a step: lane group h of the 32x32x2 instruction carries k = 16h + t
// at MFMA t (t = 0..15), so a K-major lane reads its 16 k values as 4 float4.  The
// result is an f32 fma chain over k in that order (exact f32 products and sums,
// one rounding each); split-K partials are summed in split order by the caller's
// reduction, so every result is deterministic.
#include "rg_gemm.h"

namespace rg {

namespace {

constexpr int BM = kGemmBM, BN = kGemmBN, BK = kGemmBK;
constexpr int LDK = BK + 4;      // [row][k] stride
constexpr int LDR = BM + 4;      // [k][row] stride (BM == BN)
constexpr int kThreads = 256;

typedef float v16f __attribute__((ext_vector_type(16)));

template <bool KM>
struct Stage {
    static constexpr int kFloats = KM ? BM * LDK : BK * LDR;
};

// global -> registers: 4 float4 per thread for a 128 x 32 operand tile
template <bool KM>
__device__ __forceinline__ void gload(float4 (&r)[4], const float *__restrict__ X, int64_t ld, int64_t r0,
                                      int64_t R, int64_t k0, int64_t k_end, float clampv, int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int idx = tid + kThreads * i;
        int64_t row, k;
        if constexpr (KM) {
            row = r0 + (idx >> 3);
            k = k0 + (idx & 7) * 4;
        } else {
            k = k0 + (idx >> 5);
            row = r0 + (idx & 31) * 4;
        }
        float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (row < R && k < k_end)
            v = KM ? *reinterpret_cast<const float4 *>(X + row * ld + k)
                   : *reinterpret_cast<const float4 *>(X + k * ld + row);
        if (clampv > 0.0f) {
            v.x = fminf(fmaxf(v.x, -clampv), clampv);
            v.y = fminf(fmaxf(v.y, -clampv), clampv);
            v.z = fminf(fmaxf(v.z, -clampv), clampv);
            v.w = fminf(fmaxf(v.w, -clampv), clampv);
        }
        r[i] = v;
    }
}

template <bool KM>
__device__ __forceinline__ void sstore(float *s, const float4 (&r)[4], int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int idx = tid + kThreads * i;
        float *dst = KM ? s + (idx >> 3) * LDK + (idx & 7) * 4 : s + (idx >> 5) * LDR + (idx & 31) * 4;
        *reinterpret_cast<float4 *>(dst) = r[i];
    }
}

// a lane's 16 operand values of one 32-row tile for this K step
template <bool KM>
__device__ __forceinline__ void frag(float (&f)[16], const float *s, int row, int h) {
    if constexpr (KM) {
        const float4 *p = reinterpret_cast<const float4 *>(s + row * LDK + 16 * h);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 v = p[q];
            f[4 * q] = v.x; f[4 * q + 1] = v.y; f[4 * q + 2] = v.z; f[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int t = 0; t < 16; ++t) f[t] = s[(16 * h + t) * LDR + row];
    }
}

struct TileMap {
    int64_t tm, tn, t_small, t_big, tg, nbb, gsize, groups;
    bool m_small;
    __host__ __device__ explicit TileMap(const GemmDesc &d) {
        tm = gemm_tiles_m(d.M);
        tn = gemm_tiles_n(d.N);
        m_small = tm <= tn;
        t_small = m_small ? tm : tn;
        t_big = m_small ? tn : tm;
        tg = t_small >= 16 ? 1 : 16 / t_small;
        if (tg > t_big) tg = t_big;
        nbb = (t_big + tg - 1) / tg;
        gsize = tg * t_small;
        groups = d.splits * nbb;
    }
    __host__ __device__ int64_t blocks() const { return 8 * gsize * ((groups + 7) / 8); }
    __device__ bool decode(int64_t L, int64_t &mt, int64_t &nt, int64_t &z) const {
        const int64_t local = L >> 3, w = local % gsize, P = (local / gsize) * 8 + (L & 7);
        if (P >= groups) return false;
        z = P / nbb;
        const int64_t major = (P % nbb) * tg + w / t_small, minor = w % t_small;
        if (major >= t_big) return false;
        mt = m_small ? minor : major;
        nt = m_small ? major : minor;
        return true;
    }
};

__host__ __device__ inline bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

__device__ __forceinline__ bool better(float v, float i, float bv, float bi) {
    return v > bv || (v == bv && i < bi);
}

__device__ __forceinline__ void opt1(const rg_opt_t &o, float clampv, float &p, float g, float &m, float &v) {
    float q = p;
    if (clampv > 0.0f) q = fminf(fmaxf(q, -clampv), clampv);
    p = opt_update(o, q, g, m, v);
}

__device__ __forceinline__ void opt4(const rg_opt_t &o, float clampv, float4 &p, const float4 &g, float4 &m,
                                     float4 &v) {
    opt1(o, clampv, p.x, g.x, m.x, v.x);
    opt1(o, clampv, p.y, g.y, m.y, v.y);
    opt1(o, clampv, p.z, g.z, m.z, v.z);
    opt1(o, clampv, p.w, g.w, m.w, v.w);
}

// ONE: a single operand stage (two barriers per K step) for 3 workgroups per CU instead
// of 2 -- the LDS (33.8 KB) and register budget (<= 168 per lane) of three; the argmax
// epilogue needs the double-buffered footprint for its tile
template <bool AK, bool BKM, int EPI, bool ONE>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(ONE ? 3 : 1, 8))) void gemm_kernel(GemmDesc d) {
    constexpr int kSA = Stage<AK>::kFloats, kSB = Stage<BKM>::kFloats;
    constexpr int kStages = ONE ? 1 : 2;
    __shared__ __attribute__((aligned(16))) float smem[kStages * (kSA + kSB)];
    auto sA = [&](int b) { return smem + (kStages == 2 ? b : 0) * kSA; };
    auto sB = [&](int b) { return smem + kStages * kSA + (kStages == 2 ? b : 0) * kSB; };
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
    const int h = lane >> 5, l32 = lane & 31;
    // XCD-aware order (blocks L, L + 8, L + 16, ... share an XCD and its L2): tiles are
    // grouped as (split z, block of tg long-dimension tiles) x every short-dimension
    // tile; a group's blocks run consecutively on one XCD, so the group's A and B
    // panels (for this K chunk) come from HBM once and are reused from L2
    const TileMap tmap(d);
    int64_t mt, nt, zz;
    if (!tmap.decode(blockIdx.x, mt, nt, zz)) return;
    const int64_t m0 = mt * BM, n0 = nt * BN;
    const int64_t kc = ((d.K + d.splits - 1) / d.splits + BK - 1) / BK * BK;
    const int64_t k_begin = zz * kc, k_end = min(d.K, k_begin + kc);
    const int nk = k_end > k_begin ? (int)((k_end - k_begin + BK - 1) / BK) : 0;

    v16f acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    float4 ra[4], rb[4];
    if (nk > 0) {
        gload<AK>(ra, d.A, d.lda, m0, d.M, k_begin, k_end, 0.0f, tid);
        gload<BKM>(rb, d.B, d.ldb, n0, d.N, k_begin, k_end, d.clamp_b, tid);
        sstore<AK>(sA(0), ra, tid);
        sstore<BKM>(sB(0), rb, tid);
    }
    __syncthreads();
    for (int it = 0; it < nk; ++it) {
        const int buf = it & 1;
        if (it + 1 < nk) {
            const int64_t k0 = k_begin + (int64_t)(it + 1) * BK;
            gload<AK>(ra, d.A, d.lda, m0, d.M, k0, k_end, 0.0f, tid);
            gload<BKM>(rb, d.B, d.ldb, n0, d.N, k0, k_end, d.clamp_b, tid);
        }
        float a[2][16], b[2][16];
#pragma unroll
        for (int i = 0; i < 2; ++i) frag<AK>(a[i], sA(buf), wm * 64 + i * 32 + l32, h);
#pragma unroll
        for (int j = 0; j < 2; ++j) frag<BKM>(b[j], sB(buf), wn * 64 + j * 32 + l32, h);
#pragma unroll
        for (int t = 0; t < 16; ++t)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][t], b[j][t], acc[i][j], 0, 0, 0);
        if (it + 1 < nk) {
            if constexpr (kStages == 1) __syncthreads();   // every wave is done reading the stage
            sstore<AK>(sA(buf ^ 1), ra, tid);
            sstore<BKM>(sB(buf ^ 1), rb, tid);
        }
        __syncthreads();
    }

    // ---- epilogues.  acc[i][j][r]: row m0 + wm*64 + i*32 + (r&3) + 8*(r>>2) + 4h,
    //      column n0 + wn*64 + j*32 + l32.
    auto row_of = [&](int i, int r) -> int64_t { return m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h; };
    auto col_of = [&](int j) -> int64_t { return n0 + wn * 64 + j * 32 + l32; };

    if constexpr (EPI == kEpiPartial) {
        float *C = d.C + zz * d.M * d.N;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int64_t n = col_of(j);
                if (n >= d.N) continue;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t m = row_of(i, r);
                    if (m < d.M) C[m * d.N + n] = acc[i][j][r];
                }
            }
    } else if constexpr (EPI == kEpiStore) {
        // per 16-row fragment: every operand load of the fragment is issued before any
        // store (C may alias T / Mult as far as the compiler knows: interleaving would
        // serialise one memory round trip per element)
        float cs[2] = {0.0f, 0.0f};
        const bool two = d.post == kPostTanhGrad || d.post == kPostLreluGrad;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int64_t n = col_of(j);
                if (n >= d.N) continue;
                const float bn = d.bias ? d.bias[n] : 0.0f;
                float t[16], q[16];
                if (two) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int64_t m = row_of(i, r);
                        t[r] = m < d.M ? d.T[m * d.ldt + n] : 0.0f;
                        q[r] = (m < d.M && d.Mult) ? d.Mult[m * d.ldt + n] : 1.0f;
                    }
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t m = row_of(i, r);
                    float v = acc[i][j][r] + bn;
                    if (d.post == kPostTanh) {
                        v = tanhf(v);
                    } else if (d.post == kPostTanhGrad) {
                        v = v * (1.0f - t[r] * t[r]);
                        if (m < d.M) cs[j] += v;
                    } else if (d.post == kPostLreluGrad) {
                        v = v * (t[r] > 0.0f ? 1.0f : 0.2f);
                        if (d.Mult) v = v * q[r];
                    }
                    if (m < d.M) d.C[m * d.ldc + n] = v;
                }
            }
        if (d.post == kPostTanhGrad && d.colsum) {
            // column sums of this row tile: lanes h = 0/1 hold alternating row quads,
            // waves wm = 0/1 the two 64-row halves; combined in a fixed order
            __shared__ float red[2][2][32];
#pragma unroll
            for (int j = 0; j < 2; ++j) cs[j] += __shfl_xor(cs[j], 32);
            if (wm == 1 && h == 0) {
                red[wn][0][l32] = cs[0];
                red[wn][1][l32] = cs[1];
            }
            __syncthreads();
            if (wm == 0 && h == 0) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int64_t n = col_of(j);
                    if (n < d.N) d.colsum[mt * d.N + n] = cs[j] + red[wn][j][l32];
                }
            }
        }
    } else if constexpr (EPI == kEpiOpt) {
        // sparse extra gradient rows of this column tile (hits sorted by column)
        const int lo = d.n_hits > 0 ? d.hit_tile_off[nt] : 0, hi = d.n_hits > 0 ? d.hit_tile_off[nt + 1] : 0;
        for (int x = lo; x < hi; ++x) {
            const int64_t c = d.hit_col[x];
            const float *src = d.hit_src + (int64_t)d.hit_row[x] * d.hit_ld;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (col_of(j) != c) continue;
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int64_t m = row_of(i, r);
                        if (m < d.M) acc[i][j][r] += src[m];
                    }
            }
        }
        // the gradient tile goes through LDS (the operand stages are free after the K
        // loop's last barrier; with ONE, one 64-row half at a time) and is re-read as
        // float4 column groups, a wave covering two rows of 512 B, so P and its state
        // move in dwordx4 loads / stores along rows; kQ rows in flight per thread
        constexpr int kQ = 4;
        const int c4 = tid & 31, r0 = tid >> 5;
        const bool vec = n0 + 4 * c4 + 3 < d.N && (d.ldp & 3) == 0 && aligned16(d.P) && (!d.Ms || aligned16(d.Ms)) &&
                         (!d.Vs || aligned16(d.Vs));
        constexpr int LDE = BN + 4;
        constexpr int kPass = kStages == 2 ? 1 : 2;   // row halves through LDS one at a time
        constexpr int kRows = BM / kPass;
        static_assert(kStages * (kSA + kSB) >= kRows * LDE, "LDS reuse");
        float *tile = smem;
        const int64_t n = n0 + 4 * c4;
        auto update_rows = [&](float4 (&pv)[kQ], float4 (&mv)[kQ], float4 (&vv)[kQ], int q0) {
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                const int rl = r0 + 8 * (q0 + q);
                const int64_t m = m0 + rl, e = m * d.ldp + n;
                if (m >= d.M) continue;
                const float4 g = *reinterpret_cast<const float4 *>(tile + (rl % kRows) * LDE + 4 * c4);
                if (vec) {
                    opt4(d.opt, d.clamp_p, pv[q], g, mv[q], vv[q]);
                    *reinterpret_cast<float4 *>(d.P + e) = pv[q];
                    if (d.Ms) *reinterpret_cast<float4 *>(d.Ms + e) = mv[q];
                    if (d.Vs) *reinterpret_cast<float4 *>(d.Vs + e) = vv[q];
                } else {
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        if (n + c >= d.N) continue;
                        float p = d.P[e + c], mm = d.Ms ? d.Ms[e + c] : 0.0f, v1 = d.Vs ? d.Vs[e + c] : 0.0f;
                        const float gc = c == 0 ? g.x : c == 1 ? g.y : c == 2 ? g.z : g.w;
                        opt1(d.opt, d.clamp_p, p, gc, mm, v1);
                        d.P[e + c] = p;
                        if (d.Ms) d.Ms[e + c] = mm;
                        if (d.Vs) d.Vs[e + c] = v1;
                    }
                }
            }
        };
#pragma unroll
        for (int pass = 0; pass < kPass; ++pass) {
            if (kPass == 1 || wm == pass) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            tile[((wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) % kRows) * LDE + wn * 64 +
                                 j * 32 + l32] = acc[i][j][r];
            }
            __syncthreads();
            const int qa = pass * (kRows / 8), qb = qa + kRows / 8;
            for (int q0 = qa; q0 < qb; q0 += kQ) {
                float4 pv[kQ], mv[kQ], vv[kQ];
#pragma unroll
                for (int q = 0; q < kQ; ++q) {
                    const int64_t m = m0 + r0 + 8 * (q0 + q), e = m * d.ldp + n;
                    pv[q] = mv[q] = vv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (m < d.M && vec) {
                        pv[q] = *reinterpret_cast<const float4 *>(d.P + e);
                        if (d.Ms) mv[q] = *reinterpret_cast<const float4 *>(d.Ms + e);
                        if (d.Vs) vv[q] = *reinterpret_cast<const float4 *>(d.Vs + e);
                    }
                }
                update_rows(pv, mv, vv, q0);
            }
            if (pass + 1 < kPass) __syncthreads();
        }
    } else if constexpr (EPI == kEpiArgmax) {
        // tanh(acc + bias) of the 128 x 128 tile into LDS (the operand buffers are free
        // now), then two threads per row scan 64 columns each: the first maximum per row
        // and head segment (the tile spans heads h0 and h0 + 1)
        constexpr int LDT = BN + 1;
        static_assert(2 * kSA + 2 * kSB >= BM * LDT || EPI != kEpiArgmax, "LDS reuse");
        float *tile = smem;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int64_t n = col_of(j);
                const float bn = (n < d.N && d.bias) ? d.bias[n] : 0.0f;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int rl = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    tile[rl * LDT + wn * 64 + j * 32 + l32] = tanhf(acc[i][j][r] + bn);
                }
            }
        __syncthreads();
        const int rl = tid >> 1, half = tid & 1;
        const int64_t h0 = n0 / d.seg;
        float bv[2] = {-INFINITY, -INFINITY}, bi[2] = {INFINITY, INFINITY};
        for (int c = half * 64; c < half * 64 + 64; ++c) {
            const int64_t n = n0 + c;
            if (n >= d.N) break;
            const int sg = (int)(n / d.seg - h0);
            const float v = tile[rl * LDT + c], ix = (float)(n - (h0 + sg) * d.seg);
            if (sg == 0) {
                if (better(v, ix, bv[0], bi[0])) { bv[0] = v; bi[0] = ix; }
            } else {
                if (better(v, ix, bv[1], bi[1])) { bv[1] = v; bi[1] = ix; }
            }
        }
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) {
            const float ov = __shfl_xor(bv[sg], 1), oi = __shfl_xor(bi[sg], 1);
            if (better(ov, oi, bv[sg], bi[sg])) { bv[sg] = ov; bi[sg] = oi; }
        }
        const int64_t m = m0 + rl;
        if (half == 0 && m < d.M) {
            const int64_t ntile = gemm_tiles_n(d.N);
            d.amax[(m * ntile + nt) * 2 + 0] = make_float2(bv[0], bi[0]);
            d.amax[(m * ntile + nt) * 2 + 1] = make_float2(bv[1], bi[1]);
        }
    }
}

template <bool AK, bool BKM>
void launch_epi(hipStream_t stream, const GemmDesc &d, dim3 grid) {
    switch (d.epi) {
        case kEpiStore: hipLaunchKernelGGL((gemm_kernel<AK, BKM, kEpiStore, true>), grid, dim3(kThreads), 0, stream, d); break;
        case kEpiPartial: hipLaunchKernelGGL((gemm_kernel<AK, BKM, kEpiPartial, true>), grid, dim3(kThreads), 0, stream, d); break;
        case kEpiOpt: hipLaunchKernelGGL((gemm_kernel<AK, BKM, kEpiOpt, true>), grid, dim3(kThreads), 0, stream, d); break;
        default: hipLaunchKernelGGL((gemm_kernel<AK, BKM, kEpiArgmax, false>), grid, dim3(kThreads), 0, stream, d); break;
    }
}


__global__ __launch_bounds__(256) void reduce_partials_kernel(const float *__restrict__ part, int splits, int64_t M,
                                                              int64_t N, float *__restrict__ C, int64_t ldc,
                                                              const float *__restrict__ bias) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= M * N) return;
    const int64_t m = e / N, n = e % N;
    float v = 0.0f;
    for (int z = 0; z < splits; ++z) v += part[(int64_t)z * M * N + e];
    C[m * ldc + n] = v + (bias ? bias[n] : 0.0f);
}

}  // namespace

int reduce_partials(hipStream_t stream, const float *part, int splits, int64_t M, int64_t N, float *C, int64_t ldc,
                    const float *bias) {
    const int64_t total = M * N;
    hipLaunchKernelGGL(reduce_partials_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, part,
                       splits, M, N, C, ldc, bias);
    return check_launch("reduce_partials_kernel");
}

int gemm(hipStream_t stream, const GemmDesc &d) {
    if (d.M <= 0 || d.N <= 0 || d.K < 0) return fail_arg("gemm: bad shape");
    if (((d.a_kmajor || d.b_kmajor) && d.K % 4) || d.lda % 4 || d.ldb % 4 || !aligned16(d.A) || !aligned16(d.B))
        return fail_arg("gemm: lda, ldb (and K with a K-major operand) must be multiples of 4, A and B 16-B aligned");
    // an M/N-major operand is read in float4s along its contiguous dimension: rows up to
    // round4(M) must be readable (values there only reach output rows >= M, discarded)
    const int64_t m4 = (d.M + 3) / 4 * 4, n4 = (d.N + 3) / 4 * 4;
    if (d.a_kmajor ? d.lda < d.K : d.lda < m4) return fail_arg("gemm: lda too small");
    if (d.b_kmajor ? d.ldb < d.K : d.ldb < n4) return fail_arg("gemm: ldb too small");
    if (d.splits < 1 || (d.splits > 1 && d.epi != kEpiPartial)) return fail_arg("gemm: split-K needs kEpiPartial");
    if (d.epi == kEpiArgmax && (d.seg < kGemmBN || !d.amax)) return fail_arg("gemm: argmax needs seg >= 128");
    if (d.epi == kEpiOpt && !d.P) return fail_arg("gemm: optimizer epilogue needs P");
    if (d.n_hits > 0 && (!d.hit_tile_off || !d.hit_col || !d.hit_row || !d.hit_src))
        return fail_arg("gemm: hits need hit_col, hit_row, hit_src and per-tile offsets");
    if ((d.epi == kEpiStore || d.epi == kEpiPartial) && !d.C) return fail_arg("gemm: no C");
    const dim3 grid((unsigned)TileMap(d).blocks());
    if (d.a_kmajor) {
        if (d.b_kmajor) launch_epi<true, true>(stream, d, grid);
        else launch_epi<true, false>(stream, d, grid);
    } else {
        if (d.b_kmajor) launch_epi<false, true>(stream, d, grid);
        else launch_epi<false, false>(stream, d, grid);
    }
    return check_launch("gemm_kernel");
}

}  // namespace rg

// ---------------------------------------------------------------- C-ABI test entry
extern "C" int rg_gemm_f32(void *stream, const float *A, int64_t lda, int32_t a_kmajor, const float *B,
                           int64_t ldb, int32_t b_kmajor, int64_t M, int64_t N, int64_t K, float *C, int64_t ldc,
                           const float *bias, int32_t post, int32_t splits, float *work) {
    rg::GemmDesc d;
    d.A = A; d.lda = lda; d.a_kmajor = a_kmajor != 0;
    d.B = B; d.ldb = ldb; d.b_kmajor = b_kmajor != 0;
    d.M = M; d.N = N; d.K = K;
    if (splits <= 1) {
        d.epi = rg::kEpiStore;
        d.C = C; d.ldc = ldc; d.bias = bias; d.post = post;
        return rg::gemm((hipStream_t)stream, d);
    }
    if (!work || post != rg::kPostNone) return rg::fail_arg("rg_gemm_f32: split-K needs work and post 0");
    d.epi = rg::kEpiPartial;
    d.splits = splits;
    d.C = work;
    int rc = rg::gemm((hipStream_t)stream, d);
    if (rc) return rc;
    return rg::reduce_partials((hipStream_t)stream, work, splits, M, N, C, ldc, bias);
}

// test / measurement entry: C-shaped gradient GEMM fused with an RMSprop (alpha, eps)
// update of P [M][N] (row stride ldp) and its square average V
extern "C" int rg_gemm_f32_rms(void *stream, const float *A, int64_t lda, int32_t a_kmajor, const float *B,
                               int64_t ldb, int32_t b_kmajor, int64_t M, int64_t N, int64_t K, float *P, float *V,
                               int64_t ldp, float lr, float alpha, float eps) {
    rg::GemmDesc d;
    d.A = A; d.lda = lda; d.a_kmajor = a_kmajor != 0;
    d.B = B; d.ldb = ldb; d.b_kmajor = b_kmajor != 0;
    d.M = M; d.N = N; d.K = K;
    d.epi = rg::kEpiOpt;
    d.P = P; d.Vs = V; d.ldp = ldp;
    d.opt.kind = RG_OPT_RMSPROP;
    d.opt.lr = lr; d.opt.alpha = alpha; d.opt.eps = eps;
    d.opt.one_minus_alpha = (float)(1.0 - (double)alpha);
    return rg::gemm((hipStream_t)stream, d);
}
