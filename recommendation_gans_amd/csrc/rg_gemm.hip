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

#include <atomic>

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

#if RG_AB   // measured slower than gemm_kernel's optimizer epilogue: A/B build only
// ---------------------------------------------------------------- wave-specialised optimizer GEMM
// The optimizer epilogue (kEpiOpt) with both operands M/N-major, as a persistent kernel of one
// 512-thread workgroup per CU whose waves split the two phases of a tile: waves 0-3 run the K
// loop of tile i (the 2 x 2 grid of 64 x 64 wave tiles above, operands staged by direct-to-LDS
// loads two K steps ahead, synchronised by LDS counters -- no workgroup barrier), while waves 4-7
// stream the optimizer update of tile i - 1 (P and its state, the HBM-bound half).  The matrix
// cores and the HBM stream overlap inside one CU instead of across the three lock-prone
// workgroups of gemm_kernel<.., kEpiOpt, true>.
//
// Same K order per lane (k = 16h + t at MFMA t, K steps in order), same hits order, same
// update arithmetic: results are bit-identical to gemm_kernel's optimizer epilogue.
constexpr int kWsThreads = 768;   // waves 0-3 matrix, 4-7 update, 8-11 loaders
constexpr int kWsRows = 16;      // rows per update thread (128 rows over 8 row groups)
constexpr int kWsQ = 4;          // rows of P / state in flight per update thread

// LDS hand-over counters without fences: a workgroup-scope fence (even one naming only the local
// address space) waits vmcnt(0), because a direct-to-LDS load in flight is a pending LDS write,
// and would drain the operand pipeline at every signal.  Instead a wave's LDS operations execute
// in order, so a count added after its LDS writes / reads is seen after them; the asm statements
// keep the compiler from moving memory operations across the signal or the wait, and the
// operand stages' own arrival is counted by hand (ws_vmcnt) before the `full` signal.
__device__ __forceinline__ int lds_acquire(const int *p) {
    const int v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
    return v;
}

// wait for an LDS counter; bounded (~0.5 s) so that a broken hand-over ends the kernel with
// wrong bits the tests catch instead of a wave that never finishes
__device__ __forceinline__ void lds_wait(const int *p, int target) {
    for (int n = 0; lds_acquire(p) < target && n < (1 << 23); ++n) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ void lds_release_add(int *p) {
    asm volatile("" ::: "memory");
    __hip_atomic_fetch_add(p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
}

// the loader waves' counter operations, hidden from hipcc's wait insertion (see above)
__device__ __forceinline__ uint32_t lds_addr(const int *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) int *)p;
}

__device__ __forceinline__ void asm_lds_add(int *p) {
    asm volatile("ds_add_u32 %0, %1" ::"v"(lds_addr(p)), "v"(1) : "memory");
}

__device__ __forceinline__ void asm_lds_wait(const int *p, int target) {
    for (int n = 0; n < (1 << 23); ++n) {
        int v;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
        if (__builtin_amdgcn_readfirstlane(v) >= target) break;
        __builtin_amdgcn_s_sleep(1);
    }
}

// Operand stages shared by the matrix waves: a K step's A panel [BK][128] and B panel
// [BK][128] (M/N-major rows, unpadded: 2 k rows per 1-KB direct-to-LDS load), 32 KB, three of
// them so that two K steps are in flight while one is read.  Each matrix wave issues 8 of a
// stage's 32 global_load_lds_dwordx4 (no registers hold the operands in flight); a stage is
// full when all four waves have counted their own loads landed (`full`), and free for the K
// step three later when all four matrix waves have read their fragments from it (`empty`).
// The result tile goes to the update waves in two 64-row halves through one half-tile buffer
// (`ready` / `taken`), which keeps the workgroup at 130 KB of LDS.
constexpr int kWsStages = 3;
constexpr int kWsStage = 2 * BK * BM;           // floats per stage (A and B panels)
constexpr int kWsLoads = 8;                     // direct-to-LDS loads per matrix wave per stage

struct WsTile {
    int64_t m0, n0;
};

// the global rows of a panel float4 (rows past the end clamped to the last whole float4 of the
// row: they only reach discarded outputs)
__device__ __forceinline__ const float *ws_src(const float *X, int64_t ld, int64_t R, int64_t row0, int64_t k,
                                              int lane) {
    const int64_t r4 = (R + 3) / 4 * 4;
    return X + k * ld + min(row0 + (lane & 31) * 4, r4 - 4);
}

// wait until at most n of this wave's direct-to-LDS loads are outstanding (vmcnt; the loader
// waves issue no other vector memory operation)
__device__ __forceinline__ void ws_vmcnt(int n) {
    static_assert(kWsStages <= 4 && kWsLoads == 8, "the counted waits below");
    if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool CLAMP, bool HAS_M>
__global__ __launch_bounds__(kWsThreads) void gemm_opt_ws_kernel(GemmDesc d) {
    constexpr int LDE = BN + 4;
    // ONE shared array (a second __shared__ object beside the direct-to-LDS stages makes hipcc
    // wait vmcnt(0) before LDS reads): stages | half tile | counters
    __shared__ __attribute__((aligned(16))) float lds[kWsStages * kWsStage + 64 * LDE + 16];
    float *const stages = lds, *const half = lds + kWsStages * kWsStage;
    int *const ctr = reinterpret_cast<int *>(half + 64 * LDE);
    int *const ready = ctr, *const taken = ctr + 1, *const full = ctr + 2, *const empty = ctr + 2 + kWsStages;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 2 + 2 * kWsStages) ctr[tid] = 0;
    __syncthreads();                                  // the only workgroup barrier
    // 32-bit tile arithmetic in scalars (tile counts are far below 2^31)
    const int tm = (int)gemm_tiles_m(d.M), tn = (int)gemm_tiles_n(d.N);
    const bool m_small = tm <= tn;
    const int t_small = m_small ? tm : tn, t_big = m_small ? tn : tm;
    const int x = (int)(blockIdx.x & 7);
    const int per_x = (int)((gridDim.x - x + 7) / 8), l = (int)(blockIdx.x >> 3);
    const int tiles_x = t_small * ((t_big - x + 7) / 8);                     // this XCD's tiles
    const int ntiles = l < tiles_x ? (tiles_x - l + per_x - 1) / per_x : 0;  // this workgroup's
    // the n-th tile of this workgroup: panel x + 8 * (j / t_small) of its XCD, j = l + n * per_x
    auto tile_of = [=](int n) -> WsTile {
        const int j = l + n * per_x, panel = (j / t_small) * 8 + x, minor = j % t_small;
        return m_small ? WsTile{(int64_t)minor * BM, (int64_t)panel * BN} : WsTile{(int64_t)panel * BM, (int64_t)minor * BN};
    };

    const int nk = (int)(d.K / BK);
    const int T = ntiles * nk;                       // K steps of this workgroup, one stream G
    if (wave >= 8) {
        // ---- loader waves: the operand stages, two K steps ahead of the matrix waves.  Waves
        // 8-9 load the A panel's k-row pairs, 10-11 the B panel's (8 each per stage).  They issue
        // no other vector memory operation, so the counted vmcnt below is exact; their counter
        // operations are asm (hipcc would otherwise wait vmcnt(0) before every LDS access that
        // follows a direct-to-LDS load, draining the pipeline)
        const int w = wave - 8;
        const bool opa = w < 2;
        const float *X = opa ? d.A : d.B;
        const int64_t ld = opa ? d.lda : d.ldb, R = opa ? d.M : d.N;
        const int kp0 = (w & 1) * kWsLoads;
        float *const dst0 = stages + (opa ? 0 : BK * BM) + kp0 * 2 * BM;
        auto issue = [=](int G) {
            const WsTile tl = tile_of(G / nk);
            const int64_t k0 = (int64_t)(G % nk) * BK;
            const float *src = ws_src(X, ld, R, opa ? tl.m0 : tl.n0, k0 + 2 * kp0 + (lane >> 5), lane);
            float *dst = dst0 + (G % kWsStages) * kWsStage;
#pragma unroll
            for (int i = 0; i < kWsLoads; ++i)
                __builtin_amdgcn_global_load_lds(src + 2 * i * ld, dst + i * 2 * BM, 16, 0, 0);
        };
        for (int G = 0; G < T && G < kWsStages; ++G) issue(G);
        for (int G = 0; G < T; ++G) {
            const int st = G % kWsStages, use = G / kWsStages;
            ws_vmcnt((min(T - 1, G + kWsStages - 1) - G) * kWsLoads);   // stage G landed
            if (lane == 0) asm_lds_add(full + st);
            if (G + kWsStages < T) {
                asm_lds_wait(empty + st, 4 * (use + 1));               // every matrix wave read it
                issue(G + kWsStages);
            }
        }
        ws_vmcnt(0);
        return;
    }
    if (wave < 4) {
        // ---- matrix waves: the 2 x 2 grid of 64 x 64 wave tiles, fragments from the stages
        const int wm = wave >> 1, wn = wave & 1, h = lane >> 5, l32 = lane & 31;
        v16f acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][jj][r] = 0.0f;
        for (int G = 0; G < T; ++G) {
            const int st = G % kWsStages, use = G / kWsStages;
            lds_wait(full + st, 4 * (use + 1));
            const float *sa = stages + st * kWsStage, *sb = sa + BK * BM;
            float a[2][16], b[2][16];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    a[i][t] = sa[(16 * h + t) * BM + wm * 64 + i * 32 + l32];
                    b[i][t] = sb[(16 * h + t) * BN + wn * 64 + i * 32 + l32];
                }
            if (lane == 0) lds_release_add(empty + st);      // after the reads (in order)
            if constexpr (CLAMP) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int t = 0; t < 16; ++t) b[i][t] = fminf(fmaxf(b[i][t], -d.clamp_b), d.clamp_b);
            }
#pragma unroll
            for (int t = 0; t < 16; ++t)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj)
                        acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][t], b[jj][t], acc[i][jj], 0, 0, 0);
            if (G % nk == nk - 1) {
                // hand the tile over: this wave's 64-row half u = 2n + wm, once halves < u are taken
                const int u = 2 * (G / nk) + wm;
                lds_wait(taken, 4 * u);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            half[(i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * LDE + wn * 64 + jj * 32 + l32] =
                                acc[i][jj][r];
                            acc[i][jj][r] = 0.0f;
                        }
                if (lane == 0) lds_release_add(ready);
            }
        }
        return;
    }
    // ---- update waves: hits, then the optimizer over P and its state, rows as float4 groups
    constexpr int Q = HAS_M ? 2 : kWsQ;             // rows in flight per thread (registers: Adam's m)
    const int et = tid - 256, c4 = et & 31, r0 = et >> 5;
    for (int n = 0; n < ntiles; ++n) {
        const WsTile tl = tile_of(n);
        const int64_t m0 = tl.m0, n0 = tl.n0, nn = n0 + 4 * c4;
        float4 g[kWsRows];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            lds_wait(ready, 2 * (2 * n + hf + 1));   // the half's two matrix waves
#pragma unroll
            for (int q = 0; q < kWsRows / 2; ++q)
                g[hf * (kWsRows / 2) + q] = *reinterpret_cast<const float4 *>(half + (r0 + 8 * q) * LDE + 4 * c4);
            if (lane == 0) lds_release_add(taken);  // one count per wave, after its reads (in order)
        }
        // sparse extra gradient rows of this column tile (hits sorted by column), in hit order
        const int64_t ntile = n0 / BN;
        const int lo = d.n_hits > 0 ? d.hit_tile_off[ntile] : 0, hi = d.n_hits > 0 ? d.hit_tile_off[ntile + 1] : 0;
        for (int hx = lo; hx < hi; ++hx) {
            const int64_t c = d.hit_col[hx] - nn;
            if (c < 0 || c > 3) continue;
            const float *src = d.hit_src + (int64_t)d.hit_row[hx] * d.hit_ld;
#pragma unroll
            for (int q = 0; q < kWsRows; ++q) {
                const int64_t m = m0 + r0 + 8 * q;
                if (m >= d.M) continue;
                const float sv = src[m];
                if (c == 0) g[q].x += sv; else if (c == 1) g[q].y += sv; else if (c == 2) g[q].z += sv; else g[q].w += sv;
            }
        }
        const bool vec = nn + 3 < d.N && (d.ldp & 3) == 0 && aligned16(d.P) && (!d.Ms || aligned16(d.Ms)) &&
                         (!d.Vs || aligned16(d.Vs));
#pragma unroll
        for (int q0 = 0; q0 < kWsRows; q0 += Q) {
            float4 pv[Q], mv[HAS_M ? Q : 1], vv[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int64_t m = m0 + r0 + 8 * (q0 + q), e = m * d.ldp + nn;
                pv[q] = vv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (HAS_M) mv[HAS_M ? q : 0] = pv[q];
                if (m < d.M && vec) {
                    pv[q] = *reinterpret_cast<const float4 *>(d.P + e);
                    if (HAS_M) mv[HAS_M ? q : 0] = *reinterpret_cast<const float4 *>(d.Ms + e);
                    if (d.Vs) vv[q] = *reinterpret_cast<const float4 *>(d.Vs + e);
                }
            }
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int64_t m = m0 + r0 + 8 * (q0 + q), e = m * d.ldp + nn;
                if (m >= d.M) continue;
                const float4 gg = g[q0 + q];
                if (vec) {
                    float4 mq = HAS_M ? mv[HAS_M ? q : 0] : make_float4(0.f, 0.f, 0.f, 0.f);
                    opt4(d.opt, d.clamp_p, pv[q], gg, mq, vv[q]);
                    *reinterpret_cast<float4 *>(d.P + e) = pv[q];
                    if (HAS_M) *reinterpret_cast<float4 *>(d.Ms + e) = mq;
                    if (d.Vs) *reinterpret_cast<float4 *>(d.Vs + e) = vv[q];
                } else {
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        if (nn + c >= d.N) continue;
                        float p = d.P[e + c], mm = HAS_M ? d.Ms[e + c] : 0.0f, v1 = d.Vs ? d.Vs[e + c] : 0.0f;
                        const float gc = c == 0 ? gg.x : c == 1 ? gg.y : c == 2 ? gg.z : gg.w;
                        opt1(d.opt, d.clamp_p, p, gc, mm, v1);
                        d.P[e + c] = p;
                        if (HAS_M) d.Ms[e + c] = mm;
                        if (d.Vs) d.Vs[e + c] = v1;
                    }
                }
            }
        }
    }
}

}  // namespace

// the optimizer GEMM's form: 1 the wave-specialised kernel, 0 gemm_kernel's epilogue
// (RG_GEMM_WS at load, rg_gemm_ws_mode at run time)
std::atomic<int> g_gemm_ws{[] { const char *v = getenv("RG_GEMM_WS"); return v ? atoi(v) : 0; }()};

namespace {

bool gemm_ws_enabled() { return g_gemm_ws.load(std::memory_order_relaxed) != 0; }
#endif  // RG_AB

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
#if RG_AB
    // (K a whole number of K steps; byte offsets of both operands within 32 bits)
    if (d.epi == kEpiOpt && !d.a_kmajor && !d.b_kmajor && d.K % BK == 0 && d.K > 0 &&
        d.K * d.lda * 4 < INT32_MAX && d.K * d.ldb * 4 < INT32_MAX && gemm_ws_enabled()) {
        // persistent: one workgroup per CU, a multiple of 8 (each XCD label owns its panels)
        const int64_t wg = std::min<int64_t>(num_cus(), gemm_tiles_m(d.M) * gemm_tiles_n(d.N));
        const dim3 grid((unsigned)(8 * ((wg + 7) / 8)));
        const bool cl = d.clamp_b > 0.0f, hm = d.Ms != nullptr;
        if (cl && hm) hipLaunchKernelGGL((gemm_opt_ws_kernel<true, true>), grid, dim3(kWsThreads), 0, stream, d);
        else if (cl) hipLaunchKernelGGL((gemm_opt_ws_kernel<true, false>), grid, dim3(kWsThreads), 0, stream, d);
        else if (hm) hipLaunchKernelGGL((gemm_opt_ws_kernel<false, true>), grid, dim3(kWsThreads), 0, stream, d);
        else hipLaunchKernelGGL((gemm_opt_ws_kernel<false, false>), grid, dim3(kWsThreads), 0, stream, d);
        return check_launch("gemm_opt_ws_kernel");
    }
#endif
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

// the optimizer GEMM's form (test / measurement entry): mode 0 gemm_kernel's fused epilogue,
// 1 the wave-specialised persistent kernel (A/B build only: -1 elsewhere), < 0 leaves it;
// returns the form in force before
extern "C" int rg_gemm_ws_mode(int32_t mode) {
#if RG_AB
    const int prev = rg::g_gemm_ws.load();
    if (mode >= 0) rg::g_gemm_ws.store(mode != 0 ? 1 : 0);
    return prev;
#else
    if (mode > 0) {
        rg::set_error("rg_gemm_ws_mode: the wave-specialised optimizer GEMM is in the A/B build only (DESIGN 4.3)");
        return -1;
    }
    return 0;
#endif
}
