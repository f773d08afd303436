// NCF MLP training step on gfx950 (spotlight/dnn_models/mlp.py:5-46 trained by
// implicit.py:347-364; layers [2E, E, ..., 8] -> 1 as ncf_spotlight.py:53-56).
//
// One workgroup (4 waves) walks tiles of kRows = 32 examples (the E = 64 MLP's wave kernel:
// ncfw::kR = RG_NCF_WAVE_ROWS = 48 in the product build); a tile holds whole
// columns (a positive and its n negatives, pairs prepared by rg_mf_prepare), so
// pairwise losses are resolved inside the tile.  Everything of a tile lives in
// LDS: the MLP parameters (loaded once per workgroup), the activations of every
// layer, the per-unit backward multipliers and the workgroup's running weight
// gradient.  Each layer's three products run on the fp32 MFMA (16x16x4):
//     Z_k = A_k W_k^T,   dW_k += delta_k^T A_k,   dA_k = delta_k W_k.
// LeakyReLU(0.1) then Dropout(0.5) fold into one exact multiplier per unit,
// m in {0, 2, 0.2} (training) or {1, 0.1} (eval): A_{k+1} = Z_k * m and
// delta = dA * m reproduce torch's rounding (power-of-two scalings commute).
// Outputs: per-example input gradients dX (rows of 2E) for the embedding update
// (rg_ncf_apply pulls them through the per-row lists), planned per-tile partial
// rows for the positives' items, the workgroup's weight-gradient partial and
// deterministic loss partials.
//
// NeuMF (spotlight/dnn_models/neuMF.py:7-55) is the same tower plus a GMF branch:
// the output Linear sees cat(A_NH, U_mf[u] * I_mf[i]) (mf_dim M > 0).  The GMF rows
// are gathered beside A_0, the output layer adds M products, and the GMF backward
// (dU_mf = dz w_m I_mf, dI_mf = dz w_m U_mf) runs before the tower's backward and
// writes its own per-example rows (mf_contrib), overflow rows and planned partials.
#include <cstdlib>
#include <utility>

#include "rg_common.h"
#include "rg_mlp_update.h"

namespace rg {

constexpr int kRows = 32;              // examples per tile (two 16-row MFMA tiles)
constexpr int kNcfThreads = 256;
constexpr int kNcfCap = RG_MF_LIST_CAP;

typedef float v4f __attribute__((ext_vector_type(4)));

// layer sizes H_k = 2E >> k, k = 0..NH (H_NH = 8); NH hidden Linear layers + output 8 -> 1
template <int E>
struct NcfShape {
    static constexpr int NH = E == 8 ? 1 : E == 16 ? 2 : E == 32 ? 3 : 4;
    static constexpr int H(int k) { return (2 * E) >> k; }
    static constexpr int w_off(int k) {       // flat parameter offset of layer k (W then b)
        int o = 0;
        for (int j = 0; j < k; ++j) o += H(j + 1) * H(j) + H(j + 1);
        return o;
    }
    static constexpr int P = w_off(NH) + 8 + 1;                  // + output W (1x8), b (1)
    // LDS float offsets: padded weights, activations, multipliers, dW, misc
    static constexpr int sw_off(int k) {
        int o = 0;
        for (int j = 0; j < k; ++j) o += H(j + 1) * (H(j) + 1) + H(j + 1);
        return o;
    }
    static constexpr int SW = sw_off(NH) + 9;
    static constexpr int sa_off(int k) {
        int o = 0;
        for (int j = 0; j < k; ++j) o += kRows * (H(j) + 1);
        return o;
    }
    static constexpr int SA = sa_off(NH + 1);
    static constexpr int mask_off(int k) {    // first dropout unit of hidden layer k
        int u = 0;
        for (int j = 1; j <= k; ++j) u += H(j);
        return u;
    }
    static constexpr int mask_units() {
        int u = 0;
        for (int k = 1; k <= NH; ++k) u += H(k);
        return u;
    }
    static constexpr int LDS = SW + SA + SA + P + 13 * kRows + 8;   // W, A, M(=A layout), dW, misc
    // NeuMF extra floats: dW (M more), output GMF weights (M), GMF rows unless they fit
    // the dX region (M <= E: row stride 2E + 1 holds U_mf | I_mf)
    static constexpr int lds_neumf(int M) { return M == 0 ? LDS : LDS + 2 * M + (M <= E ? 0 : kRows * (2 * M + 1)); }
};

constexpr int kLdsMax = 160 * 1024 / 4;

struct NcfArgs {
    const float *user_w, *item_w;
    const float *mlp;                 // flat parameters (named_parameters order)
    int64_t num_users, num_items;
    const int2 *pairs;                // prepared, one record per column (rg_common.h pair_stride)
    int64_t n_pos, cols, global_cols, col_offset;
    int n_neg, loss, tc;              // tc: columns per tile
    int64_t tiles;
    float n_a, n_b;                   // loss denominators (as rg_mf_pairs)
    const int32_t *perm, *pos_slot;   // plan (optional)
    int32_t *row_count;
    int2 *row_list;
    long long *hot_grad;                  // int64 fixed point (rg_common.h fix_add)
    float *part_row;
    float *loss_partials;             // [tiles * 2]
    float *contrib;                   // [tiles * kRows * 2E]
    float *wpart;                     // [gridDim.x * P]
    float *scores;                    // [tiles * kRows] (forward-only phase)
    const float *dp_in;               // [tiles * kRows] (given-dp phase)
    const uint8_t *mask_pos, *mask_neg;
    uint64_t seed;
    int training;
    // NeuMF (mf_dim > 0)
    int mf_dim;
    const float *mf_user_w, *mf_item_w;
    float *mf_contrib;
    long long *mf_hot_grad;
    float *mf_part_row;
};

enum NcfPhase { kNcfFused = 0, kNcfScores = 1, kNcfGivenDp = 2, kNcfLossOnly = 3 };

// f(integral_constant<int, 0>), ..., f(integral_constant<int, N - 1>): the layer loops
// contain barriers and were not unrolled, which left every layer's shapes (and so the
// MFMA K loop) runtime values -- an LDS round trip between consecutive MFMA pairs
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// Diagnostic build only (RG_DIAG_STAMPS): s_memrealtime at the tile phase boundaries of
// the first two tiles of every workgroup (thread 0, after the phase's barrier), for
// scripts/ncf_stamps.py.  The product library has no stamp code.
#ifdef RG_DIAG_STAMPS
__device__ unsigned long long *g_ncf_stamps;
#define NS(k)                                                                                        \
    do {                                                                                             \
        if (g_ncf_stamps && threadIdx.x == 0 && tl_ < 2) {                                           \
            unsigned long long t_;                                                                   \
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
            g_ncf_stamps[((int64_t)blockIdx.x * 2 + tl_) * 8 + (k)] = t_;                            \
        }                                                                                            \
    } while (0)
#else
#define NS(k) \
    do {      \
    } while (0)
#endif

__device__ __forceinline__ uint32_t hash32(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return (uint32_t)x;
}

// murmur3 fmix32: the per-unit dropout bit from the row's key
__device__ __forceinline__ uint32_t mix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bU;
    h ^= h >> 13;
    h *= 0xc2b2ae35U;
    h ^= h >> 16;
    return h;
}

// C tile (16x16 at i0, j0) of A.B on LDS operands, K a compile-time multiple of 4.
// A(i, k) = A[i * ai + k * ak], B(k, j) = B[k * bk + j * bj]; rows >= imax / cols >= jmax read 0.
// Every operand of the tile is read first (one batch of LDS reads; rows outside the
// tile read row 0 and are zeroed after), then the K/4 MFMAs issue over four
// independent accumulators: no LDS round trip or MFMA dependency between
// consecutive MFMAs.
template <int K, int KB = K>
__device__ __forceinline__ v4f mma16(const float *A, int ai, int ak, const float *B, int bk, int bj, int i0, int j0,
                                     int imax, int jmax, int lane) {
    // KB: K values read per batch (a multiple of 16 dividing K); the accumulator sequence,
    // and so the result, does not depend on it
    constexpr int NK = K / 4, NB = (KB < K ? KB : K) / 4;
    static_assert(NK % NB == 0 && NB % 4 == 0 || NB == NK, "batch shape");
    const int li = lane & 15, lk = lane >> 4;
    const bool iv = i0 + li < imax, jv = j0 + li < jmax;
    const float *pa = A + (iv ? (i0 + li) : 0) * ai + lk * ak;
    const float *pb = B + lk * bk + (jv ? (j0 + li) : 0) * bj;
    v4f acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = v4f{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int s0 = 0; s0 < NK; s0 += NB) {
        float av[NB], bv[NB];
#pragma unroll
        for (int s = 0; s < NB; ++s) {
            av[s] = pa[4 * (s0 + s) * ak];
            bv[s] = pb[4 * (s0 + s) * bk];
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the read batch ahead of the MFMAs
#pragma unroll
        for (int s = 0; s < NB; ++s)
            acc[(s0 + s) & 3] =
                __builtin_amdgcn_mfma_f32_16x16x4f32(iv ? av[s] : 0.0f, jv ? bv[s] : 0.0f, acc[(s0 + s) & 3], 0, 0, 0);
    }
    return (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

template <int E>
constexpr int ncf_threads() { return E >= 64 ? 512 : kNcfThreads; }

template <int E, int PHASE>
__global__ __launch_bounds__(ncf_threads<E>()) void ncf_pairs_kernel(NcfArgs a) {
    constexpr int kNT = ncf_threads<E>(), kNW = kNT / 64;
    constexpr int kKB = kNT > kNcfThreads ? 32 : 1024;   // MFMA operand batch (K values): registers for 2 waves / SIMD
    using S = NcfShape<E>;
    constexpr int NH = S::NH, IN0 = 2 * E;
    // E = 64 takes a CU's LDS alone (one wave per SIMD, registers to spare): its serial
    // LDS reductions are unrolled into one batch of reads; the small towers keep their
    // registers for occupancy (several tiles per CU)
    constexpr bool kWide = E >= 64 && kNT == 256;
    const int M = a.mf_dim, P = S::P + M;  // flat parameters: tower, output W (8 + M), output b
    constexpr int WO = S::w_off(NH);       // flat offset of the output layer
    extern __shared__ float lds[];
    float *sW = lds;                      // padded weights
    float *sA = sW + S::SW;               // activations A_0 .. A_NH, [kRows][H_k + 1]
    float *sM = sA + S::SA;               // multipliers / deltas, same layout as sA (k >= 1)
    float *sP = sM + S::SA;               // p per row
    float *sDz = sP + kRows;              // dL/dlogit per row
    int *sU = reinterpret_cast<int *>(sDz + kRows);
    int *sI = sU + kRows;
    int *sR = sI + kRows;                 // per row: reference row of its mask (pos: column, neg: draw j)
    uint32_t *sK = reinterpret_cast<uint32_t *>(sR + kRows);   // per row: dropout hash key
    float *sLa = reinterpret_cast<float *>(sK + kRows);        // per column loss terms
    float *sLb = sLa + kRows;
    int *sLu = reinterpret_cast<int *>(sLb + kRows);          // per row: user list slot (-1: none)
    int *sLi = sLu + kRows;                                   // per row: item list slot (-1: none / planned)
    int *sPs = sLi + kRows;                                   // per row: plan slot of a positive (-1: none)
    float *sX = sM + S::sa_off(0);                            // dX rows [kRows][IN0 + 1] (M_0 is unused)
    int *sUn = sPs + kRows;                                   // next tile's ids (pipelined E = 64 path)
    int *sIn = sUn + kRows;
    float *sG = reinterpret_cast<float *>(sIn + kRows) + 8;   // weight-gradient accumulator (flat, P)
    float *sWm = sG + P;                                      // NeuMF output weights of the GMF units
    // NeuMF GMF rows: U_mf at [r * gs], I_mf at [r * gs + M] (dX region, free until the tower's last backward)
    const int gs = M <= E ? IN0 + 1 : 2 * M + 1;
    float *sGm = M <= E ? sX : sWm + M;
    constexpr int cl_base = 0;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr bool kBackward = PHASE != kNcfScores && PHASE != kNcfLossOnly;
    const int n = a.n_neg, NP = n + 1, tc = a.tc;
    // E = 64 training: the next tile's pair ids are loaded at this tile's start, its list
    // slots claimed and its A_0 rows gathered into registers during this tile's backward,
    // so a tile starts with its inputs in hand (the id and gather phases were ~4 us of a
    // ~26 us tile).  The small towers keep their registers for occupancy.
    // With 8 waves (registers for two per SIMD) only the ids and slots run ahead (kPipe);
    // the A_0 rows are gathered at the tile's start (kPipeRows off).
    constexpr bool kPipe = E >= 64 && kBackward;
    constexpr bool kPipeRows = kPipe && kWide;
    constexpr int kPG = kPipeRows ? kRows * (IN0 / 4) / kNT : 1;   // float4 per thread of A_0
    static_assert(!kPipeRows || kRows * (IN0 / 4) % kNT == 0, "A_0 prefetch shape");
    bool pre_ok = false;                  // registers hold this tile's ids, slots and A_0
    int nu = -1, ni = -1, nps = -1, nlu = -1, nli = -1, ncol = 0;
    float4 pg[kPG];

    // ---- parameters into LDS (row stride H_k + 1), gradient accumulator zeroed ----
    for (int k = 0; k < NH; ++k) {
        const int in = S::H(k), out = S::H(k + 1);
        const float *W = a.mlp + S::w_off(k);
        float *dst = sW + S::sw_off(k);
        for (int e = tid; e < out * in; e += kNT) dst[(e / in) * (in + 1) + e % in] = W[e];
        for (int e = tid; e < out; e += kNT) dst[out * (in + 1) + e] = W[out * in + e];
    }
    for (int e = tid; e < 9; e += kNT) sW[S::sw_off(NH) + e] = a.mlp[WO + (e < 8 ? e : 8 + M)];
    for (int e = tid; e < M; e += kNT) sWm[e] = a.mlp[WO + 8 + e];
    for (int e = tid; e < P; e += kNT) sG[e] = 0.0f;
    __syncthreads();

    for (int64_t tile = blockIdx.x; tile < a.tiles; tile += gridDim.x) {
        const int tl_ = (int)((tile - blockIdx.x) / gridDim.x);
        NS(0);
        const int64_t c0 = tile * tc;
        // ---- row ids: row r = q * tc + cl ----------------------------------------------
        if (tid < kRows) {
            const int r = tid, q = r / tc, cl = r % tc;
            const int64_t s = c0 + cl;
            const bool pairwise = a.loss == RG_LOSS_BPR || a.loss == RG_LOSS_HINGE;
            bool valid = q < NP && s < a.cols;
            if (valid && q == 0) valid = s < a.n_pos;
            if (valid && q > 0 && pairwise) valid = s < a.n_pos;
            int u = -1, i = -1;
            if (kPipe && pre_ok) {
                u = nu;
                i = ni;
            } else if (valid) {
                const int2 pr = a.pairs[s * pair_stride(a.n_neg) + q];
                u = pr.x;
                i = pr.y;
            }
            sU[r] = u;
            sI[r] = i;
            // the example's identity for dropout: recorded-mask row, or the hash key
            const int64_t colid = (kPipe && pre_ok) ? (int64_t)ncol : a.perm && s < a.cols ? (int64_t)a.perm[s] : s;
            // (global: a data-parallel rank's column slice keys its examples as the single
            // process at the global batch does -- draw index, or column for the positive)
            const int64_t gj = q == 0 ? a.col_offset + colid : (int64_t)(q - 1) * a.global_cols + a.col_offset + colid;
            sR[r] = (int)gj;
            sK[r] = hash32(a.seed ^ ((uint64_t)(q == 0 ? 0 : 1) << 40) ^ ((uint64_t)gj * 0x9E3779B97F4A7C15ULL));
            // list slots are claimed now (the entry does not depend on the gradient), so the
            // atomics' round trip overlaps the gather; overflow rows add from LDS at the end
            int lu = -1, li = -1, ps = -1;
            if (kPipe && pre_ok) {
                // slots claimed during the previous tile's backward; their entries are
                // written now that the atomics have long returned
                lu = nlu;
                li = nli;
                ps = nps;
                const int64_t ex = tile * kRows + r;
                if (lu >= 0 && lu < kNcfCap) store_entry(a.row_list + (int64_t)u * kNcfCap + lu, (int)ex, 1.0f);
                if (li >= 0 && li < kNcfCap)
                    store_entry(a.row_list + (a.num_users + i) * kNcfCap + li, (int)ex, 1.0f);
            } else if (kBackward && u >= 0) {
                const int64_t ex = tile * kRows + r;
                lu = atomicAdd(a.row_count + u, 1);
                if (lu < kNcfCap) store_entry(a.row_list + (int64_t)u * kNcfCap + lu, (int)ex, 1.0f);
                if (q == 0 && a.pos_slot != nullptr) {
                    ps = a.pos_slot[s];
                } else {
                    const int64_t row = a.num_users + i;
                    li = atomicAdd(a.row_count + row, 1);
                    if (li < kNcfCap) store_entry(a.row_list + row * kNcfCap + li, (int)ex, 1.0f);
                }
            }
            sLu[r] = lu;
            sLi[r] = li;
            sPs[r] = ps;
            if constexpr (kPipe) {      // the next tile's record entries, consumed at backward start
                nu = ni = -1;
                const int64_t nt = tile + gridDim.x, s2 = nt * tc + cl;
                bool v2 = nt < a.tiles && q < NP && s2 < a.cols;
                if (v2 && q == 0) v2 = s2 < a.n_pos;
                if (v2 && q > 0 && pairwise) v2 = s2 < a.n_pos;
                if (v2) {
                    const int2 pr = a.pairs[s2 * pair_stride(a.n_neg) + q];
                    nu = pr.x;
                    ni = pr.y;
                }
                nps = (v2 && q == 0 && a.pos_slot != nullptr) ? a.pos_slot[s2] : -1;
                ncol = (int)(a.perm && s2 < a.cols ? (int64_t)a.perm[s2] : s2);
            }
        }
        __syncthreads();
        NS(1);
        // ---- gather A_0 = [U[u] | I[i]] ------------------------------------------------
        if (kPipeRows && pre_ok) {
#pragma unroll
            for (int j = 0; j < kPG; ++j) {
                const int e = tid + j * kNT, r = e / (IN0 / 4), c4 = (e % (IN0 / 4)) * 4;
                float *d = sA + r * (IN0 + 1) + c4;
                d[0] = pg[j].x; d[1] = pg[j].y; d[2] = pg[j].z; d[3] = pg[j].w;
            }
        } else
        for (int e = tid; e < kRows * (IN0 / 4); e += kNT) {
            const int r = e / (IN0 / 4), c4 = (e % (IN0 / 4)) * 4;
            float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (sU[r] >= 0)
                v = c4 < E ? *reinterpret_cast<const float4 *>(a.user_w + (int64_t)sU[r] * E + c4)
                           : *reinterpret_cast<const float4 *>(a.item_w + (int64_t)sI[r] * E + (c4 - E));
            float *d = sA + r * (IN0 + 1) + c4;
            d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
        for (int e = tid; e < kRows * 2 * M; e += kNT) {      // NeuMF GMF rows
            const int r = e / (2 * M), c = e % (2 * M);
            float v = 0.0f;
            if (sU[r] >= 0)
                v = c < M ? a.mf_user_w[(int64_t)sU[r] * M + c] : a.mf_item_w[(int64_t)sI[r] * M + (c - M)];
            sGm[r * gs + c] = v;
        }
        __syncthreads();
        NS(2);
        // ---- forward hidden layers ---------------------------------------------------------
        static_for<NH>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int in = S::H(k), out = S::H(k + 1), mask_base = S::mask_off(k);
            const float *Ak = sA + S::sa_off(k);
            float *An = sA + S::sa_off(k + 1);
            float *Mn = sM + S::sa_off(k + 1);
            const float *Wk = sW + S::sw_off(k);
            const float *bk = Wk + out * (in + 1);
            constexpr int ct = out < 16 ? 1 : out / 16;
            for (int t = wave; t < 2 * ct; t += kNW) {
                const int i0 = (t / ct) * 16, j0 = (t % ct) * 16;
                const v4f z = mma16<in, kKB>(Ak, in + 1, 1, Wk, 1, in + 1, i0, j0, kRows, out, lane);
                const int col = j0 + (lane & 15);
                if (col < out) {
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int row = i0 + (lane >> 4) * 4 + rr;
                        const float zz = z[rr] + bk[col];
                        float m = zz > 0.0f ? 1.0f : 0.1f;
                        if (a.training) {
                            bool keep;
                            if (a.mask_pos) {
                                const int units = S::mask_units();
                                const uint8_t *mk = row < tc ? a.mask_pos : a.mask_neg;
                                keep = sU[row] >= 0 && mk[(int64_t)sR[row] * units + mask_base + col] != 0;
                            } else {
                                keep = (mix32(sK[row] + (uint32_t)(mask_base + col) * 0x85EBCA6BU) >> 7) & 1U;
                            }
                            m = keep ? 2.0f * m : 0.0f;
                        }
                        An[row * (out + 1) + col] = zz * m;
                        Mn[row * (out + 1) + col] = m;
                    }
                }
            }
            __syncthreads();
            if (k == 0) NS(3);
        });
        // ---- output layer, scores, loss ---------------------------------------------------
        {
            const float *wo = sW + S::sw_off(NH);
            const float *AN = sA + S::sa_off(NH);
            if (tid < kRows) {
                float d = 0.0f;
#pragma unroll
                for (int j = 0; j < 8; ++j) d = fmaf(AN[tid * 9 + j], wo[j], d);
                const float *gu = sGm + tid * gs;
#pragma unroll 8
                for (int c = 0; c < M; ++c) d = fmaf(gu[c] * gu[M + c], sWm[c], d);   // GMF = U_mf * I_mf
                const float p = sigmoidf_ref(d + wo[8]);
                sP[tid] = p;
                sDz[tid] = 0.0f;   // rows no column writes below keep dz = 0
                if (PHASE == kNcfScores) a.scores[tile * kRows + tid] = sU[tid] >= 0 ? p : 0.0f;
            }
        }
        __syncthreads();
        NS(4);
        if (PHASE == kNcfScores) continue;
        // dL/dlogit per row (columns: one thread each) and the tile's loss partials
        if (tid < tc) {
            float la = 0.0f, lb = 0.0f;
            {
                const int cl = tid;
                // loops over the column's pairs run to the compile-time bound with a guard (the
                // loads come from a clamped row), so dp[] stays in registers and the LDS
                // reads of all pairs issue together
                constexpr int QM = RG_MF_MAX_NEG + 1;
                float dp[QM];
#pragma unroll
                for (int q = 0; q < QM; ++q) dp[q] = 0.0f;
                const int r0 = cl;
                const bool has_pos = sU[r0] >= 0;
                if (PHASE == kNcfGivenDp) {
#pragma unroll
                    for (int q = 0; q < QM; ++q)
                        if (q < NP && sU[q * tc + cl] >= 0) dp[q] = a.dp_in[tile * kRows + q * tc + cl];
                } else if (a.loss == RG_LOSS_POINTWISE) {
                    if (has_pos) {
                        const float p = sP[r0];
                        la += -fmaxf(logf(p), -100.0f);
                        dp[0] = ((p - 1.0f) / fmaxf((1.0f - p) * p, 1e-12f)) / a.n_a;
                    }
#pragma unroll
                    for (int q = 1; q < QM; ++q) {
                        const int r = min(q * tc + cl, kRows - 1);
                        const bool ok = q < NP && sU[r] >= 0;
                        const float p = sP[r];
                        if (ok) {
                            lb += -fmaxf(logf(1.0f - p), -100.0f);
                            dp[q] = (p / fmaxf((1.0f - p) * p, 1e-12f)) / a.n_b;
                        }
                    }
                } else if (has_pos) {   // bpr / hinge on the neg.view(n, B) pairing
                    const float g = 1.0f / a.n_a, pp = sP[r0];
#pragma unroll
                    for (int q = 1; q < QM; ++q) {
                        const int r = min(q * tc + cl, kRows - 1);
                        if (q >= NP || sU[r] < 0) continue;
                        if (a.loss == RG_LOSS_BPR) {
                            const float sg = sigmoidf_ref(pp - sP[r]);
                            la += 1.0f - sg;
                            const float dx = (-g) * (1.0f - sg) * sg;
                            dp[0] += dx;
                            dp[q] = -dx;
                        } else {
                            const float x = (sP[r] - pp) + 1.0f;
                            la += fmaxf(x, 0.0f);
                            const float dx = x >= 0.0f ? g : 0.0f;
                            dp[0] -= dx;
                            dp[q] = dx;
                        }
                    }
                }
#pragma unroll
                for (int q = 0; q < QM; ++q) {
                    const int r = min(q * tc + cl, kRows - 1);
                    const float p = sP[r];
                    if (q < NP) sDz[r] = sU[r] >= 0 ? (dp[q] * (1.0f - p)) * p : 0.0f;
                }
            }
            sLa[cl_base + tid] = la;
            sLb[cl_base + tid] = lb;
        }
        __syncthreads();
        if (tid == 0) {     // column order, as the one-thread loop summed them
            float la = 0.0f, lb = 0.0f;
            for (int cl = 0; cl < tc; ++cl) { la += sLa[cl]; lb += sLb[cl]; }
            a.loss_partials[2 * tile] = la;
            a.loss_partials[2 * tile + 1] = lb;
        }
        // (no barrier: thread 0 only reads sLa / sLb, rewritten at the next tile's loss phase)
        NS(5);
        if (PHASE == kNcfLossOnly) continue;         // validation: loss only (run_val_iteration)
        // ---- backward ------------------------------------------------------------------------
        const bool has_next = tile + gridDim.x < a.tiles;
        if constexpr (kPipe) {
            if (tid < kRows && has_next) {
                const int r = tid, q = r / tc;
                const int64_t nt = tile + gridDim.x, ex = nt * kRows + r;
                nlu = nli = -1;
                (void)ex;
                if (nu >= 0) {   // entries are written at the next tile's start (results not waited on here)
                    nlu = atomicAdd(a.row_count + nu, 1);
                    if (!(q == 0 && a.pos_slot != nullptr)) nli = atomicAdd(a.row_count + a.num_users + ni, 1);
                }
                sUn[r] = nu;
                sIn[r] = ni;
            }
        }
        {
            // output layer: dW_out += sum_r dz_r A_NH[r], db_out += sum_r dz_r; G_NH = dz w_out^T
            const float *wo = sW + S::sw_off(NH);
            const float *AN = sA + S::sa_off(NH);
            float *MN = sM + S::sa_off(NH);
            for (int e = tid; e < 9 + M; e += kNT) {     // e: 8 tower units, bias, M GMF units
                float acc = 0.0f;
                auto term = [&](int r) {
                    return e < 8 ? AN[r * 9 + e] : e == 8 ? 1.0f : sGm[r * gs + e - 9] * sGm[r * gs + M + e - 9];
                };
                // in row order; E = 64 reads the operands in batches of kCh (one LDS round
                // trip per batch; all rows at once with 4 waves), the small towers one by one
                // (their registers buy occupancy)
                if constexpr (E >= 64) {
                    constexpr int kCh = kWide ? kRows : 8;
#pragma unroll 1
                    for (int r0 = 0; r0 < kRows; r0 += kCh) {
                        float dz[kCh], tv[kCh];
#pragma unroll
                        for (int r = 0; r < kCh; ++r) {
                            dz[r] = sDz[r0 + r];
                            tv[r] = term(r0 + r);
                        }
#pragma unroll
                        for (int r = 0; r < kCh; ++r) acc = fmaf(dz[r], tv[r], acc);
                    }
                } else {
                    for (int r = 0; r < kRows; ++r) acc = fmaf(sDz[r], term(r), acc);
                }
                sG[WO + (e < 8 ? e : e == 8 ? 8 + M : e - 1)] += acc;
            }
            for (int e = tid; e < kRows * 8; e += kNT) {
                const int r = e / 8, j = e % 8;
                MN[r * 9 + j] = (sDz[r] * wo[j]) * MN[r * 9 + j];      // delta_{NH-1} = G * m
            }
            if (M > 0) {
                // GMF backward: dU_mf = (dz w_c) I_mf, dI_mf = (dz w_c) U_mf (neuMF.py:43-50 under autograd)
                for (int e = tid; e < kRows * M; e += kNT) {
                    const int r = e / M, c = e % M;
                    const float dg = sDz[r] * sWm[c];
                    const float du = dg * sGm[r * gs + M + c], di = dg * sGm[r * gs + c];
                    float *row = a.mf_contrib + (tile * kRows + r) * (int64_t)(2 * M);
                    row[c] = du;
                    row[M + c] = di;
                    if (sLu[r] >= kNcfCap) fix_add(a.mf_hot_grad + (int64_t)sU[r] * M + c, du);
                    if (sLi[r] >= kNcfCap) fix_add(a.mf_hot_grad + (a.num_users + sI[r]) * M + c, di);
                }
                if (a.pos_slot != nullptr) {
                    for (int e = tid; e < tc * M; e += kNT) {
                        const int cl = e / M, c = e % M;
                        const int slot = sPs[cl];
                        if (slot < 0 || (cl > 0 && sPs[cl - 1] == slot)) continue;
                        float acc = 0.0f;
                        for (int cc = cl; cc < tc && sPs[cc] == slot; ++cc)
                            acc += (sDz[cc] * sWm[c]) * sGm[cc * gs + c];
                        a.mf_part_row[(int64_t)slot * M + c] = acc;
                    }
                }
            }
            __syncthreads();
        }
        if constexpr (kPipeRows) {
            if (has_next) {
#pragma unroll
                for (int j = 0; j < kPG; ++j) {
                    const int e = tid + j * kNT, r = e / (IN0 / 4), c4 = (e % (IN0 / 4)) * 4;
                    const int u2 = sUn[r], i2 = sIn[r];
                    pg[j] = u2 < 0 ? make_float4(0.0f, 0.0f, 0.0f, 0.0f)
                                   : c4 < E ? *reinterpret_cast<const float4 *>(a.user_w + (int64_t)u2 * E + c4)
                                            : *reinterpret_cast<const float4 *>(a.item_w + (int64_t)i2 * E + (c4 - E));
                }
            }
        }
        if constexpr (kPipe) {
            pre_ok = has_next;
        }
        static_for<NH>([&](auto kc) {
            constexpr int k = NH - 1 - decltype(kc)::value;
            constexpr int in = S::H(k), out = S::H(k + 1);
            const float *Ak = sA + S::sa_off(k);
            const float *Dk = sM + S::sa_off(k + 1);     // delta_k: [kRows][out + 1]
            const float *Wk = sW + S::sw_off(k);
            float *gW = sG + S::w_off(k);
            // dW_k (out x in) += delta^T A_k ; db_k += column sums of delta
            constexpr int ro = out < 16 ? 1 : out / 16, ci = in / 16;
            for (int t = wave; t < ro * ci; t += kNW) {
                const int i0 = (t / ci) * 16, j0 = (t % ci) * 16;
                const v4f c = mma16<kRows>(Dk, 1, out + 1, Ak, in + 1, 1, i0, j0, out, in, lane);
                const int col = j0 + (lane & 15);
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int o = i0 + (lane >> 4) * 4 + rr;
                    if (o < out) gW[o * in + col] += c[rr];
                }
            }
            for (int o = tid; o < out; o += kNT) {
                float acc = 0.0f;
                if constexpr (E >= 64) {   // batches of LDS reads, then the same in-order sum
                    constexpr int kCh = kWide ? kRows : 8;
#pragma unroll 1
                    for (int r0 = 0; r0 < kRows; r0 += kCh) {
                        float col[kCh];
#pragma unroll
                        for (int r = 0; r < kCh; ++r) col[r] = Dk[(r0 + r) * (out + 1) + o];
#pragma unroll
                        for (int r = 0; r < kCh; ++r) acc += col[r];
                    }
                } else {
                    for (int r = 0; r < kRows; ++r) acc += Dk[r * (out + 1) + o];
                }
                gW[out * in + o] += acc;
            }
            // dA_k = delta W_k (kRows x in): k > 0 -> delta_{k-1} = dA * m_k ; k == 0 -> dX
            constexpr int cj = in / 16;
            for (int t = wave; t < 2 * cj; t += kNW) {
                const int i0 = (t / cj) * 16, j0 = (t % cj) * 16;
                const v4f c = mma16<(out < 4 ? 4 : out), kKB>(Dk, out + 1, 1, Wk, in + 1, 1, i0, j0, kRows, in, lane);
                const int col = j0 + (lane & 15);
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int row = i0 + (lane >> 4) * 4 + rr;
                    if constexpr (k > 0) {
                        float *Mk = sM + S::sa_off(k);
                        Mk[row * (in + 1) + col] = c[rr] * Mk[row * (in + 1) + col];
                    } else {
                        a.contrib[(tile * kRows + row) * (int64_t)IN0 + col] = c[rr];
                        sX[row * (IN0 + 1) + col] = c[rr];
                    }
                }
            }
            __syncthreads();
            if (k == NH - 1) NS(6);
        });
        // ---- embedding gradient: overflow rows (hot users/items), planned item partials -----------
        for (int e = tid; e < 2 * kRows * E; e += kNT) {
            const int r = e / (2 * E), half = (e / E) & 1, c = e % E;
            const int sl = half ? sLi[r] : sLu[r];
            if (sl >= kNcfCap) {
                const int64_t row = half ? a.num_users + sI[r] : (int64_t)sU[r];
                fix_add(a.hot_grad + row * E + c, sX[r * (IN0 + 1) + half * E + c]);
            }
        }
        if (a.pos_slot != nullptr) {
            // positives' item halves, same plan slot -> one partial row (fixed order, plain stores)
            for (int e = tid; e < tc * E; e += kNT) {
                const int cl = e / E, c = e % E;
                const int slot = sPs[cl];
                if (slot < 0 || (cl > 0 && sPs[cl - 1] == slot)) continue;   // not the segment head
                float acc = 0.0f;
                for (int cc = cl; cc < tc && sPs[cc] == slot; ++cc) acc += sX[cc * (IN0 + 1) + E + c];
                a.part_row[(int64_t)slot * E + c] = acc;
            }
        }
        __syncthreads();
        NS(7);
    }
    // ---- the workgroup's weight-gradient partial ------------------------------------------------
    if (kBackward)
        for (int e = tid; e < P; e += kNT) a.wpart[(int64_t)blockIdx.x * P + e] = sG[e];
}

// reduce the weight-gradient partials + optimizer update of the MLP parameters in
// place: a block owns 64 parameters, its kUpdWaves waves sum fixed slices of the
// partials (coalesced 256-B loads, four independent chains so the loads pipeline)
// and combine in LDS in a fixed order (deterministic); block 0 also finalises the loss
constexpr int kUpdWaves = 16;
// mode 0: reduce + update; 1 (data parallel, before the exchange): reduce into grad[0, P)
// and this rank's loss share into grad[P]; 2 (after it): update from grad, loss = grad[P]
__global__ __launch_bounds__(kUpdWaves * 64) void ncf_update_kernel(float *mlp, float *m, float *v, const float *wpart,
                                                        int nparts, int P, rg_opt_t opt, const float *loss_partials,
                                                        int64_t n_partials, double inv_a, double inv_b,
                                                        float *loss_out, int mode, float *grad) {
    __shared__ float red[kMlpSlices][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (mode == 2) {
        const int e = blockIdx.x * 64 + lane;
        if (loss_out && blockIdx.x == 0 && threadIdx.x == 0) *loss_out = grad[P];
        if (wave != 0 || e >= P) return;
        float mm = m ? m[e] : 0.0f, vv = v ? v[e] : 0.0f;
        mlp[e] = opt_update(opt, mlp[e], grad[e], mm, vv);
        if (m) m[e] = mm;
        if (v) v[e] = vv;
        return;
    }
    if ((loss_out || mode == 1) && loss_partials && blockIdx.x == 0 && wave == 0) {
        double sa = 0.0, sb = 0.0;
        int64_t i = lane;
        // batches of 8 strided pairs: the loads of a batch in flight before the same in-order sums
        for (; i + 7 * 64 < n_partials; i += 8 * 64) {
            float2 v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = reinterpret_cast<const float2 *>(loss_partials)[i + q * 64];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                sa += (double)v[q].x;
                sb += (double)v[q].y;
            }
        }
        for (; i < n_partials; i += 64) {
            sa += (double)loss_partials[2 * i];
            sb += (double)loss_partials[2 * i + 1];
        }
        for (int off = 32; off > 0; off >>= 1) {
            sa += __shfl_xor(sa, off);
            sb += __shfl_xor(sb, off);
        }
        if (lane == 0) {
            const float lv = (float)(sa * inv_a + sb * inv_b);
            if (loss_out) *loss_out = lv;
            if (mode == 1) grad[P] = lv;
        }
    }
    static_assert(kUpdWaves == kMlpSlices, "one slice per wave");
    const MlpUpdArgs u{mlp, m, v, wpart, nparts, P, opt, mode, grad};
    mlp_update_block<kUpdWaves>(u, blockIdx.x, red);
}

// adaptive hinge from forward-only scores: dp of every row (positives: hinge
// against the max negative; the argmax negative: minus the sum over active positives)
__global__ __launch_bounds__(256) void ncf_adapt_dp_kernel(const float *scores, float *dp, int64_t rows, int TR, int tc,
                                                          int NP, int64_t n_pos_cols, int64_t cols, float n_a,
                                                          float *loss_partial) {
    __shared__ float smax[256];
    __shared__ int64_t sidx[256];
    __shared__ float scnt[256], sloss[256];
    const int tid = threadIdx.x;
    float best = -1.0f;
    int64_t bi = -1;
    for (int64_t r = tid; r < rows; r += 256) {
        const int64_t tile = r / TR, rr = r % TR;
        const int q = (int)(rr / tc);
        const int64_t s = tile * tc + rr % tc;
        dp[r] = 0.0f;
        if (q >= 1 && q < NP && s < cols && scores[r] > best) { best = scores[r]; bi = r; }
    }
    smax[tid] = best;
    sidx[tid] = bi;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {     // max, first occurrence in draw order on ties
        if (tid < w) {
            const bool take = smax[tid + w] > smax[tid];
            if (take) { smax[tid] = smax[tid + w]; sidx[tid] = sidx[tid + w]; }
        }
        __syncthreads();
    }
    const float mx = smax[0];
    float cnt = 0.0f, ls = 0.0f;
    for (int64_t r = tid; r < rows; r += 256) {
        const int64_t tile = r / TR, rr = r % TR;
        const int64_t s = tile * tc + rr % tc;
        if (rr / tc == 0 && rr < (int64_t)tc && s < n_pos_cols) {
            const float x = (mx - scores[r]) + 1.0f;
            ls += fmaxf(x, 0.0f);
            if (x >= 0.0f) { dp[r] = -(1.0f / n_a); cnt += 1.0f; }
        }
    }
    scnt[tid] = cnt;
    sloss[tid] = ls;
    __syncthreads();
    if (tid == 0) {
        float c = 0.0f, l = 0.0f;
        for (int i = 0; i < 256; ++i) { c += scnt[i]; l += sloss[i]; }
        if (sidx[0] >= 0) dp[sidx[0]] = c * (1.0f / n_a);
        loss_partial[0] = l;
        loss_partial[1] = 0.0f;
    }
}

// ============================================================================================
// E = 64 tower (C3, mf_dim = 0): one WAVE per tile of RG_NCF_WAVE_ROWS rows -- 48 in the product
// build since round 5 (8 whole columns of 1 + 5 rows: 1,024 tiles at B = 8192, n = 5, one per wave
// of the 256 x 4-wave grid), the forward one example block at a time; 32-row tiles (1,639 tiles,
// two rounds) measured 73.3 against 64.0 us.
//
// The tile kernel above keeps every activation in LDS and spreads a tile's MFMA tiles over 8
// waves: ~12 workgroup barriers and an LDS -> MFMA -> LDS round trip per layer, 14 % of the
// fp32 MFMA peak.  Here a wave owns a whole tile and runs the chain with no barrier:
//
//   * "T layout": a 16x16 MFMA C tile of a layer's output transposed, Y^T[feature][example]
//     -- lane (g, j) holds features 16t + 4g + r (r = 0..3) of example 16 nb + j (3 example
//     blocks nb).  Fed back as the B operand of the next product, k-step r of tile t takes
//     feature 16t + 4g + r from lane group g, so  Y_{k+1}^T = W_{k+1} Y_k^T  and
//     dA_k^T = W_k^T delta_k^T  consume the previous result straight from registers (the A
//     operand, a weight, is read from LDS in the same permuted k order).
//   * the forward runs the three example blocks together; the backward one block at a time
//     (a third of the deltas live), each weight-gradient accumulator still taking the tile's
//     examples in row order (block 0's k-steps, then block 1's, ...).
//   * the weight gradients dW_k = sum_e delta_k[e] X_k[e]^T contract over EXAMPLES, which the
//     T layout keeps on lanes; X_k and delta_k are staged into the wave's own LDS rows
//     ([example][feature], unpadded with a rotated column order: conflict-free both ways) and
//     read back with examples on the k axis.  X_0 (the gathered embeddings) is re-read from L2
//     in that layout.  dW accumulates in MFMA accumulators across the wave's tiles; the hidden
//     biases' gradients are per-lane column sums taken from the same reads (no ones operand).
//   * one workgroup of 4 waves per CU (151 KB of LDS, 512 registers per lane); at the end the
//     4 waves' gradients are summed in wave order in LDS into the workgroup's partial.
// Every sum is a fixed-order f32 chain (MFMA = k-ordered fmaf chain), so results are
// deterministic; the order differs from the tile kernel's, so the two agree to fp32 rounding.
// ============================================================================================
namespace ncfw {
constexpr int kWaves = 4, kThreads = 64 * kWaves;
// The forward one 16-example block at a time (as the backward), so a 48-row tile -- 8 whole
// columns of 1 + 5 rows, 1,024 tiles at B = 8192: one per wave slot, no second round -- fits the
// registers (12 B of scratch; 80 B with the forward over all blocks at once).  Measured (round 5,
// profiles/r5/ncf/ncf_fwd_r6a.txt): 73.3 us per launch with 32-row tiles (1,639 tiles: two rounds
// on 1,024 slots), 64.0 with these; 0: every block's forward at once (32 rows: 73.2 us)
#ifndef RG_NCF_EARLY_TILE
#define RG_NCF_EARLY_TILE 0      // 1: the first tile begun before the weights' barrier (its loop-carried
                                 // state costs 156 B of scratch: 67.7-68.3 vs 62.3-63.0 us per launch,
                                 // same box, profiles/r6/ncf/ncf_early_tile_ab_r6l.txt)
#endif
#ifndef RG_NCF_FWD_ROLLED
#define RG_NCF_FWD_ROLLED 0      // 1: the blockwise forward's block loop kept rolled (400 B of scratch)
#endif
#ifndef RG_NCF_FWD_BLOCKWISE
#define RG_NCF_FWD_BLOCKWISE 1
#endif
#ifndef RG_NCF_WAVE_ROWS
#define RG_NCF_WAVE_ROWS 48   // 32: two rounds of tiles at B = 8192, n = 5 (1,639 tiles on 1,024 slots)
#endif
constexpr int kR = RG_NCF_WAVE_ROWS, NB = kR / 16;   // 48 rows = 3 example blocks of 16 (n = 5: 8 whole columns)
// weights in LDS (floats): W_k row-major [out][in + 4] (b128 rows land on distinct 16-B slots),
// W4 and the output row padded to 16 rows of zeros, biases padded with zeros
constexpr int S1 = 132, S2 = 68, S3 = 36, S4 = 20, SO = 20;
constexpr int oW1 = 0, oW2 = oW1 + 64 * S1, oW3 = oW2 + 32 * S2, oW4 = oW3 + 16 * S3, oWo = oW4 + 16 * S4;
constexpr int oB1 = oWo + 16 * SO, oB2 = oB1 + 64, oB3 = oB2 + 32, oB4 = oB3 + 16, oBo = oB4 + 16;
constexpr int kWFloats = oBo + 4;
// per wave: staged activations / deltas [48][F] (F = 64, 32, 16, 16 features, unpadded: the
// column of row r is rotated by 16 (r & 3) for F = 64 and by 16 ((r >> 1) & 1) for F = 32, so the
// example-on-k reads of lane (g, x) -- row 4 s + g, column 16 t + x -- hit 64 distinct banks),
// then the tile's small per-row arrays
constexpr int R1S = 64, R2S = 32, R3S = 16, R4S = 16;
constexpr int oR1 = 0, oR2 = oR1 + kR * R1S, oR3 = oR2 + kR * R2S, oR4 = oR3 + kR * R3S, oSm = oR4 + kR * R4S;
constexpr int kSmall = 11;
constexpr int kWaveFloats = oSm + kSmall * kR;
constexpr int kLdsFloats = kWFloats + kWaves * kWaveFloats;
constexpr int P = NcfShape<64>::P;
static_assert(kLdsFloats <= kLdsMax, "LDS");
static_assert((kR / 2) * 64 <= kR * R2S, "planned item halves ([tc <= kR / 2][64]) fit the delta2 rows");
static_assert(kWFloats % 4 == 0 && kWaveFloats % 4 == 0, "16-B alignment");
static_assert(kR <= 64 && kR % 16 == 0, "one lane per row, whole example blocks");

// float index of (row, column) in a staged [kR][RS] buffer (column a multiple of 4 for float4
// accesses stays inside its 16-column group)
template <int RS>
__device__ __forceinline__ int at(int row, int col) {
    if constexpr (RS == 64) return row * 64 + ((col + 16 * (row & 3)) & 63);
    else if constexpr (RS == 32) return row * 32 + ((col + 16 * ((row >> 1) & 1)) & 31);
    else return row * RS + col;
}

// orders this wave's LDS traffic for the compiler: DS instructions of one wave execute in
// order, so a wavefront-scope fence (no wait instruction) is all a cross-lane LDS hand-off
// inside the wave needs
__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }

__device__ __forceinline__ v4f mfma(float a, float b, v4f c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

// Y^T (TO tiles) = W X^T: W [16 TO][16 TI] (row stride S), X^T T-layout (TI tiles)
template <int TI, int TO>
__device__ __forceinline__ void fwd(const v4f (&x)[TI][NB], v4f (&y)[TO][NB], const float *W, int S, int g, int m) {
#pragma unroll
    for (int t = 0; t < TO; ++t)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) y[t][nb] = v4f{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int ti = 0; ti < TI; ++ti) {
        v4f a[TO];
#pragma unroll
        for (int t = 0; t < TO; ++t) a[t] = *reinterpret_cast<const v4f *>(W + (16 * t + m) * S + 16 * ti + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < TO; ++t)
#pragma unroll
                for (int nb = 0; nb < NB; ++nb) y[t][nb] = mfma(a[t][r], x[ti][nb][r], y[t][nb]);
    }
}

// dA^T (TI tiles) = W^T delta^T: W [16 TO][16 TI] row-major (stride S), delta^T T-layout (TO
// tiles); W may point at a column block of a wider matrix (its first of TI column tiles)
template <int TI, int TO>
__device__ __forceinline__ void bwd(const v4f (&d)[TO][NB], v4f (&da)[TI][NB], const float *W, int S, int g, int x) {
#pragma unroll
    for (int t = 0; t < TI; ++t)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) da[t][nb] = v4f{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int to = 0; to < TO; ++to)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float a[TI];
#pragma unroll
            for (int ti = 0; ti < TI; ++ti) a[ti] = W[(16 * to + 4 * g + r) * S + 16 * ti + x];
#pragma unroll
            for (int ti = 0; ti < TI; ++ti)
#pragma unroll
                for (int nb = 0; nb < NB; ++nb) da[ti][nb] = mfma(a[ti], d[to][nb][r], da[ti][nb]);
        }
}

// dW[16 TOo][16 TIi] += sum_e D[e][o] X[e][i] over the tile's examples (staged rows), and this
// lane's share of the bias gradient sum_e D[e][o]: the examples e = g (mod 4) of column 16 to + x,
// summed in the same pass over the D operand (the four lane groups are added at the end)
template <int TOo, int TIi, int SD, int SX>
__device__ __forceinline__ void dw(v4f (&acc)[TOo][TIi], float (&bs)[TOo], const float *D, const float *X, int g,
                                   int x) {
#pragma unroll
    for (int s = 0; s < kR / 4; ++s) {
        float a[TOo], b[TIi];
#pragma unroll
        for (int to = 0; to < TOo; ++to) a[to] = D[at<SD>(4 * s + g, 16 * to + x)];
#pragma unroll
        for (int ti = 0; ti < TIi; ++ti) b[ti] = X[at<SX>(4 * s + g, 16 * ti + x)];
#pragma unroll
        for (int to = 0; to < TOo; ++to) {
#pragma unroll
            for (int ti = 0; ti < TIi; ++ti) acc[to][ti] = mfma(a[to], b[ti], acc[to][ti]);
            bs[to] += a[to];
        }
    }
}

// staged rows -> T-layout tiles (the inverse of stage)
template <int T, int RS>
__device__ __forceinline__ void unstage(v4f (&y)[T][NB], const float *R, int g, int j) {
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) y[t][nb] = *reinterpret_cast<const v4f *>(R + at<RS>(nb * 16 + j, 16 * t + 4 * g));
}

// T-layout tiles -> staged rows [example][feature] (float4 per lane)
template <int T, int RS>
__device__ __forceinline__ void stage(const v4f (&y)[T][NB], float *R, int g, int j) {
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) *reinterpret_cast<v4f *>(R + at<RS>(nb * 16 + j, 16 * t + 4 * g)) = y[t][nb];
}

// torch's LeakyReLU(0.1) -> Dropout(0.5) multiplier from the kept bit and the sign of the
// output (A = z m with m > 0 keeps the sign of z; a dropped unit's delta is 0)
__device__ __forceinline__ float mult(float y, bool keep, bool training) {
    const float m1 = y > 0.0f ? 1.0f : 0.1f;
    return training ? (keep ? 2.0f * m1 : 0.0f) : m1;
}

// ---- one example block (16 examples, lane j = example 16 nb + j): the backward runs block by
// block so a third of the tile's activations / deltas is live at a time ----
// dA^T (TI tiles) = W^T delta^T for one block
template <int TI, int TO>
__device__ __forceinline__ void bwd1(const v4f (&d)[TO], v4f (&da)[TI], const float *W, int S, int g, int x) {
#pragma unroll
    for (int t = 0; t < TI; ++t) da[t] = v4f{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int to = 0; to < TO; ++to)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float a[TI];
#pragma unroll
            for (int ti = 0; ti < TI; ++ti) a[ti] = W[(16 * to + 4 * g + r) * S + 16 * ti + x];
#pragma unroll
            for (int ti = 0; ti < TI; ++ti) da[ti] = mfma(a[ti], d[to][r], da[ti]);
        }
}
// dW += the block's examples (k-steps s0 .. s0 + 3 of the tile: rows 4 s + g), bias column sums
template <int TOo, int TIi, int SD, int SX>
__device__ __forceinline__ void dw1b(v4f (&acc)[TOo][TIi], float (&bs)[TOo], const float *D, const float *X, int g,
                                     int x, int s0) {
#pragma unroll
    for (int s = s0; s < s0 + 4; ++s) {
        float a[TOo], b[TIi];
#pragma unroll
        for (int to = 0; to < TOo; ++to) a[to] = D[at<SD>(4 * s + g, 16 * to + x)];
#pragma unroll
        for (int ti = 0; ti < TIi; ++ti) b[ti] = X[at<SX>(4 * s + g, 16 * ti + x)];
#pragma unroll
        for (int to = 0; to < TOo; ++to) {
#pragma unroll
            for (int ti = 0; ti < TIi; ++ti) acc[to][ti] = mfma(a[to], b[ti], acc[to][ti]);
            bs[to] += a[to];
        }
    }
}
template <int T, int RS>
__device__ __forceinline__ void unstage1(v4f (&y)[T], const float *R, int row, int g) {
#pragma unroll
    for (int t = 0; t < T; ++t) y[t] = *reinterpret_cast<const v4f *>(R + at<RS>(row, 16 * t + 4 * g));
}
template <int T, int RS>
__device__ __forceinline__ void stage1(const v4f (&y)[T], float *R, int row, int g) {
#pragma unroll
    for (int t = 0; t < T; ++t) *reinterpret_cast<v4f *>(R + at<RS>(row, 16 * t + 4 * g)) = y[t];
}

// Y^T (TO tiles) = W X^T for one example block (the forward one 16-example block at a time)
template <int TI, int TO>
__device__ __forceinline__ void fwd1(const v4f (&x)[TI], v4f (&y)[TO], const float *W, int S, int g, int m) {
#pragma unroll
    for (int t = 0; t < TO; ++t) y[t] = v4f{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int ti = 0; ti < TI; ++ti) {
        v4f a[TO];
#pragma unroll
        for (int t = 0; t < TO; ++t) a[t] = *reinterpret_cast<const v4f *>(W + (16 * t + m) * S + 16 * ti + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < TO; ++t) y[t] = mfma(a[t][r], x[ti][r], y[t]);
    }
}

// bit of unit (t, nb, r) of a layer in its keep word
__device__ __forceinline__ constexpr int kbit(int t, int nb, int r) { return (t * NB + nb) * 4 + r; }
}  // namespace ncfw

// Diagnostic build only: per-wave phase stamps of its first two tiles (16 slots per tile),
// each draining the wave's loads and LDS traffic first (scripts/ncf_stamps.py --wave)
#ifdef RG_DIAG_STAMPS
#define WS(k)                                                                                              \
    do {                                                                                                   \
        if (g_ncf_stamps && tl_ < 2) {                                                                     \
            unsigned long long t_;                                                                         \
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memrealtime %0\n\ts_waitcnt lgkmcnt(0)"      \
                         : "=s"(t_)::"memory");                                                            \
            if (lane == 0) g_ncf_stamps[(((int64_t)blockIdx.x * ncfw::kWaves + wave) * 3 + tl_) * 16 + (k)] = t_; \
        }                                                                                                  \
    } while (0)
// stamps inside the backward's block loop: block 0's only (the later blocks' phases are the
// "blocks 1.." stamp pair, so no stamp is overwritten by a later block)
#define WSB(k)          \
    do {                \
        if (nb == 0) WS(k); \
    } while (0)
#define WSK(k)                                                                                             \
    do {                                                                                                   \
        if (g_ncf_stamps) {                                                                                \
            unsigned long long t_;                                                                         \
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memrealtime %0\n\ts_waitcnt lgkmcnt(0)"      \
                         : "=s"(t_)::"memory");                                                            \
            if (lane == 0) g_ncf_stamps[(((int64_t)blockIdx.x * ncfw::kWaves + wave) * 3 + 2) * 16 + (k)] = t_; \
        }                                                                                                  \
    } while (0)
#else
#define WS(k) \
    do {      \
    } while (0)
#define WSK(k) \
    do {      \
    } while (0)
#define WSB(k) \
    do {      \
    } while (0)
#endif

template <int PHASE>
__global__ __launch_bounds__(ncfw::kThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) void ncf_wave_kernel(NcfArgs a) {
    using namespace ncfw;
    using S64 = NcfShape<64>;
    constexpr bool kBackward = PHASE != kNcfScores && PHASE != kNcfLossOnly;
    constexpr int WO = S64::w_off(4);
    extern __shared__ float lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, j = lane & 15;
    float *sw = lds;
    float *ws = lds + kWFloats + wave * kWaveFloats;
    float *R1 = ws + oR1, *R2 = ws + oR2, *R3 = ws + oR3, *R4 = ws + oR4;
    int *sU = reinterpret_cast<int *>(ws + oSm), *sI = sU + kR, *sR = sI + kR;
    uint32_t *sK = reinterpret_cast<uint32_t *>(sR + kR);
    float *sP = reinterpret_cast<float *>(sK + kR), *sDz = sP + kR, *sLa = sDz + kR, *sLb = sLa + kR;
    int *sLu = reinterpret_cast<int *>(sLb + kR), *sLi = sLu + kR, *sPs = sLi + kR;
    WSK(0);   // kernel entry (diag: kernel-level record 2)

    // ---- parameters: every load issued first, then the LDS stores (the first tile's record is
    // fetched in between), then one barrier ----
    constexpr int kTail = kWFloats - oW4;   // W4 rows (8..15 zero), the output row, the biases
    constexpr int PT1 = 64 * 128 / 4 / kThreads, PT2 = 32 * 64 / 4 / kThreads, PT3 = (16 * 32 / 4 + kThreads - 1) / kThreads;
    constexpr int PTT = (kTail + kThreads - 1) / kThreads;
    static_assert(64 * 128 / 4 % kThreads == 0 && 32 * 64 / 4 % kThreads == 0, "weight copy shape");
    float4 wv1[PT1], wv2[PT2], wv3[PT3];
    float wvt[PTT];
    {
        const float4 *W1 = reinterpret_cast<const float4 *>(a.mlp + S64::w_off(0));
        const float4 *W2 = reinterpret_cast<const float4 *>(a.mlp + S64::w_off(1));
        const float4 *W3 = reinterpret_cast<const float4 *>(a.mlp + S64::w_off(2));
#pragma unroll
        for (int k = 0; k < PT1; ++k) wv1[k] = W1[tid + k * kThreads];
#pragma unroll
        for (int k = 0; k < PT2; ++k) wv2[k] = W2[tid + k * kThreads];
#pragma unroll
        for (int k = 0; k < PT3; ++k) wv3[k] = W3[min(tid + k * kThreads, 16 * 32 / 4 - 1)];
#pragma unroll
        for (int k = 0; k < PTT; ++k) {   // flat source index of LDS float oW4 + e (or -1: zero)
            const int o = oW4 + min(tid + k * kThreads, kTail - 1);
            int src = -1;
            if (o < oWo) {
                const int row = (o - oW4) / S4, col = (o - oW4) % S4;
                if (row < 8 && col < 16) src = S64::w_off(3) + row * 16 + col;
            } else if (o < oB1) {
                if (o - oWo < 8) src = WO + (o - oWo);
            } else if (o < oB2) {
                src = S64::w_off(0) + 64 * 128 + (o - oB1);
            } else if (o < oB3) {
                src = S64::w_off(1) + 32 * 64 + (o - oB2);
            } else if (o < oB4) {
                src = S64::w_off(2) + 16 * 32 + (o - oB3);
            } else if (o < oBo) {
                if (o - oB4 < 8) src = S64::w_off(3) + 8 * 16 + (o - oB4);
            } else if (o == oBo) {
                src = WO + 8;
            }
            const float v = a.mlp[src < 0 ? 0 : src];
            wvt[k] = src < 0 ? 0.0f : v;
        }
    }
    const float *W1s = sw + oW1, *W2s = sw + oW2, *W3s = sw + oW3, *W4s = sw + oW4, *Wos = sw + oWo;
    const bool training = a.training != 0;
    const int n = a.n_neg, NP = n + 1, tc = a.tc;
    constexpr int units = S64::mask_units();
    const bool pairwise = a.loss == RG_LOSS_BPR || a.loss == RG_LOSS_HINGE;

    // running gradients of this wave: the weight tiles and the output layer's [w_out | b_out]
    // tile in MFMA accumulators, the hidden biases as per-lane column sums (lane (g, x): the
    // examples e = g mod 4 of feature 16 t + x)
    v4f gW1[4][8], gW2[2][4], gW3[1][2], gW4[1][1], gO;
    float bB1[4] = {0.0f, 0.0f, 0.0f, 0.0f}, bB2[2] = {0.0f, 0.0f}, bB3[1] = {0.0f}, bB4[1] = {0.0f};
    const v4f z4 = v4f{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 8; ++q) gW1[p][q] = z4;
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) gW2[p][q] = z4;
    gW3[0][0] = gW3[0][1] = gW4[0][0] = gO = z4;

    // a column's pair record for row r = q * tc + cl of `tile` (lanes 0..31): the loads are
    // issued unconditionally from clamped indices (fetch) and resolved when the values are
    // needed, a tile later (finish), so no wait sits in between
    struct RowRaw {
        int2 pr;
        int ps, perm;
        int64_t s;
        int q;
        bool valid;
    };
    auto fetch_row = [&](int64_t tile, int r) {
        RowRaw w;
        w.q = r / tc;
        const int cl = r % tc;
        w.s = tile * tc + cl;
        bool valid = tile < a.tiles && w.q < NP && w.s < a.cols;
        if (valid && w.q == 0) valid = w.s < a.n_pos;
        if (valid && w.q > 0 && pairwise) valid = w.s < a.n_pos;
        w.valid = valid;
        w.pr = make_int2(-1, -1);
        w.ps = -1;
        w.perm = 0;
        if (tile < a.tiles) {   // (a tile past the end has no record to read: cols may be 0)
            const int64_t sc = w.s < a.cols ? w.s : a.cols - 1;
            w.pr = a.pairs[sc * pair_stride(a.n_neg) + min(w.q, n)];
            w.ps = a.pos_slot != nullptr ? a.pos_slot[sc] : -1;
            w.perm = a.perm ? a.perm[sc] : 0;
        }
        return w;
    };
    auto finish_row = [&](const RowRaw &w, int &u, int &i, int &ps, int64_t &gj) {
        u = w.valid ? w.pr.x : -1;
        i = w.valid ? w.pr.y : -1;
        ps = (kBackward && w.valid && w.q == 0) ? w.ps : -1;
        const int64_t colid = a.perm && w.s < a.cols ? (int64_t)w.perm : w.s;
        gj = w.q == 0 ? a.col_offset + colid : (int64_t)(w.q - 1) * a.global_cols + a.col_offset + colid;
    };

    const int64_t waves_total = (int64_t)gridDim.x * kWaves;
    const int64_t first = (int64_t)blockIdx.x * kWaves + wave;
    RowRaw nxt{};   // the next tile's record (lanes 0..31), in flight during this tile
    if (lane < kR) nxt = fetch_row(first, lane);
    // a tile's start: its record resolved into the wave's row arrays, the gather of X0 issued
    auto begin_tile = [&](int tcl, int &ru, int &ri, int &rps, int (&ue)[NB], int (&ie)[NB], int (&re)[NB],
                          uint32_t (&ke)[NB], v4f (&x0)[8][NB]) {
        int64_t ngj = 0;
        if (lane < kR) {
            finish_row(nxt, ru, ri, rps, ngj);
            const int r = lane, q = r / tcl;
            sU[r] = ru;
            sI[r] = ri;
            sR[r] = (int)ngj;
            sK[r] = hash32(a.seed ^ ((uint64_t)(q == 0 ? 0 : 1) << 40) ^ ((uint64_t)ngj * 0x9E3779B97F4A7C15ULL));
            sDz[r] = 0.0f;
            sPs[r] = rps;
        }
        wave_sync();
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
            ue[nb] = sU[nb * 16 + j];
            ie[nb] = sI[nb * 16 + j];
            re[nb] = sR[nb * 16 + j];
            ke[nb] = sK[nb * 16 + j];
        }
        // ---- gather X0^T (T layout): features 16 t + 4 g .. + 3 of example nb * 16 + j; a row
        // that is not a valid pair reads row 0 (its dz is 0, so none of its values reach a
        // gradient, and its score is never used) ----
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
            const float *pu = a.user_w + (int64_t)(ue[nb] >= 0 ? ue[nb] : 0) * 64 + 4 * g;
            const float *pi = a.item_w + (int64_t)(ue[nb] >= 0 ? ie[nb] : 0) * 64 + 4 * g;
#pragma unroll
            for (int t = 0; t < 8; ++t) x0[t][nb] = *reinterpret_cast<const v4f *>(t < 4 ? pu + 16 * t : pi + 16 * (t - 4));
        }
    };
    // the weights into LDS (the first record's loads above are in flight meanwhile; inline, not
    // a lambda: a captured register array would live in scratch)
#pragma unroll
    for (int k = 0; k < PT1; ++k) {
        const int e = tid + k * kThreads;
        *reinterpret_cast<float4 *>(sw + oW1 + (e / 32) * S1 + (e % 32) * 4) = wv1[k];
    }
#pragma unroll
    for (int k = 0; k < PT2; ++k) {
        const int e = tid + k * kThreads;
        *reinterpret_cast<float4 *>(sw + oW2 + (e / 16) * S2 + (e % 16) * 4) = wv2[k];
    }
#pragma unroll
    for (int k = 0; k < PT3; ++k) {
        const int e = tid + k * kThreads;
        if (e < 16 * 32 / 4) *reinterpret_cast<float4 *>(sw + oW3 + (e / 8) * S3 + (e % 8) * 4) = wv3[k];
    }
#pragma unroll
    for (int k = 0; k < PTT; ++k)
        if (tid + k * kThreads < kTail) sw[oW4 + tid + k * kThreads] = wvt[k];
#if RG_NCF_EARLY_TILE
    // the first tile's ids and its X0 gather issued before the weights' barrier (they touch only
    // this wave's LDS rows and global memory): its latency overlaps the other waves' weight copy
    int ru = -1, ri = -1, rps = -1, ue[NB], ie[NB], re[NB];
    uint32_t ke[NB];
    v4f x0[8][NB];
    bool begun = false;
    if (first < a.tiles) {
        begin_tile(a.tc, ru, ri, rps, ue, ie, re, ke, x0);
        begun = true;
    }
#endif
    __syncthreads();
    float warm = 0.0f;   // the next tile's embedding lines, touched during this tile's backward
    for (int64_t tile = first; tile < a.tiles; tile += waves_total) {
        int tc = a.tc;   // opaque per tile: keeps the loss / row addresses from being hoisted (and spilled)
        asm volatile("" : "+s"(tc));
        const int tl_ = (int)((tile - first) / waves_total);
        (void)tl_;
        WS(0);
#if RG_NCF_EARLY_TILE
        if (!begun) begin_tile(tc, ru, ri, rps, ue, ie, re, ke, x0);
        begun = false;
#else
        int ru = -1, ri = -1, rps = -1, ue[NB], ie[NB], re[NB];
        uint32_t ke[NB];
        v4f x0[8][NB];
        begin_tile(tc, ru, ri, rps, ue, ie, re, ke, x0);
#endif
        if (warm == 1.0e30f && a.n_pos < 0) a.scores[0] = warm;   // keeps the warm-up loads (never taken)
        WS(1);
        // dropout bits of every unit of the tile, computed while the gather is in flight
        // (bit kbit(t, nb, r) of a layer's word: feature 16 t + 4 g + r, example nb * 16 + j)
        auto keep_bits = [&](auto tc_, int out, int mask_base) -> uint64_t {
            constexpr int T = decltype(tc_)::value;
            uint64_t keep = 0;
            if (!training) return keep;
            if (a.mask_pos) {   // recorded masks (parity tests): every byte load first
                uint8_t mv[T][NB][4];
#pragma unroll
                for (int nb = 0; nb < NB; ++nb) {
                    const uint8_t *mk = (nb * 16 + j < tc ? a.mask_pos : a.mask_neg) +
                                        (int64_t)(ue[nb] >= 0 ? re[nb] : 0) * units + mask_base;
#pragma unroll
                    for (int t = 0; t < T; ++t)
#pragma unroll
                        for (int r = 0; r < 4; ++r) mv[t][nb][r] = mk[min(16 * t + 4 * g + r, out - 1)];
                }
#pragma unroll
                for (int t = 0; t < T; ++t)
#pragma unroll
                    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            keep |= (uint64_t)(mv[t][nb][r] != 0 && ue[nb] >= 0 && 16 * t + 4 * g + r < out)
                                    << kbit(t, nb, r);
            } else {
#pragma unroll
                for (int t = 0; t < T; ++t)
#pragma unroll
                    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int f = 16 * t + 4 * g + r;
                            const uint32_t h = mix32(ke[nb] + (uint32_t)(mask_base + f) * 0x85EBCA6BU);
                            keep |= (uint64_t)(((h >> 7) & 1U) & (uint32_t)(f < out)) << kbit(t, nb, r);
                        }
            }
            return keep;
        };
        // layer 1 (4 x NB x 4 = 48 bits) in kb1; layers 2, 3, 4 (24 + 12 + 12 bits) in kb2
        const uint64_t kb1 = keep_bits(std::integral_constant<int, 4>{}, 64, S64::mask_off(0));
        const uint64_t kb2 = keep_bits(std::integral_constant<int, 2>{}, 32, S64::mask_off(1)) |
                             keep_bits(std::integral_constant<int, 1>{}, 16, S64::mask_off(2)) << 24 |
                             keep_bits(std::integral_constant<int, 1>{}, 8, S64::mask_off(3)) << 36;
        static_assert(kbit(3, NB - 1, 3) < 64 && kbit(1, NB - 1, 3) + 1 + 2 * (kbit(0, NB - 1, 3) + 1) <= 64,
                      "keep words");
        // list slots claimed behind the gather (their round trip overlaps it and the first layer;
        // the entries are written after it)
        int lu = -1, li = -1;
        if (kBackward && lane < kR && ru >= 0) {
            lu = atomicAdd(a.row_count + ru, 1);
            if (rps < 0 && !(lane < tc && a.pos_slot != nullptr)) li = atomicAdd(a.row_count + a.num_users + ri, 1);
        }
        WS(2);
        // ---- forward ----
        // bias, LeakyReLU(0.1), Dropout(0.5) as one multiplier per unit
        auto activate = [&](auto &y, const float *b, uint64_t kw, int bit0) {
            constexpr int T = sizeof(y) / sizeof(y[0]);
            v4f bv[T];
#pragma unroll
            for (int t = 0; t < T; ++t) bv[t] = *reinterpret_cast<const v4f *>(b + 16 * t + 4 * g);
#pragma unroll
            for (int t = 0; t < T; ++t)
#pragma unroll
                for (int nb = 0; nb < NB; ++nb)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float z = y[t][nb][r] + bv[t][r];
                        const float m1 = z > 0.0f ? 1.0f : 0.1f;
                        const float m = training ? (((kw >> (bit0 + kbit(t, nb, r))) & 1U) ? 2.0f * m1 : 0.0f) : m1;
                        y[t][nb][r] = z * m;
                    }
        };
#if RG_NCF_FWD_BLOCKWISE
        // the forward one 16-example block at a time (as the backward): one block's activations
        // live at once, so a 48-row tile (three blocks) fits the registers of a 32-row one
        auto activate1 = [&](auto &y, const float *b, uint64_t kw, int bit0, int nb) {
            constexpr int T = sizeof(y) / sizeof(y[0]);
            v4f bv[T];
#pragma unroll
            for (int t = 0; t < T; ++t) bv[t] = *reinterpret_cast<const v4f *>(b + 16 * t + 4 * g);
#pragma unroll
            for (int t = 0; t < T; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float z = y[t][r] + bv[t][r];
                    const float m1 = z > 0.0f ? 1.0f : 0.1f;
                    const float m = training ? (((kw >> (bit0 + kbit(t, nb, r))) & 1U) ? 2.0f * m1 : 0.0f) : m1;
                    y[t][r] = z * m;
                }
        };
        const float bo = sw[oBo];
#if RG_NCF_FWD_ROLLED
#pragma unroll 1
#else
#pragma unroll
#endif
        for (int nb = 0; nb < NB; ++nb) {
            const int row = nb * 16 + j;
            v4f xb[8], a1[4], a2[2], a3[1], a4[1], zb[1];
#pragma unroll
            for (int t = 0; t < 8; ++t) xb[t] = x0[t][nb];
            fwd1<8, 4>(xb, a1, W1s, S1, g, j);
            activate1(a1, sw + oB1, kb1, 0, nb);
            stage1<4, R1S>(a1, R1, row, g);
            fwd1<4, 2>(a1, a2, W2s, S2, g, j);
            activate1(a2, sw + oB2, kb2, 0, nb);
            stage1<2, R2S>(a2, R2, row, g);
            fwd1<2, 1>(a2, a3, W3s, S3, g, j);
            activate1(a3, sw + oB3, kb2, 24, nb);
            stage1<1, R3S>(a3, R3, row, g);
            fwd1<1, 1>(a3, a4, W4s, S4, g, j);
            activate1(a4, sw + oB4, kb2, 36, nb);
            if (kBackward) {   // A_4 rows with a ones feature (8) for the output layer's bias gradient
                v4f a4s[1] = {a4[0]};
                if (g == 2) a4s[0][0] = 1.0f;
                stage1<1, R4S>(a4s, R4, row, g);
            }
            fwd1<1, 1>(a4, zb, Wos, SO, g, j);
            if (g == 0) {
                const float p = sigmoidf_ref(zb[0][0] + bo);
                sP[row] = p;
                if (PHASE == kNcfScores) a.scores[tile * kR + row] = ue[nb] >= 0 ? p : 0.0f;
            }
        }
        WS(3);
#else
        v4f y1[4][NB], y2[2][NB], y3[1][NB], y4[1][NB];
        fwd<8, 4>(x0, y1, W1s, S1, g, j);
        WS(3);
        activate(y1, sw + oB1, kb1, 0);
        stage<4, R1S>(y1, R1, g, j);
        fwd<4, 2>(y1, y2, W2s, S2, g, j);
        activate(y2, sw + oB2, kb2, 0);
        stage<2, R2S>(y2, R2, g, j);
        fwd<2, 1>(y2, y3, W3s, S3, g, j);
        activate(y3, sw + oB3, kb2, 24);
        stage<1, R3S>(y3, R3, g, j);
        fwd<1, 1>(y3, y4, W4s, S4, g, j);
        activate(y4, sw + oB4, kb2, 36);
        if (kBackward) {   // A_4 rows with a ones feature (8) for the output layer's bias gradient
            v4f y4s[1][NB];
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
                y4s[0][nb] = y4[0][nb];
                if (g == 2) y4s[0][nb][0] = 1.0f;
            }
            stage<1, R4S>(y4s, R4, g, j);
        }
        v4f zo[1][NB];
        fwd<1, 1>(y4, zo, Wos, SO, g, j);
        if (g == 0) {
            const float bo = sw[oBo];
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
                const float p = sigmoidf_ref(zo[0][nb][0] + bo);
                sP[nb * 16 + j] = p;
                if (PHASE == kNcfScores) a.scores[tile * kR + nb * 16 + j] = ue[nb] >= 0 ? p : 0.0f;
            }
        }
#endif
        // list entries of the claimed slots (the atomics have returned by now)
        if (kBackward && lane < kR) {
            const int64_t ex = tile * kR + lane;
            if (lu >= 0 && lu < kNcfCap) store_entry(a.row_list + (int64_t)ru * kNcfCap + lu, (int)ex, 1.0f);
            if (li >= 0 && li < kNcfCap)
                store_entry(a.row_list + (a.num_users + ri) * kNcfCap + li, (int)ex, 1.0f);
            sLu[lane] = lu;
            sLi[lane] = li;
        }
        // the next tile's record, in flight during this tile's loss and backward
        if (lane < kR) nxt = fetch_row(tile + waves_total, lane);
        wave_sync();
        WS(4);
        if (PHASE == kNcfScores) continue;
        // ---- loss: one lane per row, then the positives' lanes sum their column in q order
        // (the tile kernel's arithmetic and summation order) ----
        float *sT = reinterpret_cast<float *>(sK);   // row -> the positive's dL/dp term (sK is dead here)
        if (lane < kR) {
            const int r = lane, q = r / tc, cl = r % tc;
            const bool v = q < NP && sU[r] >= 0, vp = sU[cl] >= 0;
            const float p = sP[r], pp = sP[cl];
            float dpr = 0.0f, ta = 0.0f, tb = 0.0f, t0 = 0.0f;
            if (PHASE == kNcfGivenDp) {
                if (v) dpr = a.dp_in[tile * kR + r];
            } else if (a.loss == RG_LOSS_POINTWISE) {
                if (v && q == 0) {
                    ta = -fmaxf(logf(p), -100.0f);
                    dpr = ((p - 1.0f) / fmaxf((1.0f - p) * p, 1e-12f)) / a.n_a;
                } else if (v) {
                    tb = -fmaxf(logf(1.0f - p), -100.0f);
                    dpr = (p / fmaxf((1.0f - p) * p, 1e-12f)) / a.n_b;
                }
            } else if (v && vp && q > 0) {   // bpr / hinge on the neg.view(n, B) pairing
                const float gg = 1.0f / a.n_a;
                if (a.loss == RG_LOSS_BPR) {
                    const float sg = sigmoidf_ref(pp - p);
                    ta = 1.0f - sg;
                    const float dx = (-gg) * (1.0f - sg) * sg;
                    t0 = dx;
                    dpr = -dx;
                } else {
                    const float xx = (p - pp) + 1.0f;
                    ta = fmaxf(xx, 0.0f);
                    const float dx = xx >= 0.0f ? gg : 0.0f;
                    t0 = -dx;
                    dpr = dx;
                }
            }
            sLa[r] = ta;
            sLb[r] = tb;
            sT[r] = t0;
            wave_sync();
            if (q == 0 && PHASE != kNcfGivenDp) {   // the positive: its column's sums in q order
                constexpr int QM = RG_MF_MAX_NEG + 1;
                float la = ta, lb = 0.0f;
                float ca[QM], cb[QM], c0[QM];
                bool cv[QM];
#pragma unroll
                for (int k = 1; k < QM; ++k) {
                    const int rr = min(k * tc + cl, kR - 1);
                    ca[k] = sLa[rr];
                    cb[k] = sLb[rr];
                    c0[k] = sT[rr];
                    cv[k] = k < NP && sU[rr] >= 0;
                }
                if (a.loss == RG_LOSS_POINTWISE) {
#pragma unroll
                    for (int k = 1; k < QM; ++k)
                        if (cv[k]) lb += cb[k];
                } else {
                    la = 0.0f;
                    float d0 = 0.0f;
#pragma unroll
                    for (int k = 1; k < QM; ++k)
                        if (cv[k] && v) { la += ca[k]; d0 += c0[k]; }
                    dpr = d0;
                }
                wave_sync();
                sLa[cl] = la;   // column totals (row cl is this lane's own row)
                sLb[cl] = lb;
            }
            sDz[r] = v ? (dpr * (1.0f - p)) * p : 0.0f;
        }
        wave_sync();
        if (lane == 0) {   // column order, as the one-thread loop summed them
            constexpr int CM = kR / 2;   // columns per tile at most (n >= 1)
            float va[CM], vb[CM];
#pragma unroll
            for (int cl = 0; cl < CM; ++cl) {
                va[cl] = cl < tc ? sLa[cl] : 0.0f;
                vb[cl] = cl < tc ? sLb[cl] : 0.0f;
            }
            float la = 0.0f, lb = 0.0f;
#pragma unroll
            for (int cl = 0; cl < CM; ++cl)
                if (cl < tc) { la += va[cl]; lb += vb[cl]; }
            a.loss_partials[2 * tile] = la;
            a.loss_partials[2 * tile + 1] = lb;
        }
        if (PHASE == kNcfLossOnly) { wave_sync(); continue; }
        // the next tile's rows (its record arrived during the loss): one load per 128-B line of
        // each user / item row, so its gather at the next tile's start hits L2
        if (lane < kR && nxt.valid) {
            const float *pu = a.user_w + (int64_t)nxt.pr.x * 64, *pi = a.item_w + (int64_t)nxt.pr.y * 64;
            warm += (pu[0] + pu[32]) + (pi[0] + pi[32]);
        }
        WS(5);
        // ---- backward, one example block at a time (lane j: example 16 nb + j).  Every weight-
        // gradient accumulator still takes the tile's examples in row order (block 0's k-steps,
        // then block 1's, ...), so the sums are those of one pass over the tile ----
        auto mult4 = [&](v4f &d, const v4f &y, uint64_t kw, int bit) {
#pragma unroll
            for (int r = 0; r < 4; ++r) d[r] = d[r] * mult(y[r], (kw >> (bit + r)) & 1, training);
        };
        WS(6);
#pragma unroll 1
        for (int nb = 0; nb < NB; ++nb) {
            const int row = nb * 16 + j, s0 = 4 * nb;
            // X0 of the block with examples on the k axis for dW1 (lane (g, x): X0[4 s + g][16 t + x],
            // user columns t < 4, item columns t >= 4), re-read from L2 now for use after three
            // layers; rows that are not valid pairs read row 0 (their delta is 0)
            float xn[4][8];
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                const int e = 4 * (s0 + s2) + g, u = sU[e], i = sI[e];
                const float *pu = a.user_w + (int64_t)(u >= 0 ? u : 0) * 64 + j;
                const float *pi = a.item_w + (int64_t)(u >= 0 ? i : 0) * 64 + j;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    xn[s2][t] = pu[16 * t];
                    xn[s2][4 + t] = pi[16 * t];
                }
            }
            const float dzb = sDz[row];
            // output layer: [dW_out | db_out] += sum_e [A_4 | 1][e] dz[e]; delta_4 = (dz w_out) m_4
            // (A_4's feature 8 is the ones column: its output weight is 0, so its delta is too)
#pragma unroll
            for (int s = s0; s < s0 + 4; ++s) gO = mfma(R4[(4 * s + g) * R4S + j], sDz[4 * s + g], gO);
            v4f y4b[1], d4b[1], y3b[1], d3b[1];
            unstage1<1, R4S>(y4b, R4, row, g);
#pragma unroll
            for (int r = 0; r < 4; ++r)
                d4b[0][r] = (dzb * Wos[4 * g + r]) * mult(y4b[0][r], (kb2 >> (36 + kbit(0, nb, r))) & 1, training);
            unstage1<1, R3S>(y3b, R3, row, g);                  // A_3 back from its staged rows
            bwd1<1, 1>(d4b, d3b, W4s, S4, g, j);
            mult4(d3b[0], y3b[0], kb2, 24 + kbit(0, nb, 0));
            wave_sync();                                        // A_4 reads done before delta_4 lands there
            stage1<1, R4S>(d4b, R4, row, g);
            wave_sync();
            dw1b<1, 1, R4S, R3S>(gW4, bB4, R4, R3, g, j, s0);   // dW4 += delta4^T A_3
            v4f y2b[2], d2b[2];
            unstage1<2, R2S>(y2b, R2, row, g);
            bwd1<2, 1>(d3b, d2b, W3s, S3, g, j);
#pragma unroll
            for (int t = 0; t < 2; ++t) mult4(d2b[t], y2b[t], kb2, kbit(t, nb, 0));
            wave_sync();                                        // A_3 reads done before delta_3 lands there
            stage1<1, R3S>(d3b, R3, row, g);
            wave_sync();
            dw1b<1, 2, R3S, R2S>(gW3, bB3, R3, R2, g, j, s0);
            v4f y1b[4], d1b[4];
            unstage1<4, R1S>(y1b, R1, row, g);
            bwd1<4, 2>(d2b, d1b, W2s, S2, g, j);
#pragma unroll
            for (int t = 0; t < 4; ++t) mult4(d1b[t], y1b[t], kb1, kbit(t, nb, 0));
            wave_sync();
            stage1<2, R2S>(d2b, R2, row, g);
            wave_sync();
            WSB(7);
            dw1b<2, 4, R2S, R1S>(gW2, bB2, R2, R1, g, j, s0);
            WSB(8);
            wave_sync();
            stage1<4, R1S>(d1b, R1, row, g);
            wave_sync();
            WSB(9);
            // dW1 += delta1^T X0 (the block's k-steps), db1 alongside
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                float av[4];
#pragma unroll
                for (int to = 0; to < 4; ++to) av[to] = R1[at<R1S>(4 * (s0 + s2) + g, 16 * to + j)];
#pragma unroll
                for (int to = 0; to < 4; ++to) {
#pragma unroll
                    for (int t = 0; t < 8; ++t) gW1[to][t] = mfma(av[to], xn[s2][t], gW1[to][t]);
                    bB1[to] += av[to];
                }
            }
            WSB(10);
            // dX0^T = W1^T delta1^T: the block's input gradient rows, in four quarters of 32
            // columns (user 0-31, 32-63, item 0-31, 32-63), each stored at once, overflow rows
            // (lists full) in fixed point
            const int lu = sLu[row], li = sLi[row], ur = sU[row], ir = sI[row];
            float *ctile = a.contrib + (int64_t)__builtin_amdgcn_readfirstlane((int)tile) * (kR * 128);
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const int hh = qq >> 1, c0 = 32 * (qq & 1);   // table half, first column in the row
                v4f dx[2];
                bwd1<2, 4>(d1b, dx, W1s + 32 * qq, S1, g, j);
#pragma unroll
                for (int t = 0; t < 2; ++t)
                    // write-through (16-B sc1): these 25 MB of rows leave the XCD's L2 as they are
                    // written instead of waiting dirty for the kernel's end-of-kernel write-back
                    // (measured: ncf_wave_kernel 63.7-64.1 -> 62.5-63.0 us, profiles/r6/ncf/); the
                    // resource starts at this wave's tile (a wave-uniform base, small offsets)
                    __builtin_amdgcn_raw_buffer_store_b128(
                        dx[t], __builtin_amdgcn_make_buffer_rsrc(ctile, 0, 0xffffffff, 0x00020000),
                        (row * 128 + 32 * qq + 16 * t + 4 * g) * 4, 0, kSc1);
                if ((hh == 0 ? lu : li) >= kNcfCap) {
                    const int64_t orow = hh == 0 ? (int64_t)ur : a.num_users + ir;
#pragma unroll
                    for (int t = 0; t < 2; ++t)
#pragma unroll
                        for (int r = 0; r < 4; ++r) fix_add(a.hot_grad + orow * 64 + c0 + 16 * t + 4 * g + r, dx[t][r]);
                }
            }
            WSB(11);
        }
        WS(12);
        if (a.pos_slot != nullptr) {
            // planned positives: lane c runs the segments of equal plan slots in column order (the
            // same sums as a per-segment loop) over the positives' item halves just stored
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   // this wave's contrib stores visible
            float acc = 0.0f;
            int prev = -2;
            for (int cl = 0; cl < tc; ++cl) {
                const int slot = sPs[cl];
                if (slot != prev) acc = 0.0f;
                acc += a.contrib[(tile * kR + cl) * (int64_t)128 + 64 + lane];
                prev = slot;
                if (slot >= 0 && (cl + 1 == tc || sPs[cl + 1] != slot)) a.part_row[(int64_t)slot * 64 + lane] = acc;
            }
        }
        wave_sync();
        WS(13);
    }
    if constexpr (!kBackward) return;
    // ---- the workgroup's weight-gradient partial: ((w0 + w2) + (w1 + w3)) -- waves 0 and 1 store
    // into two LDS images, then waves 2 and 3 add into them (each address has one adder, so the
    // sums are deterministic), and the global write adds the two images ----
    float *red = lds;   // every wave is past its tiles (barrier below): weights and scratch are free
    static_assert(2 * P <= kLdsFloats, "two gradient images");
    // the hidden biases: the four lane groups' column sums, (g0 + g1) + (g2 + g3) on every lane
    auto gsum = [](float v) {
        v += __shfl_xor(v, 16);
        return v + __shfl_xor(v, 32);
    };
    float sB1[4], sB2[2];
#pragma unroll
    for (int to = 0; to < 4; ++to) sB1[to] = gsum(bB1[to]);
#pragma unroll
    for (int to = 0; to < 2; ++to) sB2[to] = gsum(bB2[to]);
    const float sB3 = gsum(bB3[0]), sB4 = gsum(bB4[0]);
    auto each_bias = [&](auto &&f) {   // lanes of group 0, one per feature
#pragma unroll
        for (int to = 0; to < 4; ++to) f(S64::w_off(0) + 64 * 128 + 16 * to + j, sB1[to], g == 0);
#pragma unroll
        for (int to = 0; to < 2; ++to) f(S64::w_off(1) + 32 * 64 + 16 * to + j, sB2[to], g == 0);
        f(S64::w_off(2) + 16 * 32 + j, sB3, g == 0);
        f(S64::w_off(3) + 8 * 16 + min(j, 7), sB4, g == 0 && j < 8);
    };
    WSK(1);   // tiles done
    __syncthreads();
    WSK(2);   // the workgroup's last wave is done
    for (int round = 0; round < 2; ++round) {
        if ((wave >> 1) == round) {
            float *img = red + (wave & 1) * P;
            // this lane's values and their flat indices, in a fixed order
            auto each = [&](auto &&f) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int orow = 4 * g + r;   // row of a 16x16 tile held in register r
#pragma unroll
                    for (int to = 0; to < 4; ++to)
#pragma unroll
                        for (int t = 0; t < 8; ++t) f(S64::w_off(0) + (16 * to + orow) * 128 + 16 * t + j, gW1[to][t][r], true);
#pragma unroll
                    for (int to = 0; to < 2; ++to)
#pragma unroll
                        for (int t = 0; t < 4; ++t) f(S64::w_off(1) + (16 * to + orow) * 64 + 16 * t + j, gW2[to][t][r], true);
#pragma unroll
                    for (int t = 0; t < 2; ++t) f(S64::w_off(2) + orow * 32 + 16 * t + j, gW3[0][t][r], true);
                    f(S64::w_off(3) + min(orow, 7) * 16 + j, gW4[0][0][r], orow < 8);
                    f(WO + min(orow, 8), gO[r], j == 0 && orow <= 8);   // w_out (8), then b_out
                }
            };
            if (round == 0) {
                each([&](int idx, float v, bool ok) { if (ok) img[idx] = v; });
                each_bias([&](int idx, float v, bool ok) { if (ok) img[idx] = v; });
            } else {
                each_bias([&](int idx, float v, bool ok) { if (ok) img[idx] = img[idx] + v; });   // one adder per image and address: read a group, add, store (a round trip per group)
                auto group = [&](auto nv, auto &&idx_of, auto &&val_of, auto &&ok_of) {
                    constexpr int N = decltype(nv)::value;
                    float cur[N];
#pragma unroll
                    for (int q = 0; q < N; ++q) cur[q] = ok_of(q) ? img[idx_of(q)] : 0.0f;
#pragma unroll
                    for (int q = 0; q < N; ++q)
                        if (ok_of(q)) img[idx_of(q)] = cur[q] + val_of(q);
                };
                using I32 = std::integral_constant<int, 32>;
                using I16 = std::integral_constant<int, 16>;
                using I8 = std::integral_constant<int, 8>;
                using I4 = std::integral_constant<int, 4>;
                auto yes = [](int) { return true; };
#pragma unroll
                for (int to = 0; to < 4; ++to)   // W1: (to, t, r)
                    group(I32{}, [&](int q) { return S64::w_off(0) + (16 * to + 4 * g + (q & 3)) * 128 + 16 * (q >> 2) + j; },
                          [&](int q) { return gW1[to][q >> 2][q & 3]; }, yes);
#pragma unroll
                for (int to = 0; to < 2; ++to)   // W2
                    group(I16{}, [&](int q) { return S64::w_off(1) + (16 * to + 4 * g + (q & 3)) * 64 + 16 * (q >> 2) + j; },
                          [&](int q) { return gW2[to][q >> 2][q & 3]; }, yes);
                group(I8{}, [&](int q) { return S64::w_off(2) + (4 * g + (q & 3)) * 32 + 16 * (q >> 2) + j; },
                      [&](int q) { return gW3[0][q >> 2][q & 3]; }, yes);
                group(I4{}, [&](int q) { return S64::w_off(3) + min(4 * g + q, 7) * 16 + j; },
                      [&](int q) { return gW4[0][0][q]; }, [&](int q) { return 4 * g + q < 8; });
                if (j == 0)   // the output row
                    group(I4{}, [&](int q) { return WO + min(4 * g + q, 8); },
                          [&](int q) { return gO[q]; }, [&](int q) { return 4 * g + q <= 8; });
            }
        }
        __syncthreads();
        WSK(3 + round);   // round 0 stored, round 1 added
    }
    for (int e = tid; e < P; e += kThreads) a.wpart[(int64_t)blockIdx.x * P + e] = red[e] + red[P + e];
    WSK(5);   // kernel exit
}

static bool ncf_use_wave(int E, int M) {
#if RG_AB
    // the tile kernel for E = 64 (measured slower), A/B build only
    static const bool off = [] {
        const char *s = getenv("RG_NCF_TILE");
        return s && s[0] == '1';
    }();
#else
    constexpr bool off = false;
#endif
    return E == 64 && M == 0 && !off;
}

template <int PHASE>
static int ncf_wave_launch(NcfArgs &a, hipStream_t s, int blocks) {
    const size_t lds = (size_t)ncfw::kLdsFloats * sizeof(float);
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void *>(ncf_wave_kernel<PHASE>),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
    if (!attr) return fail_arg("ncf_wave_kernel: cannot reserve LDS");
    hipLaunchKernelGGL((ncf_wave_kernel<PHASE>), dim3(blocks), dim3(ncfw::kThreads), lds, s, a);
    return check_launch("rg_ncf_pairs");
}

template <int PHASE>
struct NcfLaunchF {
    NcfArgs *a;
    hipStream_t s;
    int blocks;
    template <int E>
    int run() {
        using S = NcfShape<E>;
        const int need = S::lds_neumf(a->mf_dim);
        if (need > kLdsMax) return fail_arg("rg_ncf_pairs: NeuMF mf_dim too large for this embedding_dim (LDS)");
        const size_t lds = (size_t)need * sizeof(float);
        static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void *>(ncf_pairs_kernel<E, PHASE>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     kLdsMax * (int)sizeof(float)) == hipSuccess;
        if (!attr) return fail_arg("ncf_pairs_kernel: cannot reserve LDS");
        hipLaunchKernelGGL((ncf_pairs_kernel<E, PHASE>), dim3(blocks), dim3(ncf_threads<E>()), lds, s, *a);
        return check_launch("rg_ncf_pairs");
    }
    int operator()(int E) {
        switch (E) {
            case 8: return run<8>();
            case 16: return run<16>();
            case 32: return run<32>();
            case 64: return run<64>();
            default: return fail_arg("NCF embedding_dim must be 8, 16, 32 or 64");
        }
    }
};

int ncf_mlp_len(int E) {
    switch (E) {
        case 8: return NcfShape<8>::P;
        case 16: return NcfShape<16>::P;
        case 32: return NcfShape<32>::P;
        case 64: return NcfShape<64>::P;
        default: return -1;
    }
}

int ncf_mask_units(int E) {
    switch (E) {
        case 8: return NcfShape<8>::mask_units();
        case 16: return NcfShape<16>::mask_units();
        case 32: return NcfShape<32>::mask_units();
        case 64: return NcfShape<64>::mask_units();
        default: return -1;
    }
}

}  // namespace rg

using namespace rg;

extern "C" int64_t rg_ncf_mlp_len(int32_t dim) { return ncf_mlp_len(dim); }
extern "C" int64_t rg_neumf_param_len(int32_t dim, int32_t mf_dim) {
    const int p = ncf_mlp_len(dim);
    return p < 0 || mf_dim < 1 || mf_dim > RG_NEUMF_MAX_MF_DIM ? -1 : p + mf_dim;
}
static int64_t ncf_param_len(const rg_ncf_model_t *m) {
    return m->mf_dim == 0 ? ncf_mlp_len(m->dim) : rg_neumf_param_len(m->dim, m->mf_dim);
}
extern "C" int64_t rg_ncf_mask_units(int32_t dim) { return ncf_mask_units(dim); }
// rows per tile: RG_NCF_WAVE_ROWS for the wave kernel (E = 64 MLP; 48 in the product build --
// 8 columns of 1 + 5 rows, one tile per wave at B = 8192), 32 for the tile kernel (the other
// towers, NeuMF)
extern "C" int64_t rg_ncf_rows_per_tile(int32_t dim, int32_t mf_dim) {
    if (ncf_mlp_len(dim) < 0 || mf_dim < 0 || mf_dim > RG_NEUMF_MAX_MF_DIM) return -1;
    return ncf_use_wave(dim, mf_dim) ? ncfw::kR : kRows;
}
extern "C" int64_t rg_ncf_cols_per_tile(int32_t n_neg, int32_t dim, int32_t mf_dim) {
    const int64_t R = rg_ncf_rows_per_tile(dim, mf_dim);
    return R < 0 || n_neg < 0 || n_neg >= R ? -1 : R / (n_neg + 1);
}
extern "C" int64_t rg_ncf_tiles(int64_t cols, int32_t n_neg, int32_t dim, int32_t mf_dim) {
    const int64_t tc = rg_ncf_cols_per_tile(n_neg, dim, mf_dim);
    return tc <= 0 ? -1 : (cols + tc - 1) / tc;
}
// the scores / dp layout of an adaptive-hinge launch: the work's tile_rows (the model's
// rg_ncf_rows_per_tile, checked by rg_ncf_pairs)
static int ncf_geometry(const rg_ncf_work_t *nw, const rg_mf_batch_t *b, int &TR, int &tc, int64_t &tiles) {
    TR = nw->tile_rows;
    if (TR != kRows && TR != ncfw::kR) return fail_arg("rg_ncf: ncf_work.tile_rows must be rg_ncf_rows_per_tile(dim, mf_dim)");
    if (b->n_neg < 1 || b->n_neg >= TR) return fail_arg("rg_ncf: n_neg out of range");
    tc = TR / (b->n_neg + 1);
    tiles = (b->cols + tc - 1) / tc;
    return RG_OK;
}
// workgroups resident per CU by LDS (at most 4): the E = 64 MLP takes a CU's LDS alone,
// the small towers (and NeuMF's) leave room for several tiles in flight per CU, which is
// what hides their gather / barrier latency
static int ncf_lds_floats(int E, int M) {
    switch (E) {
        case 8: return NcfShape<8>::lds_neumf(M);
        case 16: return NcfShape<16>::lds_neumf(M);
        case 32: return NcfShape<32>::lds_neumf(M);
        case 64: return NcfShape<64>::lds_neumf(M);
        default: return -1;
    }
}

extern "C" int64_t rg_ncf_blocks(int64_t cols, int32_t n_neg, int32_t dim, int32_t mf_dim) {
    const int64_t t = rg_ncf_tiles(cols, n_neg, dim, mf_dim);
    const int lds = ncf_lds_floats(dim, mf_dim);
    if (t <= 0 || lds <= 0 || lds > kLdsMax || mf_dim < 0 || mf_dim > RG_NEUMF_MAX_MF_DIM) return -1;
    if (ncf_use_wave(dim, mf_dim)) {   // one wave per tile, 4 waves per workgroup, one workgroup per CU
        const int64_t w = (t + ncfw::kWaves - 1) / ncfw::kWaves;
        return w < 256 ? w : 256;
    }
    int per_cu = kLdsMax / lds;
    if (per_cu > 4) per_cu = 4;
    const int64_t cap = 256 * (int64_t)per_cu;
    return t < cap ? t : cap;
}

extern "C" int rg_ncf_pairs(void *stream, const rg_ncf_model_t *m, const rg_mf_batch_t *b, rg_mf_work_t *w,
                            rg_ncf_work_t *nw, int32_t phase) {
    if (!m || !b || !w || !nw) return fail_arg("rg_ncf_pairs: null argument");
    if (ncf_mlp_len(m->dim) < 0) return fail_arg("rg_ncf_pairs: embedding_dim must be 8, 16, 32 or 64");
    if (b->n_neg < 1 || b->n_neg > RG_MF_MAX_NEG) return fail_arg("rg_ncf_pairs: n_neg out of range");
    if (b->loss < RG_LOSS_POINTWISE || b->loss > RG_LOSS_ADAPTIVE_HINGE)   // no positives-only NCF step
        return fail_arg("rg_ncf_pairs: loss must be pointwise, bpr, hinge or adaptive hinge");
    if (!b->pairs || !m->user_w || !m->item_w || !m->mlp) return fail_arg("rg_ncf_pairs: null tables / pairs");
    if (b->n_pos > b->cols) return fail_arg("rg_ncf_pairs: n_pos > cols");
    if (phase != kNcfScores && phase != kNcfLossOnly && (!w->row_count || !w->row_list || !w->hot_grad ||
                                                         !w->loss_partials || !nw->contrib || !nw->mlp_partials))
        return fail_arg("rg_ncf_pairs: null scratch");
    if (phase == kNcfLossOnly && !w->loss_partials) return fail_arg("rg_ncf_pairs: loss needs partials");
    if (phase == kNcfScores && !nw->scores) return fail_arg("rg_ncf_pairs: scores buffer needed");
    if (phase == kNcfGivenDp && !nw->dp) return fail_arg("rg_ncf_pairs: dp buffer needed");
    if ((phase == kNcfFused || phase == kNcfLossOnly) && b->loss == RG_LOSS_ADAPTIVE_HINGE)
        return fail_arg("rg_ncf_pairs: adaptive hinge runs as scores -> rg_ncf_adapt_dp -> given-dp");
    if (nw->training && (nw->mask_pos == nullptr) != (nw->mask_neg == nullptr))
        return fail_arg("rg_ncf_pairs: give both dropout mask arrays or neither");
    if (w->plan_pos_slot && !w->part_row) return fail_arg("rg_ncf_pairs: plan needs part_row");
    if (ncf_param_len(m) < 0) return fail_arg("rg_ncf_pairs: mf_dim out of range");
    if (m->mf_dim > 0) {
        if (!m->mf_user_w || !m->mf_item_w) return fail_arg("rg_ncf_pairs: NeuMF needs the GMF tables");
        if (phase != kNcfScores && phase != kNcfLossOnly && (!nw->mf_contrib || !nw->mf_hot_grad))
            return fail_arg("rg_ncf_pairs: NeuMF needs mf_contrib / mf_hot_grad");
        if (phase != kNcfScores && phase != kNcfLossOnly && w->plan_pos_slot && !nw->mf_part_row)
            return fail_arg("rg_ncf_pairs: NeuMF plan needs mf_part_row");
    }
    NcfArgs a{};
    a.user_w = m->user_w; a.item_w = m->item_w; a.mlp = m->mlp;
    a.num_users = m->num_users; a.num_items = m->num_items;
    a.pairs = reinterpret_cast<const int2 *>(b->pairs);
    a.n_pos = b->n_pos; a.cols = b->cols; a.global_cols = b->global_cols; a.col_offset = b->col_offset;
    a.n_neg = b->n_neg; a.loss = b->loss;
    if (nw->tile_rows != rg_ncf_rows_per_tile(m->dim, m->mf_dim))
        return fail_arg("rg_ncf_pairs: ncf_work.tile_rows must be rg_ncf_rows_per_tile(dim, mf_dim)");
    a.tc = (int)rg_ncf_cols_per_tile(b->n_neg, m->dim, m->mf_dim);
    a.tiles = rg_ncf_tiles(b->cols, b->n_neg, m->dim, m->mf_dim);
    if (a.tiles >= ((int64_t)1 << 31)) return fail_arg("rg_ncf_pairs: more than 2^31 tiles");
    const int64_t negc = b->neg_cols > 0 ? b->neg_cols : b->global_cols;
    switch (b->loss) {
        case RG_LOSS_POINTWISE: a.n_a = (float)b->global_pos; a.n_b = (float)((int64_t)b->n_neg * negc); break;
        case RG_LOSS_BPR:
        case RG_LOSS_HINGE: a.n_a = (float)((int64_t)b->n_neg * b->global_pos); a.n_b = 1.0f; break;
        default: a.n_a = (float)b->global_pos; a.n_b = 1.0f;
    }
    a.perm = w->plan_perm; a.pos_slot = w->plan_pos_slot;
    a.row_count = w->row_count; a.row_list = reinterpret_cast<int2 *>(w->row_list);
    a.hot_grad = reinterpret_cast<long long *>(w->hot_grad); a.part_row = w->part_row;
    a.loss_partials = w->loss_partials;
    a.contrib = nw->contrib; a.wpart = nw->mlp_partials; a.scores = nw->scores; a.dp_in = nw->dp;
    a.mask_pos = nw->mask_pos; a.mask_neg = nw->mask_neg; a.seed = nw->seed; a.training = nw->training;
    a.mf_dim = m->mf_dim; a.mf_user_w = m->mf_user_w; a.mf_item_w = m->mf_item_w;
    a.mf_contrib = nw->mf_contrib; a.mf_hot_grad = reinterpret_cast<long long *>(nw->mf_hot_grad);
    a.mf_part_row = nw->mf_part_row;
    const int blocks = (int)rg_ncf_blocks(b->cols, b->n_neg, m->dim, m->mf_dim);
    if (blocks <= 0) return fail_arg("rg_ncf_pairs: no launch shape for this dim / mf_dim");
    if (ncf_use_wave(m->dim, m->mf_dim)) {
        hipStream_t st = (hipStream_t)stream;
        if (phase == kNcfFused) return ncf_wave_launch<kNcfFused>(a, st, blocks);
        if (phase == kNcfScores) return ncf_wave_launch<kNcfScores>(a, st, blocks);
        if (phase == kNcfGivenDp) return ncf_wave_launch<kNcfGivenDp>(a, st, blocks);
        if (phase == kNcfLossOnly) return ncf_wave_launch<kNcfLossOnly>(a, st, blocks);
        return fail_arg("rg_ncf_pairs: bad phase");
    }
    if (phase == kNcfFused) { NcfLaunchF<kNcfFused> f{&a, (hipStream_t)stream, blocks}; return f(m->dim); }
    if (phase == kNcfScores) { NcfLaunchF<kNcfScores> f{&a, (hipStream_t)stream, blocks}; return f(m->dim); }
    if (phase == kNcfGivenDp) { NcfLaunchF<kNcfGivenDp> f{&a, (hipStream_t)stream, blocks}; return f(m->dim); }
    if (phase == kNcfLossOnly) { NcfLaunchF<kNcfLossOnly> f{&a, (hipStream_t)stream, blocks}; return f(m->dim); }
    return fail_arg("rg_ncf_pairs: bad phase");
}

extern "C" int rg_ncf_adapt_dp(void *stream, const rg_mf_batch_t *b, rg_ncf_work_t *nw, float *loss_partials) {
    if (!b || !nw || !nw->scores || !nw->dp || !loss_partials) return fail_arg("rg_ncf_adapt_dp: null argument");
    int TR = 0, tc = 0;
    int64_t tiles = 0;
    if (ncf_geometry(nw, b, TR, tc, tiles)) return RG_E_ARG;
    hipLaunchKernelGGL(ncf_adapt_dp_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, nw->scores, nw->dp,
                       tiles * TR, TR, tc, b->n_neg + 1, b->n_pos, b->cols, (float)b->global_pos, loss_partials);
    return check_launch("rg_ncf_adapt_dp");
}

// ---- adaptive hinge over several ranks (each holds its column slice of ONE global draw) ----
// The global maximum negative (torch.max over the flat draw: the largest score, the first
// draw index j = k * global_cols + column on ties) is found in three small launches around
// two float SUM all-reduces of the caller: each rank's (score, j) goes into its own slot of a
// zeroed [world][4] buffer (one writer per slot, x + 0 = x: the sum is an all-gather), every
// rank picks the same winner, and the active-positive count is summed before the winner's
// rank sets its row's dp (spotlight/losses.py:133-172, implicit.py:194-199).
__device__ __forceinline__ bool adapt_better(float s, int64_t j, float bs, int64_t bj) {
    return s > bs || (s == bs && j < bj);
}

__device__ __forceinline__ int adapt_winner(const float *slots, int world) {
    int w = 0;
    float bs = slots[0];
    int64_t bj = ((int64_t)slots[1] << 16) | (int64_t)slots[2];
    for (int r = 1; r < world; ++r) {
        const float sc = slots[4 * r];
        const int64_t j = ((int64_t)slots[4 * r + 1] << 16) | (int64_t)slots[4 * r + 2];
        if (adapt_better(sc, j, bs, bj)) { w = r; bs = sc; bj = j; }
    }
    return w;
}

__global__ __launch_bounds__(256) void ncf_adapt_local_kernel(const float *scores, int64_t rows, int TR, int tc, int NP,
                                                             int64_t cols, const int32_t *perm, int64_t global_cols,
                                                             int64_t col_offset, float *slots, int rank, int world,
                                                             int32_t *local_row) {
    __shared__ float ss[256];
    __shared__ int64_t sj[256], sr[256];
    const int tid = threadIdx.x;
    float best = -1.0f;
    int64_t bj = INT64_MAX, br = -1;
    for (int64_t r = tid; r < rows; r += 256) {
        const int64_t tile = r / TR, rr = r % TR;
        const int q = (int)(rr / tc);
        const int64_t s = tile * tc + rr % tc;
        if (q >= 1 && q < NP && s < cols) {
            const int64_t col = perm ? (int64_t)perm[s] : s;
            const int64_t j = (int64_t)(q - 1) * global_cols + col_offset + col;
            if (adapt_better(scores[r], j, best, bj)) { best = scores[r]; bj = j; br = r; }
        }
    }
    ss[tid] = best; sj[tid] = bj; sr[tid] = br;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (tid < w && adapt_better(ss[tid + w], sj[tid + w], ss[tid], sj[tid])) {
            ss[tid] = ss[tid + w]; sj[tid] = sj[tid + w]; sr[tid] = sr[tid + w];
        }
        __syncthreads();
    }
    if (tid == 0) {
        for (int i = 0; i < 4 * world; ++i) slots[i] = 0.0f;
        const int64_t j = sj[0] == INT64_MAX ? 0 : sj[0];
        slots[4 * rank] = ss[0];
        slots[4 * rank + 1] = (float)(j >> 16);
        slots[4 * rank + 2] = (float)(j & 0xffff);
        local_row[0] = (int32_t)sr[0];
    }
}

__global__ __launch_bounds__(256) void ncf_adapt_global_kernel(const float *scores, float *dp, int64_t rows, int TR, int tc,
                                                              int64_t n_pos_cols, float n_a, const float *slots,
                                                              int world, float *count, float *loss_partial) {
    __shared__ float scnt[256], sloss[256];
    const int tid = threadIdx.x;
    const float mx = slots[4 * adapt_winner(slots, world)];
    float cnt = 0.0f, ls = 0.0f;
    for (int64_t r = tid; r < rows; r += 256) {
        const int64_t tile = r / TR, rr = r % TR;
        const int64_t s = tile * tc + rr % tc;
        dp[r] = 0.0f;
        if (rr < (int64_t)tc && s < n_pos_cols) {
            const float x = (mx - scores[r]) + 1.0f;
            ls += fmaxf(x, 0.0f);
            if (x >= 0.0f) { dp[r] = -(1.0f / n_a); cnt += 1.0f; }
        }
    }
    scnt[tid] = cnt;
    sloss[tid] = ls;
    __syncthreads();
    if (tid == 0) {
        float c = 0.0f, l = 0.0f;
        for (int i = 0; i < 256; ++i) { c += scnt[i]; l += sloss[i]; }
        count[0] = c;
        loss_partial[0] = l;
        loss_partial[1] = 0.0f;
    }
}

__global__ void ncf_adapt_winner_kernel(float *dp, const float *slots, int world, int rank, const int32_t *local_row,
                                        const float *count, float n_a) {
    if (threadIdx.x == 0 && adapt_winner(slots, world) == rank && local_row[0] >= 0)
        dp[local_row[0]] = count[0] * (1.0f / n_a);
}

extern "C" int rg_ncf_adapt_local(void *stream, const rg_mf_batch_t *b, const rg_mf_work_t *w, rg_ncf_work_t *nw,
                                  float *slots, int32_t rank, int32_t world, int32_t *local_row) {
    if (!b || !w || !nw || !nw->scores || !slots || !local_row || world < 1 || rank < 0 || rank >= world)
        return fail_arg("rg_ncf_adapt_local: bad argument");
    int TR = 0, tc = 0;
    int64_t tiles = 0;
    if (ncf_geometry(nw, b, TR, tc, tiles)) return RG_E_ARG;
    hipLaunchKernelGGL(ncf_adapt_local_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, nw->scores, tiles * TR, TR,
                       tc, b->n_neg + 1, b->cols, w->plan_perm, b->global_cols, b->col_offset, slots, rank, world,
                       local_row);
    return check_launch("rg_ncf_adapt_local");
}

extern "C" int rg_ncf_adapt_global(void *stream, const rg_mf_batch_t *b, rg_ncf_work_t *nw, const float *slots,
                                   int32_t world, float *count, float *loss_partials) {
    if (!b || !nw || !nw->scores || !nw->dp || !slots || !count || !loss_partials || world < 1)
        return fail_arg("rg_ncf_adapt_global: bad argument");
    int TR = 0, tc = 0;
    int64_t tiles = 0;
    if (ncf_geometry(nw, b, TR, tc, tiles)) return RG_E_ARG;
    hipLaunchKernelGGL(ncf_adapt_global_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, nw->scores, nw->dp,
                       tiles * TR, TR, tc, b->n_pos, (float)b->global_pos, slots, world, count, loss_partials);
    return check_launch("rg_ncf_adapt_global");
}

extern "C" int rg_ncf_adapt_winner(void *stream, const rg_mf_batch_t *b, rg_ncf_work_t *nw, const float *slots,
                                   int32_t world, int32_t rank, const int32_t *local_row, const float *count) {
    if (!b || !nw || !nw->dp || !slots || !local_row || !count || world < 1 || rank < 0 || rank >= world)
        return fail_arg("rg_ncf_adapt_winner: bad argument");
    hipLaunchKernelGGL(ncf_adapt_winner_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, nw->dp, slots, world, rank,
                       local_row, count, (float)b->global_pos);
    return check_launch("rg_ncf_adapt_winner");
}

extern "C" int rg_ncf_update(void *stream, const rg_ncf_model_t *m, const rg_ncf_work_t *nw, int64_t nparts,
                             const rg_opt_t *opt, const float *loss_partials, const rg_mf_loss_t *loss) {
    if (!m || !nw || !opt || !nw->mlp_partials || !m->mlp) return fail_arg("rg_ncf_update: null argument");
    if (opt->kind == RG_OPT_ADAM && !m->mlp_m) return fail_arg("rg_ncf_update: Adam needs m state");
    if (opt->kind != RG_OPT_SGD && !m->mlp_v) return fail_arg("rg_ncf_update: optimizer needs v state");
    if (loss && loss->out && !loss_partials) return fail_arg("rg_ncf_update: loss needs partials");
    const int P = (int)ncf_param_len(m);
    if (P < 0) return fail_arg("rg_ncf_update: bad dim / mf_dim");
    const bool with_loss = loss && loss->out;
    hipLaunchKernelGGL(ncf_update_kernel, dim3((P + 63) / 64), dim3(kUpdWaves * 64), 0, (hipStream_t)stream, m->mlp,
                       opt->kind == RG_OPT_ADAM ? m->mlp_m : nullptr, opt->kind == RG_OPT_SGD ? nullptr : m->mlp_v,
                       nw->mlp_partials, (int)nparts, P, *opt, with_loss ? loss_partials : nullptr,
                       with_loss ? loss->n_partials : 0, with_loss ? loss->inv_a : 0.0,
                       with_loss ? loss->inv_b : 0.0, with_loss ? loss->out : nullptr, 0, nullptr);
    return check_launch("rg_ncf_update");
}

extern "C" int rg_ncf_mlp_grad(void *stream, const rg_ncf_model_t *m, const rg_ncf_work_t *nw, int64_t nparts,
                               const float *loss_partials, const rg_mf_loss_t *loss, float *grad) {
    if (!m || !nw || !nw->mlp_partials || !grad || !loss || !loss_partials)
        return fail_arg("rg_ncf_mlp_grad: null argument");
    const int P = (int)ncf_param_len(m);
    if (P < 0) return fail_arg("rg_ncf_mlp_grad: bad dim / mf_dim");
    hipLaunchKernelGGL(ncf_update_kernel, dim3((P + 63) / 64), dim3(kUpdWaves * 64), 0, (hipStream_t)stream, m->mlp,
                       nullptr, nullptr, nw->mlp_partials, (int)nparts, P, rg_opt_t{}, loss_partials,
                       loss->n_partials, loss->inv_a, loss->inv_b, loss->out, 1, grad);
    return check_launch("rg_ncf_mlp_grad");
}

extern "C" int rg_ncf_mlp_apply(void *stream, const rg_ncf_model_t *m, const float *grad, const rg_opt_t *opt,
                                float *loss_out) {
    if (!m || !grad || !opt || !m->mlp) return fail_arg("rg_ncf_mlp_apply: null argument");
    if (opt->kind == RG_OPT_ADAM && !m->mlp_m) return fail_arg("rg_ncf_mlp_apply: Adam needs m state");
    if (opt->kind != RG_OPT_SGD && !m->mlp_v) return fail_arg("rg_ncf_mlp_apply: optimizer needs v state");
    const int P = (int)ncf_param_len(m);
    if (P < 0) return fail_arg("rg_ncf_mlp_apply: bad dim / mf_dim");
    hipLaunchKernelGGL(ncf_update_kernel, dim3((P + 63) / 64), dim3(kUpdWaves * 64), 0, (hipStream_t)stream, m->mlp,
                       opt->kind == RG_OPT_ADAM ? m->mlp_m : nullptr, opt->kind == RG_OPT_SGD ? nullptr : m->mlp_v,
                       nullptr, 0, P, *opt, nullptr, 0, 0.0, 0.0, loss_out, 2, const_cast<float *>(grad));
    return check_launch("rg_ncf_mlp_apply");
}

#ifdef RG_DIAG_STAMPS
extern "C" int rg_diag_set_ncf_stamps(unsigned long long *dev_buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(rg::g_ncf_stamps), &dev_buf, sizeof(dev_buf)) == hipSuccess ? RG_OK
                                                                                                  : RG_E_LAUNCH;
}
#endif
