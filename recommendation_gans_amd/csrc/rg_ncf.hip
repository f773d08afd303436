// NCF MLP training step on gfx950 (spotlight/dnn_models/mlp.py:5-46 trained by
// implicit.py:347-364; layers [2E, E, ..., 8] -> 1 as ncf_spotlight.py:53-56).
//
// One workgroup (4 waves) walks tiles of kRows = 32 examples; a tile holds whole
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
                if (lu >= 0 && lu < kNcfCap) a.row_list[(int64_t)u * kNcfCap + lu] = make_int2((int)ex, __float_as_int(1.0f));
                if (li >= 0 && li < kNcfCap)
                    a.row_list[(a.num_users + i) * kNcfCap + li] = make_int2((int)ex, __float_as_int(1.0f));
            } else if (kBackward && u >= 0) {
                const int64_t ex = tile * kRows + r;
                lu = atomicAdd(a.row_count + u, 1);
                if (lu < kNcfCap) a.row_list[(int64_t)u * kNcfCap + lu] = make_int2((int)ex, __float_as_int(1.0f));
                if (q == 0 && a.pos_slot != nullptr) {
                    ps = a.pos_slot[s];
                } else {
                    const int64_t row = a.num_users + i;
                    li = atomicAdd(a.row_count + row, 1);
                    if (li < kNcfCap) a.row_list[row * kNcfCap + li] = make_int2((int)ex, __float_as_int(1.0f));
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
    __shared__ float red[kUpdWaves][64];
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
        for (int64_t i = lane; i < n_partials; i += 64) {
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
    const int e = blockIdx.x * 64 + lane;
    const int q = (nparts + kUpdWaves - 1) / kUpdWaves, k0 = wave * q, k1 = min(nparts, k0 + q);
    float g = 0.0f;
    if (e < P) {
        float c[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        int k = k0;
        for (; k + 4 <= k1; k += 4) {
#pragma unroll
            for (int j = 0; j < 4; ++j) c[j] += wpart[(int64_t)(k + j) * P + e];
        }
        for (; k < k1; ++k) c[0] += wpart[(int64_t)k * P + e];
        g = (c[0] + c[1]) + (c[2] + c[3]);
    }
    red[wave][lane] = g;
    __syncthreads();
    if (wave != 0 || e >= P) return;
    g = red[0][lane];
#pragma unroll
    for (int w = 1; w < kUpdWaves; ++w) g += red[w][lane];
    if (mode == 1) {
        grad[e] = g;
        return;
    }
    float mm = m ? m[e] : 0.0f, vv = v ? v[e] : 0.0f;
    const float p = opt_update(opt, mlp[e], g, mm, vv);
    mlp[e] = p;
    if (m) m[e] = mm;
    if (v) v[e] = vv;
}

// adaptive hinge from forward-only scores: dp of every row (positives: hinge
// against the max negative; the argmax negative: minus the sum over active positives)
__global__ __launch_bounds__(256) void ncf_adapt_dp_kernel(const float *scores, float *dp, int64_t rows, int tc,
                                                          int NP, int64_t n_pos_cols, int64_t cols, float n_a,
                                                          float *loss_partial) {
    __shared__ float smax[256];
    __shared__ int64_t sidx[256];
    __shared__ float scnt[256], sloss[256];
    const int tid = threadIdx.x;
    float best = -1.0f;
    int64_t bi = -1;
    for (int64_t r = tid; r < rows; r += 256) {
        const int64_t tile = r / kRows, rr = r % kRows;
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
        const int64_t tile = r / kRows, rr = r % kRows;
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
extern "C" int64_t rg_ncf_cols_per_tile(int32_t n_neg) { return n_neg < 0 || n_neg >= kRows ? -1 : kRows / (n_neg + 1); }
extern "C" int64_t rg_ncf_tiles(int64_t cols, int32_t n_neg) {
    const int64_t tc = rg_ncf_cols_per_tile(n_neg);
    return tc <= 0 ? -1 : (cols + tc - 1) / tc;
}
extern "C" int64_t rg_ncf_rows_per_tile(void) { return kRows; }
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
    const int64_t t = rg_ncf_tiles(cols, n_neg);
    const int lds = ncf_lds_floats(dim, mf_dim);
    if (t <= 0 || lds <= 0 || lds > kLdsMax || mf_dim < 0 || mf_dim > RG_NEUMF_MAX_MF_DIM) return -1;
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
    a.tc = (int)rg_ncf_cols_per_tile(b->n_neg);
    a.tiles = rg_ncf_tiles(b->cols, b->n_neg);
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
    if (phase == kNcfFused) { NcfLaunchF<kNcfFused> f{&a, (hipStream_t)stream, blocks}; return f(m->dim); }
    if (phase == kNcfScores) { NcfLaunchF<kNcfScores> f{&a, (hipStream_t)stream, blocks}; return f(m->dim); }
    if (phase == kNcfGivenDp) { NcfLaunchF<kNcfGivenDp> f{&a, (hipStream_t)stream, blocks}; return f(m->dim); }
    if (phase == kNcfLossOnly) { NcfLaunchF<kNcfLossOnly> f{&a, (hipStream_t)stream, blocks}; return f(m->dim); }
    return fail_arg("rg_ncf_pairs: bad phase");
}

extern "C" int rg_ncf_adapt_dp(void *stream, const rg_mf_batch_t *b, rg_ncf_work_t *nw, float *loss_partials) {
    if (!b || !nw || !nw->scores || !nw->dp || !loss_partials) return fail_arg("rg_ncf_adapt_dp: null argument");
    const int64_t tiles = rg_ncf_tiles(b->cols, b->n_neg);
    hipLaunchKernelGGL(ncf_adapt_dp_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, nw->scores, nw->dp,
                       tiles * kRows, (int)rg_ncf_cols_per_tile(b->n_neg), b->n_neg + 1, b->n_pos, b->cols,
                       (float)b->global_pos, loss_partials);
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

__global__ __launch_bounds__(256) void ncf_adapt_local_kernel(const float *scores, int64_t rows, int tc, int NP,
                                                             int64_t cols, const int32_t *perm, int64_t global_cols,
                                                             int64_t col_offset, float *slots, int rank, int world,
                                                             int32_t *local_row) {
    __shared__ float ss[256];
    __shared__ int64_t sj[256], sr[256];
    const int tid = threadIdx.x;
    float best = -1.0f;
    int64_t bj = INT64_MAX, br = -1;
    for (int64_t r = tid; r < rows; r += 256) {
        const int64_t tile = r / kRows, rr = r % kRows;
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

__global__ __launch_bounds__(256) void ncf_adapt_global_kernel(const float *scores, float *dp, int64_t rows, int tc,
                                                              int64_t n_pos_cols, float n_a, const float *slots,
                                                              int world, float *count, float *loss_partial) {
    __shared__ float scnt[256], sloss[256];
    const int tid = threadIdx.x;
    const float mx = slots[4 * adapt_winner(slots, world)];
    float cnt = 0.0f, ls = 0.0f;
    for (int64_t r = tid; r < rows; r += 256) {
        const int64_t tile = r / kRows, rr = r % kRows;
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
    const int64_t tiles = rg_ncf_tiles(b->cols, b->n_neg);
    hipLaunchKernelGGL(ncf_adapt_local_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, nw->scores, tiles * kRows,
                       (int)rg_ncf_cols_per_tile(b->n_neg), b->n_neg + 1, b->cols, w->plan_perm, b->global_cols,
                       b->col_offset, slots, rank, world, local_row);
    return check_launch("rg_ncf_adapt_local");
}

extern "C" int rg_ncf_adapt_global(void *stream, const rg_mf_batch_t *b, rg_ncf_work_t *nw, const float *slots,
                                   int32_t world, float *count, float *loss_partials) {
    if (!b || !nw || !nw->scores || !nw->dp || !slots || !count || !loss_partials || world < 1)
        return fail_arg("rg_ncf_adapt_global: bad argument");
    const int64_t tiles = rg_ncf_tiles(b->cols, b->n_neg);
    hipLaunchKernelGGL(ncf_adapt_global_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, nw->scores, nw->dp,
                       tiles * kRows, (int)rg_ncf_cols_per_tile(b->n_neg), b->n_pos, (float)b->global_pos, slots,
                       world, count, loss_partials);
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
