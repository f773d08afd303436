// Matrix-factorisation training step for gfx950 (MI355X).
//
// Replaces, per step (implicit.py:347-364 run_train_iteration):
//   BilinearNet.forward on B positives and n*B negatives
//       (spotlight/factorization/representations.py:62-91),
//   the loss (spotlight/losses.py: pointwise :20, bpr :59, hinge :99, adaptive :133),
//   loss.backward() -> embedding_dense_backward into dense (U,d),(I,d),(U,1),(I,1) grads,
//   optimizer.step() (spotlight/optimizers.py) over EVERY row (coupled L2).
//
// Two kernels per step, both HBM-bound:
//   mf_pairs  one "unit" = one batch column b: its positive and its n negatives
//             (flat draws k*B + b).  LPU lanes per unit, one float4 of every
//             gathered row per lane, dot products by DPP row reductions, loss
//             terms, dL/dz.  Instead of scatter-adding row gradients with float
//             atomics (memory-side, ~1.3 TB/s chip-wide) each pair appends a
//             4+4-byte {other row, dz} entry to the list of each of its two rows
//             (one returning int atomic per row); rows touched more than
//             RG_MF_LIST_CAP times spill the excess into dense overflow
//             accumulators with float atomics (Zipf-hot items only).
//   mf_apply  streams every row of both tables once: p, m, v in; the row's
//             gradient is PULLED from its list (gathering the other table's
//             pre-step row, which is why the parameter tables ping-pong) plus
//             weight_decay * p; Adam / SGD / RMSprop; p', m, v out; the list
//             counter and overflow accumulators are reset in the same pass.
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include <hip/hip_ext.h>

#include "rg_common.h"
#include "rg_mt.h"
#include "rg_owner.h"
#include "rg_mlp_update.h"

namespace rg {

constexpr int kCap = RG_MF_LIST_CAP;
#ifndef RG_MF_PULL_GROUP
#define RG_MF_PULL_GROUP 4
#endif
constexpr int kNMax = RG_MF_MAX_NEG;
constexpr int kBlock = 256;
#ifndef RG_MF_PAIR_BLOCK
#define RG_MF_PAIR_BLOCK 256
#endif
constexpr int kPairBlock = RG_MF_PAIR_BLOCK;   // threads of a pair-pass workgroup (the plan's block)

// kFused: forward + loss + lists.  kLossOnly: forward + loss (validation).
// Adaptive hinge needs the global max first: kAdaptFwd (scores + max),
// then kAdaptBwd (positives vs max + lists) or kAdaptLoss (loss only).
enum Phase : int { kFused = 0, kLossOnly = 1, kAdaptFwd = 2, kAdaptBwd = 3, kAdaptLoss = 4 };

struct PairsArgs {
    const float *user_w, *item_w, *user_b, *item_b;
    int64_t num_users;
    int32_t dim;
    const int64_t *pos_user, *pos_item;
    int64_t n_pos, cols, col_offset, global_cols;
    const uint2 *words;
    const int2 *pool;
    int64_t pool_len;
    int32_t n_neg, loss;
    float n_a, n_b;            // mean denominators (as ATen divides: grad / numel)
    int32_t *row_count;
    int2 *row_list;
    long long *hot_grad, *hot_bias_grad;     // int64 fixed point (rg_common.h fix_add)
    float *partials;
    float *scores;             // adaptive: [cols] positive scores
    unsigned long long *max_key;
    int32_t *active_count;
    const int32_t *perm;       // plan: processing position -> column (null: identity)
    const int32_t *pos_slot;   // plan: position -> partial slot of its positive's item side
    float *part_row, *part_bias;
    const int2 *pairs;         // prepared (user, item) per pair: [(1 + n) * cols], processing order
    int32_t *stamp;            // prepare: per-row serial of the last stamping prepare (null: no stamps)
    int32_t serial;
    int32_t *umark;            // prepare (lazy dense pass): umark[user] = umark_step for every pair's user
    int32_t umark_step;
    // claimed list slots (rg_mf_work_t claim_num_users): the prepare claims them in row_count and
    // stores them in the ids' bits 27-30; the pair pass reads them instead of claiming
    int32_t claimed;
    // pipelined step (mf_pipe_kernel): the prepare appends every user it claims a first slot of
    // (the users this step's pair pass reads) to hot_out, its length in *nhot_out
    int32_t *hot_out, *nhot_out;
};

// Prepared ids carry ownership flags in bit 31 when the prepare pass stamped rows:
// the first pair (any order) to stamp a row with this step's serial owns it, and
// the hot-row apply (mf_hot_kernel) updates each touched row through its owner only.
constexpr int32_t kOwnerBit = (int32_t)0x80000000;
constexpr int32_t kIdMask = 0x7fffffff;
// claimed records: slot min(slot, kCap) of the row side in bits 27-30 of its id
constexpr int kSlotShift = 27;
constexpr int32_t kClaimIdMask = (1 << kSlotShift) - 1;

// Diagnostic build only (RG_DIAG_STAMPS, librg_hip_diag.so; scripts/mf_pairs_stamps.py):
// per-wave s_memrealtime stamps at the pair pass's phase boundaries, each after a full
// vmcnt drain so it marks when that phase's data had landed.  The product library has
// no stamp code.
#ifdef RG_DIAG_STAMPS
__device__ unsigned long long *g_diag_stamps;
__device__ int g_diag_flags;   // timing only (results are wrong): bit 0 skip the list-slot atomics,
                               // bit 1 skip the list-entry stores, bit 2 skip the planned partial rows,
                               // bit 3 return right after the ids
#define RG_DIAG_FLAG(b) ((g_diag_flags >> (b)) & 1)
#else
#define RG_DIAG_FLAG(b) 0
#endif
#ifdef RG_DIAG_STAMPS
#define RG_STAMP(k)                                                                                   \
    do {                                                                                              \
        if (g_diag_stamps) {                                                                          \
            unsigned long long t_;                                                                    \
            asm volatile("s_waitcnt vmcnt(0)\n\ts_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
            if ((threadIdx.x & 63) == 0) g_diag_stamps[(blk * (kPairBlock / 64) + (threadIdx.x >> 6)) * 8 + (k)] = t_; \
        }                                                                                             \
    } while (0)
#else
#define RG_STAMP(k) \
    do {            \
    } while (0)
#endif

// rg_mf_prepare: record s of the prepared pairs (rg_common.h pair_stride): [q] for
// q = 0 (positive) and q = 1 + k (negative k), [n + 1] the positive's plan slot; one
// thread per entry, column-major so the record is written contiguously.
// With stamps, every row a pair touches (valid or not: extra rows are harmless, a
// missed one would not be) is stamped with the serial, and the first stamper owns it.
// Returns the user this entry claimed a FIRST list slot of (the users the prepared step's pair pass
// reads, for a hot list), else -1.
__device__ __forceinline__ int prepare_body(const PairsArgs &a, int2 *__restrict__ out, int64_t idx) {
    const int NP = 1 + a.n_neg, E = NP + 1;              // entries written per column
    const int64_t total = (int64_t)E * a.cols;
    if (idx >= total) return -1;
    const int64_t s = idx / E;
    const int q = (int)(idx - s * E);
    int2 *rec = out + s * pair_stride(a.n_neg);
    if (q == NP) {                                       // the plan slot of the positive
        rec[q] = make_int2(a.pos_slot != nullptr && s < a.n_pos ? a.pos_slot[s] : -1, 0);
        return -1;
    }
    const int64_t col = a.perm ? (int64_t)a.perm[s] : s;
    int2 r;
    if (q == 0) {
        r = (s < a.n_pos) ? make_int2((int)a.pos_user[col], (int)a.pos_item[col]) : make_int2(0, 0);
    } else {
        const int64_t j = (q - 1) * a.global_cols + a.col_offset + col;
        const uint2 w = a.words[j];
        r = a.pool[choice_index(w.x, w.y, a.pool_len)];
    }
    if (a.umark != nullptr) a.umark[r.x] = a.umark_step;   // plain store: every writer stores the same value
    int hot = -1;
    if (a.claimed) {
        // the list slots the pair pass would claim (pairs_body's validity): the positive if the
        // position has one, a negative if its column pairs with a positive or the loss is
        // pointwise; the planned positives' item side is reduced in LDS instead
        const bool pairwise = a.loss == RG_LOSS_BPR || a.loss == RG_LOSS_HINGE;
        const bool v = q == 0 ? s < a.n_pos : (a.loss != RG_LOSS_POINTWISE_POS && (s < a.n_pos || !pairwise));
        if (v) {
            const int su = atomicAdd(a.row_count + r.x, 1);
            if (su == 0) hot = r.x;
            const bool item_side = !(q == 0 && a.pos_slot != nullptr);
            const int si = item_side ? atomicAdd(a.row_count + a.num_users + r.y, 1) : 0;
            r.x |= (su < kCap ? su : kCap) << kSlotShift;
            r.y |= (si < kCap ? si : kCap) << kSlotShift;
        }
    }
    if (a.stamp != nullptr) {
        const int32_t ou = atomicExch(a.stamp + r.x, a.serial);
        const int32_t oi = atomicExch(a.stamp + a.num_users + r.y, a.serial);
        if (ou != a.serial) r.x |= kOwnerBit;
        if (oi != a.serial) r.y |= kOwnerBit;
    }
    rec[q] = r;
    return hot;
}

// append each lane's `user` (>= 0) to a.hot_out: one atomic per wave (a ballot and a prefix count),
// not one per user -- tens of thousands of returning atomics on ONE counter serialise; every lane of
// the wave calls it
__device__ __forceinline__ void hot_append(const PairsArgs &a, int user) {
    const unsigned long long m = __ballot(user >= 0);
    if (m == 0) return;
    const int lane = threadIdx.x & (kWave - 1);
    const int leader = __ffsll((unsigned long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(a.nhot_out, __popcll(m));
    base = __shfl(base, leader);
    if (user >= 0) a.hot_out[base + __popcll(m & ((1ull << lane) - 1ull))] = user;
}

// one prepared entry (every thread of the workgroup calls it: the hot-list append is per wave)
__device__ __forceinline__ void prepare_one(const PairsArgs &a, int2 *__restrict__ out, int64_t idx) {
    const int hot = prepare_body(a, out, idx);
    if (a.hot_out != nullptr) hot_append(a, hot);
}


__host__ __device__ inline int64_t prepare_threads(int64_t cols, int n_neg) { return (int64_t)(n_neg + 3) * cols; }

__global__ __launch_bounds__(kBlock) void mf_prepare_kernel(PairsArgs a, int2 *__restrict__ out, int prio) {
    if (prio) __builtin_amdgcn_s_setprio(2);   // small latency-bound kernel running beside the HBM-bound apply
    prepare_one(a, out, (int64_t)blockIdx.x * kBlock + threadIdx.x);
}

// atomically add a row-vector contribution (overflow path, rare; fixed point, rg_common.h)
template <class L>
__device__ __forceinline__ void overflow_add(long long *__restrict__ hot, int64_t row, int D, int sub, float dz,
                                             const float (&o)[L::EPL]) {
#pragma unroll
    for (int e = 0; e < L::EPL; ++e) {
        const int c = L::elem(sub, e);
        if (L::VEC || c < D) fix_add(hot + row * (int64_t)D + c, dz * o[e]);
    }
}

// select x[q] for a runtime q without dynamic register indexing (no scratch)
template <int N, class T>
__device__ __forceinline__ T pick(const T (&x)[N], int q) {
    T r = x[0];
#pragma unroll
    for (int k = 1; k < N; ++k) r = (q == k) ? x[k] : r;
    return r;
}

constexpr int kLdsFloats = 5 * kPairBlock;   // >= units per block * (dim + 1) for every layout (1280 at 256 threads)

// One unit = one batch column: pair q = 0 is the positive, q = 1..n the
// negatives k*global_cols + col.  Every gather uses an always-valid index and is
// issued unconditionally (results of invalid pairs are masked afterwards), so a
// wave has all of its rows in flight at once.  The gathered rows die after their
// dot product except the positive's user row, which feeds the planned item-side
// partial sums; the rare list-overflow path re-gathers.
//
// List tasks: t = 2q + side (side 0: user row of pair q, 1: its item row), spread
// over the unit's lanes as t = sub + j*LPU.  With a plan, the positives are
// processed in item-sorted order and the positive's item side (t = 1, the Zipf-hot
// rows) is instead reduced per block in LDS into one partial row per
// (item, block): plain stores, no atomics, fixed order.
template <class L, int PHASE, int NMAX, bool SC1 = false>
__device__ __forceinline__ void pairs_body(const PairsArgs &a, const int64_t blk) {
    constexpr int LPU = L::LPU, EPL = L::EPL, NP = NMAX + 1;
    constexpr int UPB = kPairBlock / LPU;                  // units per block
    constexpr int TPL = (2 * NP + LPU - 1) / LPU;      // list tasks per lane
    constexpr bool kBackward = (PHASE == kFused) || (PHASE == kAdaptBwd);
    constexpr bool kScoresFromBuf = (PHASE == kAdaptBwd) || (PHASE == kAdaptLoss);
    __shared__ float red[2][kPairBlock / kWave];
    __shared__ float lrow[UPB * (LPU * EPL + 1)];   // a planned partial row (D <= LPU * EPL) per unit
    __shared__ int lslot[UPB];
    __shared__ float ldz[kBackward ? UPB * NP : 1];
    const int lane = threadIdx.x & (kWave - 1);
    const int sub = lane & (LPU - 1);
    const int ubase = lane & ~(LPU - 1);
    const int ublk = threadIdx.x / LPU;               // unit within the block
    const int64_t s = blk * UPB + ublk;                 // processing position
    const bool active = s < a.cols;
    const bool plan = a.pos_slot != nullptr;
    const bool has_pos = active && s < a.n_pos;        // a plan puts the positives first
    const int D = a.dim;
    const int n = a.n_neg;
    const bool pairwise = (a.loss == RG_LOSS_BPR) || (a.loss == RG_LOSS_HINGE);
    const bool negs = a.loss != RG_LOSS_POINTWISE_POS;   // no negative pool: positives only
    RG_STAMP(0);

    // ---- ids of every pair, prepared in processing order (one coalesced round trip) ----
    int uid[NP], iid[NP];
    bool valid[NP];
    valid[0] = has_pos;
#pragma unroll
    for (int k = 0; k < NMAX; ++k)   // flat negatives that pair with no positive only matter to pointwise / adaptive
        valid[k + 1] = !kScoresFromBuf && negs && active && k < n && (has_pos || !pairwise);
    // the column's record: every pair's ids and the positive's plan slot in one line
    // (the slot entry is loaded with the ids, unconditionally: issued after them it became a
    // second round trip that queued behind the gathers of the waves already past this point)
    const int2 *rec = a.pairs + (active ? s : 0) * (int64_t)pair_stride(n);
    const int2 slot_entry = rec[n + 1];
    const bool claimed = kBackward && a.claimed;
    const int32_t idm = a.claimed ? kClaimIdMask : kIdMask;   // drop the ownership flags / slots
#pragma unroll
    for (int q = 0; q < NP; ++q) {
        const int2 pr = rec[(valid[q] || q == 0) ? q : 0];
        uid[q] = pr.x & idm;
        iid[q] = pr.y & idm;
    }
    const int myslot = (kBackward && plan && has_pos) ? slot_entry.x : -1;
    // each list task's own pair, loaded from the record beside the ids: indexing uid[] /
    // iid[] / valid[] by the lane-dependent pair index made the compiler keep them as a
    // per-thread LDS array (18 KB per workgroup), which slowed this whole phase ~10x
    int tu[TPL], ti[TPL];
    bool tv[TPL];
    int slot[TPL];
#pragma unroll
    for (int j = 0; j < TPL; ++j) {
        const int t = sub + j * LPU, q = t >> 1;
        const bool inb = t < 2 * NP && q <= n;
        tv[j] = inb && (q == 0 ? has_pos : (!kScoresFromBuf && negs && active && (has_pos || !pairwise)));
        const int2 e = rec[inb ? q : 0];
        tu[j] = e.x & idm;
        ti[j] = e.y & idm;
        slot[j] = claimed ? (int)(((uint32_t)((t & 1) ? e.y : e.x) >> kSlotShift) & 15u) : 0;
    }
    RG_STAMP(1);
    if (RG_DIAG_FLAG(3)) return;

    // ---- claim list slots early (their latency hides under the gathers) -------
#pragma unroll
    for (int j = 0; j < TPL; ++j) {
        const int t = sub + j * LPU;
        if (kBackward && !claimed && t < 2 * NP && !(plan && t == 1)) {
            if (tv[j] && !RG_DIAG_FLAG(0)) {
                const int64_t row = (t & 1) ? a.num_users + ti[j] : (int64_t)tu[j];
                slot[j] = atomicAdd(a.row_count + row, 1);
            }
        }
    }

    // ---- gather rows, scores ---------------------------------------------------
    float p[NP];
    float upos[EPL];      // the positive's user row (planned item-side partial sums)
    L::zero(upos);
    if (kScoresFromBuf) {
        p[0] = has_pos ? a.scores[s] : 0.5f;
#pragma unroll
        for (int q = 1; q < NP; ++q) p[q] = 0.5f;
        if (plan && kBackward) L::load(upos, a.user_w, uid[0], D, sub);
    } else {
        float ur[NP][EPL], ir[NP][EPL], ub[NP], ib[NP];
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            if constexpr (SC1) {   // rows written by this launch's hot workgroups (mf_pipe_kernel)
                L::load_sc1(ur[q], a.user_w, uid[q], D, sub);
                L::load_sc1(ir[q], a.item_w, iid[q], D, sub);
                ub[q] = L::load1_sc1(a.user_b + uid[q]);
                ib[q] = L::load1_sc1(a.item_b + iid[q]);
            } else {
                L::load(ur[q], a.user_w, uid[q], D, sub);
                L::load(ir[q], a.item_w, iid[q], D, sub);
                ub[q] = a.user_b[uid[q]];
                ib[q] = a.item_b[iid[q]];
            }
        }
#pragma unroll
        for (int e = 0; e < EPL; ++e) upos[e] = ur[0][e];
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            float d = 0.0f;
#pragma unroll
            for (int e = 0; e < EPL; ++e) d = fmaf(ur[q][e], ir[q][e], d);
            d = group_sum<LPU>(d);
            p[q] = sigmoidf_ref((d + ub[q]) + ib[q]);
        }
    }

    RG_STAMP(2);
    // ---- loss terms and dL/dp ---------------------------------------------------
    float la = 0.0f, lb = 0.0f;
    float dp[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) dp[q] = 0.0f;
    if (PHASE == kAdaptFwd) {
        if (sub == 0 && has_pos) a.scores[s] = p[0];
        const int64_t col = a.perm ? (int64_t)a.perm[active ? s : 0] : s;
#pragma unroll
        for (int k = 0; k < NMAX; ++k) {
            if (valid[k + 1] && sub == 0) {
                const int64_t j = (int64_t)k * a.global_cols + a.col_offset + col;
                const unsigned long long key = ((unsigned long long)__float_as_uint(p[k + 1]) << 32) |
                                               (unsigned long long)(0xFFFFFFFFu - (uint32_t)j);
                atomicMax(a.max_key, key);
            }
        }
    } else if (kScoresFromBuf) {  // adaptive hinge, positives only (max negative: mf_adapt_max_kernel)
        if (has_pos) {
            const unsigned long long key = *a.max_key;
            const float m = __uint_as_float((uint32_t)(key >> 32));
            const float x = (m - p[0]) + 1.0f;
            la = fmaxf(x, 0.0f);
            if (x >= 0.0f) {
                dp[0] = -(1.0f / a.n_a);
                if (PHASE == kAdaptBwd && sub == 0) atomicAdd(a.active_count, 1);
            }
        }
    } else if (a.loss == RG_LOSS_POINTWISE || a.loss == RG_LOSS_POINTWISE_POS) {
        if (has_pos) {
            la = -fmaxf(logf(p[0]), -100.0f);
            dp[0] = ((p[0] - 1.0f) / fmaxf((1.0f - p[0]) * p[0], 1e-12f)) / a.n_a;
        }
#pragma unroll
        for (int k = 1; k < NP; ++k) {
            if (valid[k]) {
                lb += -fmaxf(logf(1.0f - p[k]), -100.0f);
                dp[k] = (p[k] / fmaxf((1.0f - p[k]) * p[k], 1e-12f)) / a.n_b;
            }
        }
    } else {  // bpr / hinge on the neg.view(n, B) pairing
        const float g = 1.0f / a.n_a;
        if (has_pos) {
#pragma unroll
            for (int k = 1; k < NP; ++k) {
                if (valid[k]) {
                    if (a.loss == RG_LOSS_BPR) {
                        const float sg = sigmoidf_ref(p[0] - p[k]);
                        la += 1.0f - sg;
                        const float dx = (-g) * (1.0f - sg) * sg;
                        dp[0] += dx;
                        dp[k] = -dx;
                    } else {
                        const float x = (p[k] - p[0]) + 1.0f;
                        la += fmaxf(x, 0.0f);
                        const float dx = x >= 0.0f ? g : 0.0f;
                        dp[0] -= dx;
                        dp[k] = dx;
                    }
                }
            }
        }
    }

    // ---- dz, list entries, planned partials ----------------------------------------
    if (kBackward) {
        float dz[NP];
#pragma unroll
        for (int q = 0; q < NP; ++q) dz[q] = (dp[q] * (1.0f - p[q])) * p[q];
        // the list tasks index dz by a lane-dependent pair: stage it through LDS
        // (a register select chain is turned back into scratch by the compiler).  A
        // unit's lanes share one wave and a wave's LDS operations complete in order, so
        // only the compiler must keep the reads after the writes (no workgroup barrier)
        if (sub == 0) {
#pragma unroll
            for (int q = 0; q < NP; ++q) ldz[ublk * NP + q] = dz[q];
        }
        static_assert(kWave % LPU == 0, "a unit's lanes must share a wave");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        RG_STAMP(3);
        bool ovf = false;
#pragma unroll
        for (int j = 0; j < TPL; ++j) {
            const int t = sub + j * LPU;
            if (t < 2 * NP && !(plan && t == 1)) {
                const int q = t >> 1;
                if (tv[j]) {
                    const int u = tu[j], i = ti[j];
                    const int64_t row = (t & 1) ? a.num_users + i : (int64_t)u;
                    if (slot[j] < kCap) {
                        if (!RG_DIAG_FLAG(1)) store_entry(a.row_list + row * kCap + slot[j], (t & 1) ? u : i, ldz[ublk * NP + q]);
                    }
                    else
                        ovf = true;
                }
            }
        }
        if (__any(ovf)) {   // wave-uniform: rows touched more than kCap times this step (re-gather)
#pragma unroll
            for (int t = 0; t < 2 * NP; ++t) {
                const int sl = __shfl(slot[t / LPU], ubase + (t % LPU));
                const int q = t >> 1;
                if (valid[q] && sl >= kCap && !(plan && t == 1)) {
                    float o[EPL];
                    if (t & 1) {
                        const int64_t row = a.num_users + iid[q];
                        if constexpr (SC1) L::load_sc1(o, a.user_w, uid[q], D, sub);
                        else L::load(o, a.user_w, uid[q], D, sub);
                        overflow_add<L>(a.hot_grad, row, D, sub, dz[q], o);
                        if (sub == 0) fix_add(a.hot_bias_grad + row, dz[q]);
                    } else {
                        if constexpr (SC1) L::load_sc1(o, a.item_w, iid[q], D, sub);
                        else L::load(o, a.item_w, iid[q], D, sub);
                        overflow_add<L>(a.hot_grad, uid[q], D, sub, dz[q], o);
                        if (sub == 0) fix_add(a.hot_bias_grad + uid[q], dz[q]);
                    }
                }
            }
        }
        RG_STAMP(4);
        if (plan) {
            // block-level segmented sum of the positives' item-side rows, sorted by item
            const int stride = D + 1;
            if (has_pos) {
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    const int c = L::elem(sub, e);
                    if (L::VEC || c < D) lrow[ublk * stride + c] = dz[0] * upos[e];
                }
                if (sub == 0) lrow[ublk * stride + D] = dz[0];
            }
            if (sub == 0) lslot[ublk] = myslot;
            lds_barrier();
            if (has_pos && (ublk == 0 || lslot[ublk - 1] != myslot)) {   // segment head
                float acc[EPL];
                float accb = 0.0f;
                L::zero(acc);
                for (int v = ublk; v < UPB && lslot[v] == myslot; ++v) {
#pragma unroll
                    for (int e = 0; e < EPL; ++e) {
                        const int c = L::elem(sub, e);
                        if (L::VEC || c < D) acc[e] += lrow[v * stride + c];
                    }
                    accb += lrow[v * stride + D];
                }
                if (!RG_DIAG_FLAG(2)) {
                    L::store(a.part_row, myslot, D, sub, acc);
                    if (sub == 0) a.part_bias[myslot] = accb;
                }
            }
        }
    }

    // ---- deterministic loss partials: wave DPP sum -> block -> partials[block] ----
    if (PHASE != kAdaptFwd) {
        float va = (sub == 0) ? la : 0.0f;
        float vb = (sub == 0) ? lb : 0.0f;
        va = group_sum<kWave>(va);
        vb = group_sum<kWave>(vb);
        const int w = threadIdx.x >> 6;
        if (lane == 0) { red[0][w] = va; red[1][w] = vb; }
        lds_barrier();
        if (threadIdx.x == 0) {
            float sa = 0.0f, sb = 0.0f;
#pragma unroll
            for (int i = 0; i < kPairBlock / kWave; ++i) { sa += red[0][i]; sb += red[1][i]; }
            a.partials[2 * blk] = sa;
            a.partials[2 * blk + 1] = sb;
        }
    }
    RG_STAMP(5);
}

template <class L, int PHASE, int NMAX>
__global__ __launch_bounds__(kPairBlock) void mf_pairs_kernel(PairsArgs a) {
    pairs_body<L, PHASE, NMAX>(a, blockIdx.x);
}

// the pair pass of this step (blocks [0, pair_blocks)) and the prepare pass of the NEXT
// step (the remaining blocks) in one launch: the lazy split step needs the
// next step's user marks before its dense pass starts, so the prepare moves out of the
// dense pass into this latency-bound launch, where its random pool reads run beside the
// pair pass's gathers
template <class L, int NMAX>
__global__ __launch_bounds__(kPairBlock) void mf_pairs_prep_kernel(PairsArgs a, PairsArgs prep, int2 *prep_out,
                                                                   int64_t pair_blocks) {
    const int64_t blk = blockIdx.x;
    if (blk < pair_blocks) {
        pairs_body<L, kFused, NMAX>(a, blk);
        return;
    }
    if constexpr (kPairBlock == kBlock) prepare_one(prep, prep_out, (blk - pair_blocks) * kBlock + threadIdx.x);
}

// adaptive hinge: the global-max negative receives sum_b 1/Bp over active b
// (spotlight/losses.py:170 torch.max(dim 0) backward -> argmax, first index on ties)
template <class L>
__global__ __launch_bounds__(kWave) void mf_adapt_max_kernel(PairsArgs a) {
    constexpr int LPU = L::LPU, EPL = L::EPL;
    const int lane = threadIdx.x;
    const int sub = lane & (LPU - 1);
    const unsigned long long key = *a.max_key;
    const int64_t j = (int64_t)(0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull));
    const int64_t colg = j % a.global_cols;
    const int64_t col = colg - a.col_offset;
    if (col < 0 || col >= a.cols) return;            // another rank owns the max
    if (lane >= LPU) return;
    const float pm = __uint_as_float((uint32_t)(key >> 32));
    const float dpv = (float)(*a.active_count) * (1.0f / a.n_a);
    const float dz = (dpv * (1.0f - pm)) * pm;
    const uint2 w = a.words[j];
    const int2 pr = a.pool[choice_index(w.x, w.y, a.pool_len)];
    float ur[EPL], ir[EPL];
    L::load(ur, a.user_w, pr.x, a.dim, sub);
    L::load(ir, a.item_w, pr.y, a.dim, sub);
    for (int side = 0; side < 2; ++side) {
        const int64_t row = side ? a.num_users + pr.y : (int64_t)pr.x;
        int sl = 0;
        if (sub == 0) sl = atomicAdd(a.row_count + row, 1);
        sl = __shfl(sl, 0);
        if (sl < kCap) {
            if (sub == 0) store_entry(a.row_list + row * kCap + sl, side ? pr.x : pr.y, dz);
        } else {
            overflow_add<L>(a.hot_grad, row, a.dim, sub, dz, side ? ur : ir);
            if (sub == 0) fix_add(a.hot_bias_grad + row, dz);
        }
    }
}

// ---------------------------------------------------------------------------- apply
struct ApplyArgs {
    const float *w_in[2], *b_in[2];
    float *w_out[2], *b_out[2];
    float *w_m[2], *w_v[2], *b_m[2], *b_v[2];
    int64_t num_users, num_items;
    int32_t dim;
    int64_t row_begin, row_end;   // unified rows: users [0, U), items [U, U + I)
    int32_t *row_count;
    const int2 *row_list;
    long long *hot_grad, *hot_bias_grad;     // int64 fixed point
    const int32_t *item_slot_off; // plan: item i's partial slots [off[i], off[i+1])
    const float *part_row, *part_bias;
    rg_opt_t opt;
    const float *partials;
    int64_t n_partials;
    double inv_a, inv_b;
    float *loss_out;
    float *grad;                  // flat [(re-rb)*D | (re-rb) | loss] (kGradOnly / kApplyDense)
    // NCF: list entries {example slot, 1.0f} point at per-example gradient rows
    // contrib[slot * contrib_stride + table * D ..] instead of partner rows (then no biases)
    const float *contrib;
    int64_t contrib_stride;
    bool has_bias;
    bool keep_count;              // NeuMF: the MF tables read the lists first, the MLP tables reset them
    // rank-major flat gradient of the replicated data-parallel step (rg_mf_grads_sharded /
    // rg_mf_apply_shard; shard_users == 0: the plain [(re-rb)*D | (re-rb) | loss] layout):
    // chunk s (chunk floats) = [user rows s*Us .. (s+1)*Us | item rows s*Is .. | their
    // biases (Us + Is) | loss], D floats per row
    int64_t shard_users, shard_items, chunk;
    int32_t world, rank;
    // owner-sharded step's item exchange (rg_mf_grads_item_shard / rg_mf_apply_item_shard): the
    // rank-major chunks hold item rows only (shard_users = 0): chunk s = [item rows s*Is .. | their
    // biases | loss]
    int32_t item_shard;
    // lazy dense pass: a USER row with a zero data gradient that the next step
    // does not read is skipped; its cold updates (weight decay + optimizer state only) are
    // applied, in order and with each step's constants, when the row is next processed
    int32_t *last_rel;            // [num_users] last step applied to the row, minus lazy_base
    const int32_t *umark;         // [num_users] step whose pair pass reads the row (prepare marks)
    const float2 *step_consts;    // [s] Adam (step_size, bias_correction2_sqrt) of absolute step s
    int64_t lazy_base;            // absolute step of last_rel == 0
    int32_t lazy_t;               // this step (absolute)
    int32_t lazy_full;            // process every user row (no next step known)
    unsigned long long *lazy_rows;   // optional: count of user rows processed (diagnostic steps)
    int32_t lazy_dbg;             // timing experiments only (RG_LAZY_DBG; wrong results): bit 0 no catch-up,
                                  // 1 every user row processed, 2 no constants window, 3 no odd-lag reload
    int32_t lazy_cap;             // > 0: a row that has missed this many steps is processed anyway
    // apply_row<..., GUARD>: a row with guard[r] > 0 is left alone (another launch updates it); the
    // guard is loaded beside the row's other loads, so it costs no round trip of its own
    const int32_t *guard;
};

#ifndef RG_MF_SORTED_PULL
#define RG_MF_SORTED_PULL 1
#endif
// sort the first ne of kCap list entries ascending by (other, dz bits) -- an 8-input
// sorting network (19 compare-exchanges, register only); entries past ne key as +inf
__device__ __forceinline__ uint64_t ent_key(int2 e, bool valid) {
    return valid ? ((uint64_t)(uint32_t)e.x << 32) | (uint64_t)(uint32_t)e.y : ~0ull;
}
__device__ __forceinline__ void sort_entries(int2 (&ent)[8], int ne) {
    uint64_t k[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) k[e] = ent_key(ent[e], e < ne);
#define RG_CX(i, j)                                     \
    {                                                   \
        const uint64_t lo = k[i] < k[j] ? k[i] : k[j];  \
        const uint64_t hi = k[i] < k[j] ? k[j] : k[i];  \
        k[i] = lo;                                      \
        k[j] = hi;                                      \
    }
    RG_CX(0, 2) RG_CX(1, 3) RG_CX(4, 6) RG_CX(5, 7)
    RG_CX(0, 4) RG_CX(1, 5) RG_CX(2, 6) RG_CX(3, 7)
    RG_CX(0, 1) RG_CX(2, 3) RG_CX(4, 5) RG_CX(6, 7)
    RG_CX(2, 4) RG_CX(3, 5)
    RG_CX(1, 4) RG_CX(3, 6)
    RG_CX(1, 2) RG_CX(3, 4) RG_CX(5, 6)
#undef RG_CX
#pragma unroll
    for (int e = 0; e < 8; ++e) ent[e] = make_int2((int)(uint32_t)(k[e] >> 32), (int)(uint32_t)k[e]);
}

// location of unified row r's gradient in the flat buffer: *row_base + k*D, bias at *bias
__device__ __forceinline__ void grad_loc(const ApplyArgs &a, int t, int64_t lr_, int64_t gk, int64_t nr,
                                         const float *&row_base, int64_t &k, int64_t &bias) {
    if (a.shard_users > 0 || a.item_shard) {
        const int64_t s = t ? lr_ / a.shard_items : lr_ / a.shard_users;
        k = t ? a.shard_users + lr_ % a.shard_items : lr_ % a.shard_users;
        row_base = a.grad + s * a.chunk;
        bias = s * a.chunk + (a.shard_users + a.shard_items) * (int64_t)a.dim + k;
    } else {
        row_base = a.grad;
        k = gk;
        bias = nr * (int64_t)a.dim + gk;
    }
}

// mf_apply modes: pull the gradient from the lists and update (single GPU);
// pull into the flat dense gradient (before an all-reduce);
// update from the (all-reduced) flat gradient.
enum ApplyMode : int { kApplyPull = 0, kGradOnly = 1, kApplyDense = 2, kApplyCold = 3 /* arg checks only */ };

// loss of the step from the pair kernel's per-block partials (one wave, fixed order)
__device__ __forceinline__ float finalize_loss(const float *__restrict__ partials, int64_t np_, double inv_a,
                                               double inv_b, int lane) {
    // eight partials per lane in flight per round (the owner step's backward leaves ~3k): one
    // round trip per 512 partials instead of per 64; fixed order, so the sum is deterministic
    constexpr int kU = 8;
    double sa = 0.0, sb = 0.0;
    for (int64_t i0 = lane; i0 < np_; i0 += kU * kWave) {
        float2 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t i = i0 + (int64_t)u * kWave;
            v[u] = i < np_ ? reinterpret_cast<const float2 *>(partials)[i] : make_float2(0.0f, 0.0f);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            sa += (double)v[u].x;
            sb += (double)v[u].y;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        sa += __shfl_xor(sa, off);
        sb += __shfl_xor(sb, off);
    }
    return (float)(sa * inv_a + sb * inv_b);
}

// The same loss over a whole workgroup (every thread of it calls this; every thread gets
// the value): a data-parallel step's backward leaves thousands of partials, which one wave
// reads in ~6 dependent rounds -- a floor under the short launch that finalizes them.
// Fixed partition and combine order: deterministic.
template <int NT>
__device__ __forceinline__ float finalize_loss_wg(const float *__restrict__ partials, int64_t np_, double inv_a,
                                                  double inv_b) {
    constexpr int kU = 8, NW = NT / kWave;
    __shared__ double red[2][NW];
    __shared__ float out;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    double sa = 0.0, sb = 0.0;
    for (int64_t i0 = tid; i0 < np_; i0 += (int64_t)kU * NT) {
        float2 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t i = i0 + (int64_t)u * NT;
            v[u] = i < np_ ? reinterpret_cast<const float2 *>(partials)[i] : make_float2(0.0f, 0.0f);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            sa += (double)v[u].x;
            sb += (double)v[u].y;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        sa += __shfl_xor(sa, off);
        sb += __shfl_xor(sb, off);
    }
    if (lane == 0) { red[0][w] = sa; red[1][w] = sb; }
    __syncthreads();
    if (tid == 0) {
        double ta = 0.0, tb = 0.0;
#pragma unroll
        for (int k = 0; k < NW; ++k) { ta += red[0][k]; tb += red[1][k]; }
        out = (float)(ta * inv_a + tb * inv_b);
    }
    __syncthreads();
    return out;
}

// Gradient + optimizer update of unified row r (users [0, U), items [U, U + I)).
// COLD: a row no pair of the step touches -- its data gradient is exactly zero
// (only the coupled weight decay acts), so nothing of the step's scratch is read.
struct LazyRow {
    int cnt;          // list count (data gradient this step)
    int32_t mk, lsr;  // prepare mark, last step applied (relative)
    bool active;      // false: a lane group past the end of the rows
};

// wave-uniform maximum (every lane ends with the same value)
__device__ __forceinline__ int wave_max(int x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = max(x, __shfl_xor(x, o));
    return __builtin_amdgcn_readfirstlane(x);
}

// this lane's Adam constants of window step `lane` (absolute step s0 + lane, lane < n)
__device__ __forceinline__ float2 window_const(const ApplyArgs &a, int64_t s0, int n) {
    const int lane = threadIdx.x & (kWave - 1);
    return (a.opt.kind == RG_OPT_ADAM && lane < n) ? a.step_consts[s0 + lane] : make_float2(0.0f, 0.0f);
}

// The cold updates a row missed (zero data gradient: the coupled weight decay and the
// optimizer state only), in step order, each with its own Adam constants -- the exact
// operation sequence the eager dense pass applies to a row no pair touches (opt_update with
// gdata = 0), so the row ends bit-identical.  The loop runs over the wave's window of the
// `wmax` steps before `upto`, so the step is wave-uniform: its constants come from lane k of
// `cl` (loaded beside the row, 64 steps per load) by readlane, and each row updates only at
// the last `mylag` steps of the window.
template <class L>
__device__ __forceinline__ void catch_up(const ApplyArgs &a, float2 cl, int wmax, int mylag, int64_t upto, int sub,
                                         float (&p)[L::EPL], float (&m)[L::EPL], float (&v)[L::EPL], float &pb,
                                         float &mb, float &vb) {
    if (wmax <= 0) return;
    rg_opt_t o = a.opt;
    const bool adam = o.kind == RG_OPT_ADAM;
    const int first = wmax - mylag;
    for (int c0 = 0; c0 < wmax; c0 += kWave) {
        if (c0 > 0) cl = window_const(a, upto - wmax + c0, wmax - c0);
        const int n = wmax - c0 < kWave ? wmax - c0 : kWave;
        for (int k = 0; k < n; ++k) {
            if (adam) {
                o.step_size = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cl.x), k));
                o.bias_correction2_sqrt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cl.y), k));
            }
            if (c0 + k < first) continue;
#pragma unroll
            for (int q = 0; q < L::EPL; ++q) p[q] = opt_update(o, p[q], 0.0f, m[q], v[q]);
            if (sub == 0 && a.has_bias) pb = opt_update(o, pb, 0.0f, mb, vb);
        }
    }
}

#ifndef RG_LEAN_PULL
#define RG_LEAN_PULL 0
#endif
#ifndef RG_LEAN_PG
#define RG_LEAN_PG 2
#endif
// Ascending sort of the 8 list entries held one per lane (lanes sub 0..7 of each LPU-lane row
// group; sub >= 8 hold +inf keys and sort among themselves): a bitonic network over lane
// XOR partners, 6 compare-exchange stages of 64-bit keys.  The result (entry e on lane e) is
// the order sort_entries gives, so the row sums its contributions in the same order.
template <int LPU>
__device__ __forceinline__ uint64_t lane_sort8(uint64_t key, int sub) {
#pragma unroll
    for (int k = 2; k <= 8; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint64_t o = __shfl_xor(key, j, LPU);
            const bool up = (sub & k) == 0;
            const bool lower = (sub & j) == 0;
            const uint64_t lo = key < o ? key : o, hi = key < o ? o : key;
            key = (lower == up) ? lo : hi;
        }
    }
    return key;
}

// Pull-and-update of unified row r (the single-GPU dense pass, MODE kApplyPull) with a small
// register footprint: each row's 8 list entries are held one per lane and sorted across the
// lanes (apply_row holds all 8 in every lane and sorts them in registers).  Split in two so a
// wave can hold the NEXT row group's loads in flight while it finishes this one
// (mf_dense_kernel): lean_load issues every load a row needs that does not depend on another
// load (p, m, v, biases, count, its list entries, the item's partial-slot range); lean_finish
// pulls the partner rows (and planned partials) those name, updates and stores.  The
// summation order is apply_row's (sorted entries, fma chain; overflowed rows in fixed point;
// planned partials after), so the result is bit-identical to it.
template <class L>
struct LeanRow {
    float p[L::EPL], m[L::EPL], v[L::EPL];
    float pb, mb, vb;
    int c;
    int2 ent;
    int s0, s1;
};

template <class L>
__device__ __forceinline__ void lean_load(const ApplyArgs &a, const int64_t r, const int sub, const bool valid,
                                          LeanRow<L> &x) {
    const int t = r < a.num_users ? 0 : 1;
    const int64_t lr_ = t ? r - a.num_users : r;
    const bool adam = a.opt.kind == RG_OPT_ADAM;
    const bool has_v = a.opt.kind != RG_OPT_SGD;
    const int D = a.dim;
    L::zero(x.p); L::zero(x.m); L::zero(x.v);
    x.pb = x.mb = x.vb = 0.0f;
    x.c = 0;
    x.ent = make_int2(0, 0);
    x.s0 = x.s1 = 0;
    if (!valid) return;
    L::load(x.p, a.w_in[t], lr_, D, sub);
    if (adam) L::load(x.m, a.w_m[t], lr_, D, sub);
    if (has_v) L::load(x.v, a.w_v[t], lr_, D, sub);
    if (sub == 0 && a.has_bias) {
        x.pb = a.b_in[t][lr_];
        if (adam) x.mb = a.b_m[t][lr_];
        if (has_v) x.vb = a.b_v[t][lr_];
    }
    x.c = a.row_count[r];
    if (sub < kCap) x.ent = a.row_list[r * kCap + sub];
    if (t == 1 && a.item_slot_off != nullptr) { x.s0 = a.item_slot_off[lr_]; x.s1 = a.item_slot_off[lr_ + 1]; }
}

template <class L, bool WT = false>
__device__ __forceinline__ void lean_finish(const ApplyArgs &a, const int64_t r, const int sub, const bool valid,
                                            LeanRow<L> &x) {
    constexpr int EPL = L::EPL, LPU = L::LPU, PG = RG_LEAN_PG;
    static_assert(LPU >= kCap, "one list entry per lane");
    const int D = a.dim;
    const int t = r < a.num_users ? 0 : 1;
    const int64_t lr_ = t ? r - a.num_users : r;
    const bool adam = a.opt.kind == RG_OPT_ADAM;
    const bool has_v = a.opt.kind != RG_OPT_SGD;
    const int c = x.c;
    float g[EPL];
    float gb = 0.0f;
    L::zero(g);
    const int lane = threadIdx.x & (kWave - 1);
    const int rowbase = lane & ~(LPU - 1);
    if (__any(c > 0)) {
        const int ne = c < kCap ? c : kCap;
        uint64_t key = ent_key(x.ent, sub < ne);
#if RG_MF_SORTED_PULL
        key = lane_sort8<LPU>(key, sub);
#endif
        const float *other = a.contrib ? a.contrib + t * D : a.w_in[t ^ 1];
        const int64_t ostride = a.contrib ? a.contrib_stride : (int64_t)D;
        const bool fixp = c > kCap;   // an overflowed row sums list and surplus in fixed point
        long long gf[EPL];
        long long gbf = 0;
#pragma unroll
        for (int q = 0; q < EPL; ++q) gf[q] = 0;
#pragma unroll
        for (int h = 0; h < kCap; h += PG) {
            if (h > 0 && !__any(ne > h)) break;
            uint64_t k[PG];
            float o[PG][EPL];
#pragma unroll
            for (int e = 0; e < PG; ++e) {
                k[e] = __shfl(key, rowbase + h + e);
                if (h + e < ne) L::load_strided(o[e], other, (int)(uint32_t)(k[e] >> 32), ostride, D, sub);
                else L::zero(o[e]);
            }
#pragma unroll
            for (int e = 0; e < PG; ++e) {
                if (h + e < ne) {
                    const float dz = __uint_as_float((uint32_t)k[e]);
                    if (fixp) {
#pragma unroll
                        for (int q = 0; q < EPL; ++q) gf[q] += to_fix(dz * o[e][q]);
                        gbf += to_fix(dz);
                    } else {
#pragma unroll
                        for (int q = 0; q < EPL; ++q) g[q] = fmaf(dz, o[e][q], g[q]);
                        gb += dz;
                    }
                }
            }
        }
        if (fixp) {
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                const int cc = L::elem(sub, e);
                if (L::VEC || cc < D) {
                    long long *hp = a.hot_grad + r * (int64_t)D + cc;
                    gf[e] += *hp;
                    *hp = 0;
                }
            }
#pragma unroll
            for (int q = 0; q < EPL; ++q) g[q] = from_fix(gf[q]);
            if (sub == 0 && a.has_bias) {
                gbf += a.hot_bias_grad[r];
                a.hot_bias_grad[r] = 0;
            }
            gb = from_fix(gbf);
        }
        if (valid && sub == 0 && c > 0 && !a.keep_count) a.row_count[r] = 0;
    }
    const int s0 = x.s0, s1 = x.s1;
    if (__any(s1 > s0)) {   // planned positive partials of this item, in slot order
        for (int sl = s0; __any(sl < s1); sl += PG) {
            float h[PG][EPL];
            float hb[PG];
#pragma unroll
            for (int u = 0; u < PG; ++u) {
                const bool in = sl + u < s1;
                if (in) {
                    L::load(h[u], a.part_row, sl + u, D, sub);
                    hb[u] = a.has_bias ? a.part_bias[sl + u] : 0.0f;
                } else {
                    L::zero(h[u]);
                    hb[u] = 0.0f;
                }
            }
#pragma unroll
            for (int u = 0; u < PG; ++u) {
                if (sl + u < s1) {
#pragma unroll
                    for (int q = 0; q < EPL; ++q) g[q] += h[u][q];
                    gb += hb[u];
                }
            }
        }
    }
    if (!valid) return;
#pragma unroll
    for (int q = 0; q < EPL; ++q) x.p[q] = opt_update(a.opt, x.p[q], g[q], x.m[q], x.v[q]);
    // WT: the row and bias write-through (another workgroup of the launch reads them:
    // mf_pipe_kernel's pair pass); the optimizer state is not read there
    if (WT) L::store_wt(a.w_out[t], lr_, D, sub, x.p);
    else L::store(a.w_out[t], lr_, D, sub, x.p);
    if (adam) L::store(a.w_m[t], lr_, D, sub, x.m);
    if (has_v) L::store(a.w_v[t], lr_, D, sub, x.v);
    if (sub == 0 && a.has_bias) {
        x.pb = opt_update(a.opt, x.pb, gb, x.mb, x.vb);
        if (WT) L::store1_wt(a.b_out[t] + lr_, x.pb);
        else a.b_out[t][lr_] = x.pb;
        if (adam) a.b_m[t][lr_] = x.mb;
        if (has_v) a.b_v[t][lr_] = x.vb;
    }
}

template <class L>
__device__ __forceinline__ void apply_row_lean(const ApplyArgs &a, const int64_t r, const int sub) {
    LeanRow<L> x;
    lean_load<L>(a, r, sub, true, x);
    lean_finish<L>(a, r, sub, true, x);
}

template <class L, int MODE, int NT, bool COLD, bool SPEC = false, bool LAZY = false, bool LSPEC = false,
          bool GUARD = false>
__device__ __forceinline__ void apply_row(const ApplyArgs &a, const int64_t r, const int sub,
                                          const LazyRow lzr = LazyRow{}) {
    constexpr int EPL = L::EPL;
    if constexpr (RG_LEAN_PULL && MODE == kApplyPull && !LAZY && !COLD && NT == 0 && L::LPU >= kCap) {
        apply_row_lean<L>(a, r, sub);
        return;
    }
    const int64_t rb = a.row_begin, nr = a.row_end - rb;
    const int D = a.dim;
    const int t = r < a.num_users ? 0 : 1;          // 0: user table, 1: item table
    const int64_t lr_ = t ? r - a.num_users : r;
    const int64_t gk = r - rb;                      // index in the flat gradient
    const bool adam = a.opt.kind == RG_OPT_ADAM;
    const bool has_v = a.opt.kind != RG_OPT_SGD;

    // lazy user row: processed iff it has a data gradient this step (list count), the next
    // step's pair pass reads it (prepare mark), or the pass is a full one; its current value
    // is in the set written at its last step -- w_in if an even number of steps was missed
    // since, else w_out (then the update is in place)
    const bool lz = LAZY && t == 0;
    int lag = 0;
    const int32_t lsr = lzr.lsr;
    // proc: this row is updated this step (false: a lazily skipped user row, which still runs
    // through to the wave's catch-up loop -- a wave-collective -- doing nothing)
    const int missed = lz ? (int)((int64_t)a.lazy_t - 1 - a.lazy_base - lsr) : 0;
    const bool proc = !lz || (lzr.active && (a.lazy_full || (a.lazy_dbg & 2) || lzr.cnt > 0 ||
                                             lzr.mk == a.lazy_t + 1 || (a.lazy_cap > 0 && missed >= a.lazy_cap)));
    const int cnt = proc ? lzr.cnt : 0;
    const float *src_w = a.w_in[t], *src_b = a.b_in[t];
    float p[EPL], m[EPL], v[EPL], g[EPL];
    float pb = 0.0f, mb = 0.0f, vb = 0.0f;
    L::zero(p); L::zero(m); L::zero(v);
    int2 lspec[LSPEC ? kCap : 1];
    if (lz) {
        // LSPEC: p (from the set a row processed last step holds it in), m, v and the list are
        // loaded with the decision words, in one round trip as the eager pass; a processed row
        // that missed an odd number of steps reloads p from the other set
        if (LSPEC && lzr.active) {
            L::load(p, a.w_in[0], lr_, D, sub);
            if (adam) L::load(m, a.w_m[0], lr_, D, sub);
            if (has_v) L::load(v, a.w_v[0], lr_, D, sub);
            if (sub == 0 && a.has_bias) {
                pb = a.b_in[0][lr_];
                if (adam) mb = a.b_m[0][lr_];
                if (has_v) vb = a.b_v[0][lr_];
            }
            const int4 *lst = reinterpret_cast<const int4 *>(a.row_list + r * kCap);
#pragma unroll
            for (int e = 0; e < kCap / 2; ++e) {
                const int4 q = lst[e];
                lspec[2 * e] = make_int2(q.x, q.y);
                lspec[2 * e + 1] = make_int2(q.z, q.w);
            }
        }
        lag = proc ? missed : 0;
        if (lag & 1) {
            src_w = a.w_out[t];
            src_b = a.b_out[t];
        }
    }
    // the wave's catch-up window and its constants (issued with the row's loads)
    const int wmax = LAZY ? wave_max(lag) : 0;
    const float2 wconst = (LAZY && wmax > 0 && !(a.lazy_dbg & 4)) ? window_const(a, (int64_t)a.lazy_t - wmax, wmax)
                                                                    : make_float2(0.0f, 0.0f);
    if (LSPEC && lz && proc && (lag & 1) && !(a.lazy_dbg & 8)) {
        L::load(p, src_w, lr_, D, sub);
        if (sub == 0 && a.has_bias) pb = src_b[lr_];
    }

    if (MODE != kGradOnly && proc && !(LSPEC && lz)) {
        if (NT == 2) {
            L::load_nt(p, src_w, lr_, D, sub);
            if (adam) L::load_nt(m, a.w_m[t], lr_, D, sub); else L::zero(m);
            if (has_v) L::load_nt(v, a.w_v[t], lr_, D, sub); else L::zero(v);
        } else {
            L::load(p, src_w, lr_, D, sub);
            if (!(LSPEC && lz)) {
                if (adam) L::load(m, a.w_m[t], lr_, D, sub); else L::zero(m);
                if (has_v) L::load(v, a.w_v[t], lr_, D, sub); else L::zero(v);
            }
        }
        if (sub == 0 && a.has_bias) {
            pb = src_b[lr_];
            if (!(LSPEC && lz)) {
                if (adam) mb = a.b_m[t][lr_];
                if (has_v) vb = a.b_v[t][lr_];
            }
        }
    }
    L::zero(g);
    float gb = 0.0f;
    bool guarded = false;
    if constexpr (GUARD) guarded = a.guard[r] > 0;

    if (MODE == kApplyDense) {
        const float *gbase;
        int64_t gkk, gbi;
        grad_loc(a, t, lr_, gk, nr, gbase, gkk, gbi);
        L::load(g, gbase, gkk, D, sub);
        if (sub == 0) gb = a.grad[gbi];
    } else if (!COLD) {
        const int c = lz ? cnt : (COLD ? 0 : a.row_count[r]);
        // SPEC: the list and the item's partial-slot range are loaded beside the count
        // (entries past the count are stale and never used), so a touched row's partner
        // rows are its only dependent round trip
        int2 spec[SPEC ? kCap : 1];
        int s0 = 0, s1 = 0;
        if (SPEC && !lz) {
            const int4 *lst = reinterpret_cast<const int4 *>(a.row_list + r * kCap);
#pragma unroll
            for (int e = 0; e < kCap / 2; ++e) {
                const int4 v = lst[e];
                spec[2 * e] = make_int2(v.x, v.y);
                spec[2 * e + 1] = make_int2(v.z, v.w);
            }
            if (t == 1 && a.item_slot_off != nullptr) { s0 = a.item_slot_off[lr_]; s1 = a.item_slot_off[lr_ + 1]; }
        }
        // kGradOnly (the data-parallel item gradient: a short, latency-bound launch over rows
        // that are nearly all touched): every load of the row -- all partner rows, the
        // overflow accumulators, the first planned partials -- issues in ONE round trip after
        // the list instead of a dependent chain; the sums keep their order (same bits)
        constexpr bool kOneTrip = MODE == kGradOnly && SPEC;
        float h0[kOneTrip ? 4 : 1][EPL];
        float hb0[kOneTrip ? 4 : 1];
        const bool parts = t == 1 && a.item_slot_off != nullptr;
        if (kOneTrip && parts && s1 > s0) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int ss = s0 + u < s1 ? s0 + u : s0;
                L::load(h0[kOneTrip ? u : 0], a.part_row, ss, D, sub);
                hb0[kOneTrip ? u : 0] = a.has_bias ? a.part_bias[ss] : 0.0f;
            }
        }
        if (c > 0 && !guarded) {
            const int ne = c < kCap ? c : kCap;
            int2 ent[kCap];
#pragma unroll
            for (int e = 0; e < kCap; ++e)
                ent[e] = e < ne ? ((LSPEC && lz) ? lspec[LSPEC ? e : 0]
                                   : (SPEC && !lz) ? spec[SPEC ? e : 0] : a.row_list[r * kCap + e]) : make_int2(0, 0);
#if RG_MF_SORTED_PULL
            // the entries' slots were claimed by atomics in arrival order: sorted by (partner,
            // dz bits) the row sums them in an order independent of that timing, so a step
            // whose rows do not overflow is bit-reproducible run to run
            sort_entries(ent, ne);
#endif
            // MF: the partner row of the other table; NCF: the stored gradient half
            const float *other = a.contrib ? a.contrib + t * D : a.w_in[t ^ 1];
            const int64_t ostride = a.contrib ? a.contrib_stride : (int64_t)D;
            // partner rows in groups of PG list entries (RG_MF_PULL_GROUP; most touched rows have
            // 1-2 entries): a later group's gathers issue only when some row of the wave needs them,
            // and the smaller register footprint raises occupancy
            constexpr int PG = kOneTrip ? kCap : RG_MF_PULL_GROUP;
            // an overflowed row (c > kCap) sums list and surplus in fixed point (see fix_add)
            const bool fixp = c > kCap;
            long long gf[EPL];
            long long gbf = 0;
#pragma unroll
            for (int q = 0; q < EPL; ++q) gf[q] = 0;
            long long hv[kOneTrip ? EPL : 1];
            long long hbv = 0;
            if (kOneTrip && fixp) {     // the surplus' accumulators, loaded with the partner rows
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    const int cc = L::elem(sub, e);
                    hv[kOneTrip ? e : 0] = (L::VEC || cc < D) ? a.hot_grad[r * (int64_t)D + cc] : 0;
                }
                if (sub == 0 && a.has_bias) hbv = a.hot_bias_grad[r];
            }
#pragma unroll
            for (int h = 0; h < kCap / PG; ++h) {
                if (h > 0 && !__any(ne > h * PG)) break;
                float o[PG][EPL];
#pragma unroll
                for (int e = 0; e < PG; ++e) {
                    if (h * PG + e < ne) L::load_strided(o[e], other, ent[h * PG + e].x, ostride, D, sub);
                    else L::zero(o[e]);
                }
#pragma unroll
                for (int e = 0; e < PG; ++e) {
                    if (h * PG + e < ne) {
                        const float dz = __int_as_float(ent[h * PG + e].y);
                        if (fixp) {
#pragma unroll
                            for (int q = 0; q < EPL; ++q) gf[q] += to_fix(dz * o[e][q]);
                            gbf += to_fix(dz);
                        } else {
#pragma unroll
                            for (int q = 0; q < EPL; ++q) g[q] = fmaf(dz, o[e][q], g[q]);
                            gb += dz;
                        }
                    }
                }
            }
            if (fixp) {
                // the surplus' accumulators (fixed point), read and reset
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    const int cc = L::elem(sub, e);
                    if (L::VEC || cc < D) {
                        long long *hp = a.hot_grad + r * (int64_t)D + cc;
                        gf[e] += kOneTrip ? hv[kOneTrip ? e : 0] : *hp;
                        *hp = 0;
                    }
                }
#pragma unroll
                for (int q = 0; q < EPL; ++q) g[q] = from_fix(gf[q]);
                if (sub == 0 && a.has_bias) {
                    gbf += kOneTrip ? hbv : a.hot_bias_grad[r];
                    a.hot_bias_grad[r] = 0;
                }
                gb = from_fix(gbf);
            }
            if (sub == 0 && !a.keep_count) a.row_count[r] = 0;
        }
        if (parts && !guarded) {   // planned positive partials of this item
            if (!SPEC || lz) { s0 = a.item_slot_off[lr_]; s1 = a.item_slot_off[lr_ + 1]; }
            for (int sl = s0; sl < s1; sl += 4) {
                float h[4][EPL];
                float hb[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (kOneTrip && sl == s0) {        // the first four, loaded beside the partner rows
#pragma unroll
                        for (int q = 0; q < EPL; ++q) h[u][q] = h0[kOneTrip ? u : 0][q];
                        hb[u] = hb0[kOneTrip ? u : 0];
                        continue;
                    }
                    const int ss = sl + u < s1 ? sl + u : s0;
                    L::load(h[u], a.part_row, ss, D, sub);
                    hb[u] = a.has_bias ? a.part_bias[ss] : 0.0f;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (sl + u < s1) {
#pragma unroll
                        for (int q = 0; q < EPL; ++q) g[q] += h[u][q];
                        gb += hb[u];
                    }
                }
            }
        }
        if (MODE == kGradOnly) {
            const float *gbase;
            int64_t gkk, gbi;
            grad_loc(a, t, lr_, gk, nr, gbase, gkk, gbi);
            L::store(const_cast<float *>(gbase), gkk, D, sub, g);
            if (sub == 0) a.grad[gbi] = gb;
            return;
        }
    }

    if (LAZY && !(a.lazy_dbg & 1))   // every lane of the wave (item / skipped rows: nothing to catch up)
        catch_up<L>(a, wconst, wmax, lag, a.lazy_t, sub, p, m, v, pb, mb, vb);
    if (!proc || guarded) return;
#pragma unroll
    for (int q = 0; q < EPL; ++q) p[q] = opt_update(a.opt, p[q], g[q], m[q], v[q]);
    if (NT == 3) {          // optimizer state streamed past the caches, the new row kept (next gathers)
        L::store(a.w_out[t], lr_, D, sub, p);
        if (adam) L::store_nt(a.w_m[t], lr_, D, sub, m);
        if (has_v) L::store_nt(a.w_v[t], lr_, D, sub, v);
    } else if (NT >= 1) {
        L::store_nt(a.w_out[t], lr_, D, sub, p);
        if (adam) L::store_nt(a.w_m[t], lr_, D, sub, m);
        if (has_v) L::store_nt(a.w_v[t], lr_, D, sub, v);
    } else {
        L::store(a.w_out[t], lr_, D, sub, p);
        if (adam) L::store(a.w_m[t], lr_, D, sub, m);
        if (has_v) L::store(a.w_v[t], lr_, D, sub, v);
    }
    if (sub == 0 && a.has_bias) {
        pb = opt_update(a.opt, pb, gb, mb, vb);
        a.b_out[t][lr_] = pb;
        if (adam) a.b_m[t][lr_] = mb;
        if (has_v) a.b_v[t][lr_] = vb;
    }
    if (lz && sub == 0) {
        a.last_rel[r] = (int32_t)((int64_t)a.lazy_t - a.lazy_base);
        if (a.lazy_rows) atomicAdd(a.lazy_rows, 1ull);
    }
}

// Catch every lazily skipped user row up to step lazy_t (all of its cold updates), into the
// current set: the in-side tables of `a` (the set the last step wrote).  A row last updated
// at step ls holds its value in the set written then: the current one if lazy_t - ls is even
// (updated in place), else the other (a.w_out).
template <class L>
__global__ __launch_bounds__(kBlock) void mf_lazy_flush_kernel(ApplyArgs a) {
    constexpr int LPU = L::LPU, UPW = L::UPW, EPL = L::EPL;
    const int lane = threadIdx.x & (kWave - 1);
    const int sub = lane & (LPU - 1);
    const int64_t r = (((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6) * UPW + (lane / LPU);
    if (((((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6) * UPW) >= a.num_users) return;   // wave-uniform
    const bool in = r < a.num_users;
    const int32_t lsr = in ? a.last_rel[r] : 0;
    const int lag = in ? (int)((int64_t)a.lazy_t - a.lazy_base - lsr) : 0;
    const int D = a.dim;
    const bool adam = a.opt.kind == RG_OPT_ADAM;
    const bool has_v = a.opt.kind != RG_OPT_SGD;
    const float *src_w = (lag & 1) ? a.w_out[0] : a.w_in[0];
    const float *src_b = (lag & 1) ? a.b_out[0] : a.b_in[0];
    const int64_t rr = in ? r : 0;
    float p[EPL], m[EPL], v[EPL];
    float pb = 0.0f, mb = 0.0f, vb = 0.0f;
    L::zero(p); L::zero(m); L::zero(v);
    if (lag > 0) {              // current rows are read and written by nobody
        L::load(p, src_w, rr, D, sub);
        if (adam) L::load(m, a.w_m[0], rr, D, sub);
        if (has_v) L::load(v, a.w_v[0], rr, D, sub);
        if (sub == 0) {
            pb = src_b[rr];
            if (adam) mb = a.b_m[0][rr];
            if (has_v) vb = a.b_v[0][rr];
        }
    }
    // steps [lazy_t + 1 - lag, lazy_t] (the flush's window ends at lazy_t itself)
    const int wmax = wave_max(lag > 0 ? lag : 0);
    const float2 wc = wmax > 0 ? window_const(a, (int64_t)a.lazy_t + 1 - wmax, wmax) : make_float2(0.0f, 0.0f);
    catch_up<L>(a, wc, wmax, lag > 0 ? lag : 0, (int64_t)a.lazy_t + 1, sub, p, m, v, pb, mb, vb);
    if (lag <= 0) return;
    L::store(const_cast<float *>(a.w_in[0]), r, D, sub, p);
    if (adam) L::store(a.w_m[0], r, D, sub, m);
    if (has_v) L::store(a.w_v[0], r, D, sub, v);
    if (sub == 0) {
        const_cast<float *>(a.b_in[0])[r] = pb;
        if (adam) a.b_m[0][r] = mb;
        if (has_v) a.b_v[0][r] = vb;
        a.last_rel[r] = (int32_t)((int64_t)a.lazy_t - a.lazy_base);
    }
}

// Streams every row of [row_begin, row_end) once (item rows first, so the few
// long Zipf-hot item rows start early instead of trailing the grid).
// NT: 1 = streaming stores of the updated p, m, v; 2 = also streaming loads of the
// pre-step p, m, v (each touched once per step)
template <class L, int MODE, int NT = 0, bool SPEC = false>
__global__ __launch_bounds__(kBlock) void mf_apply_kernel(ApplyArgs a) {
    constexpr int LPU = L::LPU, UPW = L::UPW;
    const int lane = threadIdx.x & (kWave - 1);
    const int sub = lane & (LPU - 1);
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t k = wave * UPW + (lane / LPU);
    const int64_t rb = a.row_begin, re = a.row_end, nr = re - rb;
    const int D = a.dim;

    const int64_t slot_off = (a.shard_users + a.shard_items) * (int64_t)(D + 1);   // loss slot in a chunk
    if (MODE != kApplyDense && a.loss_out != nullptr && blockIdx.x == 0) {
        const float lv = finalize_loss_wg<kBlock>(a.partials, a.n_partials, a.inv_a, a.inv_b);
        if (threadIdx.x < kWave) {
            if (lane == 0) *a.loss_out = lv;
            if (MODE == kGradOnly && (a.shard_users > 0 || a.item_shard)) {
                for (int s = lane; s < a.world; s += kWave) a.grad[s * a.chunk + slot_off] = lv;   // summed by the RS
            } else if (MODE == kGradOnly && lane == 0) {
                a.grad[nr * (int64_t)(D + 1)] = lv;
            }
        }
    }
    if (MODE == kApplyDense && a.loss_out != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
        *a.loss_out = (a.shard_users > 0 || a.item_shard) ? a.grad[a.rank * a.chunk + slot_off]
                                                         : a.grad[nr * (int64_t)(D + 1)];

    if (k >= nr) return;
    int64_t r;
    if (MODE == kApplyDense && a.item_shard) {
        r = a.num_users + a.rank * a.shard_items + k;         // this rank's item shard only
    } else if (MODE == kApplyDense && a.shard_users > 0) {
        // this rank's shard: [rb, rb + nu) users, then items from U + rank * Is
        const int64_t u0 = a.rank * a.shard_users, i0 = a.rank * a.shard_items;
        const int64_t u1 = u0 + a.shard_users < a.num_users ? u0 + a.shard_users : a.num_users;
        const int64_t nu = u1 > u0 ? u1 - u0 : 0;
        r = k < nu ? u0 + k : a.num_users + i0 + (k - nu);
    } else {
        const int64_t ia0 = rb > a.num_users ? rb : a.num_users;      // item part [ia0, re)
        const int64_t ni = re > ia0 ? re - ia0 : 0;
        r = k < ni ? ia0 + k : rb + (k - ni);
    }
    apply_row<L, MODE, NT, false, SPEC>(a, r, sub);
}

// the dense update of rows [row_begin, row_end) (blocks [0, apply_blocks), as
// mf_apply_kernel) and the prepare pass of the NEXT step (the remaining blocks) in one
// launch: the split step then needs no side stream and no per-step cross-stream event
// Optional: workgroup 0 walks a LATER step's MT19937 words (rg_mt_gen_t) -- the walk
// (~0.47 ns/word, one workgroup) hides under the HBM-bound pass, so a single-GPU step
// needs no generator stream and no cross-stream event.
struct MtGenArgs {
    uint32_t *state, *out, *state_before;
    int64_t nwords;
};

// Grid of mf_back_kernel: [MT walk block (optional)] [prepare blocks] [padding] [apply
// blocks, apply_padded = a multiple of 8 starting at an absolute index that is one].
// Workgroups go to the 8 XCDs round-robin by absolute index, so with xcd_map the apply
// block of absolute index B processes row group (B % 8) * apply_padded / 8 + B / 8: each
// XCD streams one contiguous eighth of the rows, and the per-row small arrays (biases,
// counts: 4 B per row, 16 B per wave) fill whole lines in ONE XCD's L2 instead of each
// line being fetched and partially written back by all eight.
struct BackGrid {
    int64_t prep_blocks, apply_start, apply_padded;
    int32_t prep_first, xcd_map;
    int64_t upd_blocks;   // NCF step: MLP update workgroups after the prepare's (rg_ncf_tail)
};

template <class L, int NT, bool SPEC = false, bool OWN = false, bool LAZY = false, bool LSPEC = false>
#ifdef RG_BACK_WAVES
#define RG_BACK_ATTR __attribute__((amdgpu_waves_per_eu(RG_BACK_WAVES, 8)))
#else
#define RG_BACK_ATTR
#endif
__global__ __launch_bounds__(kBlock) RG_BACK_ATTR void mf_back_kernel(ApplyArgs a, PairsArgs prep, int2 *prep_out,
                                                        int64_t apply_blocks, MtGenArgs gen, BackGrid bg,
                                                        OwnerArgs own, MlpUpdArgs upd) {
    static_assert(kBlock == kOwnSeg, "an owner prepare segment is one workgroup");
    static_assert(kBlock == kGenThreads, "the MT walk runs on one full workgroup");
    const int64_t B = blockIdx.x;
    int64_t blk = B;
    if (gen.nwords > 0) {
        if (B == 0) {
            __shared__ uint32_t X[kRing + 2];
            mt_generate_block(X, gen.state, gen.out, gen.nwords, gen.state_before);
            return;
        }
        --blk;
    }
    // the next step's prepare (latency-bound random pool reads) in the FIRST blocks, so it
    // overlaps the streaming rows instead of trailing the grid (RG_PREP_FIRST=0: last)
    if (bg.prep_first) {
        if (blk < bg.prep_blocks) {
            if (OWN) owner_prepare_block(own, blk);
            else prepare_one(prep, prep_out, blk * kBlock + threadIdx.x);
            return;
        }
        if (blk < bg.prep_blocks + bg.upd_blocks) {             // the NCF step's MLP update
            __shared__ float red[kMlpSlices][64];
            mlp_update_block<kBlock / kWave>(upd, blk - bg.prep_blocks, red);
            return;
        }
        if (B < bg.apply_start) return;                         // alignment padding
        blk = B - bg.apply_start;
        if (bg.xcd_map) blk = (blk & 7) * (bg.apply_padded >> 3) + (blk >> 3);
        if (blk >= apply_blocks) return;
    } else if (blk >= apply_blocks) {
        if (OWN) owner_prepare_block(own, blk - apply_blocks);
        else prepare_one(prep, prep_out, (blk - apply_blocks) * kBlock + threadIdx.x);
        return;
    }
    constexpr int LPU = L::LPU, UPW = L::UPW;
    const int lane = threadIdx.x & (kWave - 1);
    const int sub = lane & (LPU - 1);
    const int64_t wave = (blk * kBlock + threadIdx.x) >> 6;
    const int64_t k = wave * UPW + (lane / LPU);
    const int64_t rb = a.row_begin, re = a.row_end, nr = re - rb;
    if (a.loss_out != nullptr && blk == 0 && threadIdx.x < kWave) {
        const float lv = finalize_loss(a.partials, a.n_partials, a.inv_a, a.inv_b, lane);
        if (lane == 0) *a.loss_out = lv;
    }
    const int64_t ia0 = rb > a.num_users ? rb : a.num_users;      // item rows first, as mf_apply_kernel
    const int64_t ni = re > ia0 ? re - ia0 : 0;
    const int64_t r = k < ni ? ia0 + k : rb + (k - ni);
    if (LAZY) {
        // a user row's decision words first (the row's loads depend on them)
        if ((wave * UPW) >= nr) return;                     // wave-uniform: the catch-up loop is per wave
        const bool in = k < nr;
        const int64_t rr = in ? r : rb;
        LazyRow lzr{0, 0, 0, in};
        if (in && rr < a.num_users) {
            lzr.cnt = a.row_count[rr];
            lzr.mk = a.umark[rr];
            lzr.lsr = a.last_rel[rr];
        }
        // a lane group past the end runs as an inactive user row (row 0: no loads, no stores)
        apply_row<L, kApplyPull, NT, false, SPEC, true, LSPEC>(a, in ? r : 0, sub, lzr);
        return;
    }
    if (k >= nr) return;
    apply_row<L, kApplyPull, NT, false, SPEC>(a, r, sub);
}

// ---------------------------------------------------------------------------- two-launch pipelined step
// The single-GPU step as two launches per step t, overlapping step t+1's latency-bound pair pass
// with the HBM-bound update of the rows that pass does not read:
//
//   hot launch  (mf_pipe2_hot_kernel):  the dense update of step t for every item row and for the
//               users step t+1's pair pass reads (its prepare's hot list); step t's loss
//   cold launch (mf_pipe2_cold_kernel): [step t+1's pair pass] [the MT walk of a later unit]
//               [step t+2's prepare, appending its hot list] [the dense update of step t for every
//               other user (its claim count of step t+1 is zero)]
//
// The pair pass reads only rows the hot launch wrote (stream order: no gate, no spin), and the
// cold rows it leaves to the same launch are rows it does not read.  Per-row and per-column
// arithmetic is the split step's, so results are bit-identical to it.  A unit's scratch alternates
// by parity (claims in three count arrays, lists / overflow accumulators / partials in two sets:
// rg_stepper.cpp train_pipe2).
struct Pipe2Args {
    const int32_t *hot;           // hot launch: the users step t+1's pair pass reads
    const int32_t *nhot;          // hot launch: their number (device)
    int64_t hot_blocks, item_blocks;
    int32_t *nhot_clear;          // hot launch: zeroed (the list the cold launch's prepare appends to)
    const int32_t *counts_next;   // cold launch: step t+1's claims (a user with one is hot)
    int64_t pair_blocks, prep_blocks, cold_blocks;
};

template <class LD>
__global__ __launch_bounds__(kBlock) void mf_pipe2_hot_kernel(ApplyArgs a, Pipe2Args p, MtGenArgs gen) {
    int64_t blk = blockIdx.x;
    if (gen.nwords > 0) {
        if (blk == 0) {
            __shared__ uint32_t X[kRing + 2];
            mt_generate_block(X, gen.state, gen.out, gen.nwords, gen.state_before);
            return;
        }
        --blk;
    }
    constexpr int LPU = LD::LPU, UPW = LD::UPW;
    const int lane = threadIdx.x & (kWave - 1);
    const int sub = lane & (LPU - 1);
    if (blk == 0) {
        if (threadIdx.x == 0 && p.nhot_clear != nullptr) *p.nhot_clear = 0;
        if (a.loss_out != nullptr && threadIdx.x >= kWave && threadIdx.x < 2 * kWave) {
            const float lv = finalize_loss(a.partials, a.n_partials, a.inv_a, a.inv_b, lane);   // step t's loss
            if (lane == 0) *a.loss_out = lv;
        }
    }
    constexpr int64_t rpb = (kBlock / kWave) * UPW;
    const int64_t in_block = (threadIdx.x >> 6) * UPW + lane / LPU;
    int64_t r;
    if (blk < p.item_blocks) {
        const int64_t k = blk * rpb + in_block;
        if (k >= a.num_items) return;
        r = a.num_users + k;
    } else {
        const int64_t j = (blk - p.item_blocks) * rpb + in_block;
        if (j >= (int64_t)*p.nhot) return;
        r = p.hot[j];
    }
    apply_row<LD, kApplyPull, 0, false, true>(a, r, sub);
}

template <class LP, class LD, int NMAX>
__global__ __launch_bounds__(kBlock) void mf_pipe2_cold_kernel(ApplyArgs a, PairsArgs pa, PairsArgs prep,
                                                               int2 *prep_out, Pipe2Args p, MtGenArgs gen) {
    static_assert(kPairBlock == kBlock, "the pair workgroups share the launch's block size");
    int64_t blk = blockIdx.x;
    if (blk < p.pair_blocks) {                  // first in the grid: the step's latency chain
        pairs_body<LP, kFused, NMAX>(pa, blk);
        return;
    }
    blk -= p.pair_blocks;
    if (gen.nwords > 0) {
        if (blk == 0) {
            __shared__ uint32_t X[kRing + 2];
            mt_generate_block(X, gen.state, gen.out, gen.nwords, gen.state_before);
            return;
        }
        --blk;
    }
    if (blk < p.prep_blocks) {
        prepare_one(prep, prep_out, blk * kBlock + threadIdx.x);
        return;
    }
    blk -= p.prep_blocks;
    constexpr int LPU = LD::LPU, UPW = LD::UPW;
    const int lane = threadIdx.x & (kWave - 1);
    const int sub = lane & (LPU - 1);
    const int64_t u = blk * ((kBlock / kWave) * UPW) + (threadIdx.x >> 6) * UPW + lane / LPU;
    if (u >= a.num_users) return;
#ifdef RG_PIPE2_CHECK_FIRST   // timing experiments: the hot test as a round trip of its own
    if (p.counts_next[u] > 0) return;
    apply_row<LD, kApplyPull, 0, false, true>(a, u, sub);
#else
    // a user with a claim of step t+1 was updated by the hot launch: its guard is loaded beside its
    // other loads (wasted bytes for it, but no round trip in front of every row)
    apply_row<LD, kApplyPull, 0, false, true, false, false, true>(a, u, sub);
#endif
}


// The single-GPU dense pass as a software pipeline (the default split step): a grid of a few
// workgroups per CU whose waves each walk a contiguous chunk of row groups (UPW rows per group),
// the NEXT group's independent loads (p, m, v, biases, count, list entries, slot range) issued
// before this group's dependent ones (partner rows, planned partials).  One memory round trip
// per group instead of two: in mf_back_kernel a touched row's wave waited for its list, then for
// its partner rows, with nothing else in flight (rows with a contribution are ~40 % of all,
// ~87 % of the 4-row groups).  Grid as mf_back_kernel's: [MT walk] [next prepare] [pad] [dense].
template <class L>
__global__ __launch_bounds__(kBlock) void mf_dense_kernel(ApplyArgs a, PairsArgs prep, int2 *prep_out,
                                                          int64_t dense_blocks, MtGenArgs gen, BackGrid bg) {
    const int64_t B = blockIdx.x;
    int64_t blk = B;
    if (gen.nwords > 0) {
        if (B == 0) {
            __shared__ uint32_t X[kRing + 2];
            mt_generate_block(X, gen.state, gen.out, gen.nwords, gen.state_before);
            return;
        }
        --blk;
    }
    if (blk < bg.prep_blocks) {
        prepare_one(prep, prep_out, blk * kBlock + threadIdx.x);
        return;
    }
    if (B < bg.apply_start) return;                         // alignment padding
    blk = B - bg.apply_start;
    if (blk >= dense_blocks) return;
    constexpr int LPU = L::LPU, UPW = L::UPW;
    const int lane = threadIdx.x & (kWave - 1);
    const int sub = lane & (LPU - 1);
    const int64_t rb = a.row_begin, re = a.row_end, nr = re - rb;
    if (a.loss_out != nullptr && blk == 0 && threadIdx.x < kWave) {
        const float lv = finalize_loss(a.partials, a.n_partials, a.inv_a, a.inv_b, lane);
        if (lane == 0) *a.loss_out = lv;
    }
    const int64_t ia0 = rb > a.num_users ? rb : a.num_users;      // item rows first, as mf_apply_kernel
    const int64_t ni = re > ia0 ? re - ia0 : 0;
    // this wave's row groups [g0, g1): contiguous, so a wave's stores fill whole lines
    const int64_t waves = dense_blocks * (kBlock / kWave);
    const int64_t wave = (blk * kBlock + threadIdx.x) >> 6;
    const int64_t groups = (nr + UPW - 1) / UPW;
    const int64_t per = (groups + waves - 1) / waves;
    const int64_t g0 = wave * per, g1 = g0 + per < groups ? g0 + per : groups;
    if (g0 >= g1) return;                                   // wave-uniform
    auto row_of = [&](int64_t g, bool &valid) {
        const int64_t k = g * UPW + lane / LPU;
        valid = k < nr;
        const int64_t kk = valid ? k : 0;
        return kk < ni ? ia0 + kk : rb + (kk - ni);
    };
    LeanRow<L> cur, nxt;
    bool vc, vn;
    int64_t rc = row_of(g0, vc), rn = 0;
    lean_load<L>(a, rc, sub, vc, cur);
    for (int64_t g = g0; g < g1; ++g) {
        const bool more = g + 1 < g1;                       // wave-uniform
        if (more) {
            rn = row_of(g + 1, vn);
            lean_load<L>(a, rn, sub, vn, nxt);
        }
        lean_finish<L>(a, rc, sub, vc, cur);
        if (!more) break;
        cur = nxt;
        rc = rn;
        vc = vn;
    }
}

// ---------------------------------------------------------------------------- pipelined step
// One launch per training step t that also runs the pair pass of step t + 1 and the prepare of
// step t + 2 (rg_mf_pipe_step, the stepper's default single-GPU step):
//
//   [prepare t+2]  the next-but-one step's draws -> pool pairs, list-slot claims, and the list
//                  of users it claims a first slot of (the users pair pass t+2 will read)
//   [hot items]    the dense update of every item row              } the rows pair pass t+1
//   [hot users]    the dense update of the users of step t+1's list } reads; write-through
//                  stores, then each workgroup adds 1 to the gate
//   [cold users 1] the dense update of the other users
//   [pair t+1]     waits until the gate counts every hot workgroup, then runs step t+1's pair
//                  pass on the updated rows (loads past L1) beside the cold stream
//   [cold users 2]
//
// The latency-bound pair pass (~11 us on its own) thus overlaps the HBM-bound update of the rows
// it does not read.  Deadlock-free by construction: only pair workgroups wait, on workgroups that
// never wait, and they are too few (cols / units-per-workgroup) to hold every slot of the chip.
// Results are bit-identical to the split step (same per-row and per-column arithmetic).
struct PipeArgs {
    const int32_t *hot_users, *nhot;   // step t+1's hot user list
    const int32_t *counts_next;        // step t+1's claims (a user with one is hot)
    int32_t *gate, *gate_next, *nhot_free, *err;
    int64_t prep_blocks, item_blocks, huser_blocks, cold1_blocks, pair_blocks, cold2_blocks;
    int64_t users_begin;               // unified row of user 0 in the dense rows (0)
    uint32_t spin_limit;
};

template <class L, bool WT>
__device__ __forceinline__ void pipe_rows(const ApplyArgs &a, const int64_t r, const bool valid, const int sub) {
    LeanRow<L> x;
    lean_load<L>(a, r, sub, valid, x);
    lean_finish<L, WT>(a, r, sub, valid, x);
}

template <class L, int NMAX>
__global__ __launch_bounds__(kBlock) void mf_pipe_kernel(ApplyArgs a, PairsArgs pa, PairsArgs prep, int2 *prep_out,
                                                         PipeArgs pp, MtGenArgs gen) {
    static_assert(kPairBlock == kBlock, "the pair workgroups share the launch's block size");
    constexpr int LPU = L::LPU, UPW = L::UPW;
    int64_t blk = blockIdx.x;
    if (gen.nwords > 0) {
        if (blk == 0) {
            __shared__ uint32_t X[kRing + 2];
            mt_generate_block(X, gen.state, gen.out, gen.nwords, gen.state_before);
            return;
        }
        --blk;
    }
    const int lane = threadIdx.x & (kWave - 1);
    const int sub = lane & (LPU - 1);
    const int64_t rows_per_block = (kBlock / kWave) * UPW;
    const int64_t U = a.num_users;
    if (blk < pp.prep_blocks) {                              // prepare of step t + 2
        if (blk == 0 && threadIdx.x == 0) {                  // counters of later launches
            *pp.gate_next = 0;
            *pp.nhot_free = 0;
        }
        if (blk == 0 && a.loss_out != nullptr && threadIdx.x >= kWave && threadIdx.x < 2 * kWave) {
            const float lv = finalize_loss(a.partials, a.n_partials, a.inv_a, a.inv_b, lane);   // step t's loss
            if (lane == 0) *a.loss_out = lv;
        }
        prepare_one(prep, prep_out, blk * kBlock + threadIdx.x);
        return;
    }
    blk -= pp.prep_blocks;
    const int64_t in_block = (threadIdx.x >> 6) * UPW + lane / LPU;   // row slot of this lane group
    const bool hot = blk < pp.item_blocks + pp.huser_blocks;
    int64_t row = 0;
    bool valid = false;
    if (hot) {                                               // the rows pair pass t + 1 reads
        if (blk < pp.item_blocks) {
            const int64_t k = blk * rows_per_block + in_block;
            valid = k < a.num_items;
            row = U + (valid ? k : 0);
        } else {
            const int64_t k = (blk - pp.item_blocks) * rows_per_block + in_block;
            valid = k < *pp.nhot;
            row = valid ? (int64_t)pp.hot_users[k] : 0;
        }
    } else {
        blk -= pp.item_blocks + pp.huser_blocks;
        int64_t cold;
        if (blk < pp.cold1_blocks) {
            cold = blk;
        } else if (blk < pp.cold1_blocks + pp.pair_blocks) {     // pair pass of step t + 1
        const int64_t pb = blk - pp.cold1_blocks;
#ifdef RG_PIPE_X   // timing experiments only (wrong results): bit 0 no pair pass, bit 1 no wait either
        if (RG_PIPE_X & 2) return;
#endif
        if (threadIdx.x == 0) {
            const int target = (int)(pp.item_blocks + pp.huser_blocks);
            uint32_t spins = 0;
            while (__hip_atomic_load(pp.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(8);
                if (++spins > pp.spin_limit) {               // bounded: flag and go on (wrong results)
                    atomicOr(pp.err, 1);
                    break;
                }
            }
        }
        __syncthreads();
#ifdef RG_PIPE_X
        if (RG_PIPE_X & 1) return;
#endif
        pairs_body<L, kFused, NMAX, true>(pa, pb);
        return;
        } else {
            cold = blk - pp.pair_blocks;
        }
        // cold users: chunk `cold` of the user rows, minus the hot ones
        const int64_t u = cold * rows_per_block + in_block;
        valid = u < U && pp.counts_next[u] <= 0;
        row = valid ? u : 0;
    }
    if (__any(valid)) {
        if (hot) pipe_rows<L, true>(a, row, valid, sub);   // read by the pair pass: write-through
        else pipe_rows<L, false>(a, row, valid, sub);
    }
    if (hot) {   // publish: every wave's write-through stores done, then one add for the workgroup
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(pp.gate, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---------------------------------------------------------------------------- overlapped step
// One training step as two launches instead of prepare / pairs / apply:
//
//   mf_front_kernel  blocks [0, P)        the pair pass of this step (pairs_body)
//                    blocks [P, P + Q)    the prepare pass of the NEXT step (stamps
//                                         the rows it will touch with its serial)
//                    blocks [P + Q, ...)  the optimizer update of every COLD row of
//                                         this step (stamp != this step's serial):
//                                         zero data gradient, so it needs nothing
//                                         from the pair pass and streams beside it
//   mf_hot_kernel    the update of the touched rows, one per owner flag of the
//                    prepared pairs, pulling the pair pass's lists / partials
//
// The latency-bound pair pass (gathers, atomics, LDS) thus hides under two thirds
// of the HBM-bound dense optimizer pass instead of preceding all of it.
struct FrontArgs {
    int64_t pair_blocks, prep_blocks;
    int2 *prep_out;                 // next step's pairs buffer (prep_blocks > 0)
    const int32_t *cold_stamp;      // this step's stamps
    int32_t cold_serial;
};

template <class L, int NMAX>
__global__ __launch_bounds__(kBlock) void mf_front_kernel(PairsArgs pa, PairsArgs prep, ApplyArgs aa, FrontArgs f) {
    const int64_t blk = blockIdx.x;
    if (blk < f.pair_blocks) {
        if constexpr (kPairBlock == kBlock) pairs_body<L, kFused, NMAX>(pa, blk);   // (host refuses otherwise)
        return;
    }
    if (blk < f.pair_blocks + f.prep_blocks) {
        prepare_one(prep, f.prep_out, (blk - f.pair_blocks) * kBlock + threadIdx.x);
        return;
    }
    constexpr int LPU = L::LPU, UPW = L::UPW;
    const int lane = threadIdx.x & (kWave - 1);
    const int sub = lane & (LPU - 1);
    const int64_t wave = ((blk - f.pair_blocks - f.prep_blocks) * kBlock + threadIdx.x) >> 6;
    const int64_t r = aa.row_begin + wave * UPW + (lane / LPU);
    if (r >= aa.row_end) return;
    if (f.cold_stamp[r] == f.cold_serial) return;           // touched: mf_hot_kernel
    apply_row<L, kApplyPull, 0, true>(aa, r, sub);
}

// the cold-row update of the front grid as a launch of its own (two-stream schedule:
// beside rg_mf_pairs on another stream, at its own register budget)
template <class L>
__global__ __launch_bounds__(kBlock) void mf_cold_kernel(ApplyArgs a, const int32_t *__restrict__ stamp,
                                                        int32_t serial) {
    constexpr int LPU = L::LPU, UPW = L::UPW;
    const int lane = threadIdx.x & (kWave - 1);
    const int sub = lane & (LPU - 1);
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t r = a.row_begin + wave * UPW + (lane / LPU);
    if (r >= a.row_end) return;
    if (stamp[r] == serial) return;
    apply_row<L, kApplyPull, 0, true>(a, r, sub);
}

// row-ordered variant: scan the rows, update those stamped with this step's serial
// (sequential addresses with holes instead of the pairs' random order)
template <class L>
__global__ __launch_bounds__(kBlock) void mf_hot_scan_kernel(ApplyArgs a, const int32_t *__restrict__ stamp,
                                                            int32_t serial) {
    constexpr int LPU = L::LPU, UPW = L::UPW;
    const int lane = threadIdx.x & (kWave - 1);
    const int sub = lane & (LPU - 1);
    if (a.loss_out != nullptr && blockIdx.x == 0 && threadIdx.x < kWave) {
        const float lv = finalize_loss(a.partials, a.n_partials, a.inv_a, a.inv_b, lane);
        if (lane == 0) *a.loss_out = lv;
    }
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t r = a.row_begin + wave * UPW + (lane / LPU);
    if (r >= a.row_end) return;
    if (stamp[r] != serial) return;
    apply_row<L, kApplyPull, 0, false>(a, r, sub);
}

// slot k = (pair k >> 1, side k & 1): the row the slot's pair touches on that side,
// updated here iff the slot owns it (exactly one owner per touched row)
template <class L>
__global__ __launch_bounds__(kBlock) void mf_hot_kernel(ApplyArgs a, const int2 *__restrict__ pairs, int64_t n_slots,
                                                       int stride, int np_) {
    constexpr int LPU = L::LPU, UPW = L::UPW;
    const int lane = threadIdx.x & (kWave - 1);
    const int sub = lane & (LPU - 1);
    if (a.loss_out != nullptr && blockIdx.x == 0 && threadIdx.x < kWave) {
        const float lv = finalize_loss(a.partials, a.n_partials, a.inv_a, a.inv_b, lane);
        if (lane == 0) *a.loss_out = lv;
    }
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t k = wave * UPW + (lane / LPU);
    if (k >= n_slots) return;
    if ((int)((k >> 1) % stride) >= np_) return;   // a record's plan-slot / padding entries
    const int2 pr = pairs[k >> 1];
    const int32_t x = (k & 1) ? pr.y : pr.x;
    if (x >= 0) return;                                     // owner flag (bit 31) not set
    const int64_t r = (k & 1) ? a.num_users + (x & kIdMask) : (int64_t)(x & kIdMask);
    if (r < a.row_begin || r >= a.row_end) return;
    apply_row<L, kApplyPull, 0, false>(a, r, sub);
}

// ---------------------------------------------------------------------------- scores / loss
template <class L>
__global__ __launch_bounds__(kBlock) void mf_scores_kernel(const float *__restrict__ uw, const float *__restrict__ iw,
                                                           const float *__restrict__ ub, const float *__restrict__ ib,
                                                           int D, const int64_t *__restrict__ users,
                                                           const int64_t *__restrict__ items, int64_t n,
                                                           float *__restrict__ out) {
    constexpr int LPU = L::LPU, EPL = L::EPL, UPW = L::UPW;
    const int lane = threadIdx.x & (kWave - 1);
    const int sub = lane & (LPU - 1);
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t k = wave * UPW + (lane / LPU);
    float ur[EPL], ir[EPL];
    L::zero(ur);
    L::zero(ir);
    int64_t u = 0, i = 0;
    if (k < n) {
        u = users[k];
        i = items[k];
        L::load(ur, uw, u, D, sub);
        L::load(ir, iw, i, D, sub);
    }
    float d = 0.0f;
#pragma unroll
    for (int e = 0; e < EPL; ++e) d = fmaf(ur[e], ir[e], d);
    d = group_sum<LPU>(d);      // all lanes converged here (DPP)
    if (k < n && sub == 0) out[k] = sigmoidf_ref((d + ub[u]) + ib[i]);
}

__global__ __launch_bounds__(kWave) void loss_finalize_kernel(const float *__restrict__ partials, int64_t np_,
                                                              double inv_a, double inv_b, float *out) {
    const float lv = finalize_loss(partials, np_, inv_a, inv_b, threadIdx.x);
    if (threadIdx.x == 0) *out = lv;
}

template <class L>
int64_t pairs_blocks(int64_t cols) {
    constexpr int64_t UPB = kPairBlock / L::LPU;
    return (cols + UPB - 1) / UPB;
}

}  // namespace rg

using namespace rg;

namespace {
struct PartialsLenF {
    int64_t cols;
    int64_t *nb;
    template <class L>
    int operator()() { *nb = pairs_blocks<typename PairLayout<L>::type>(cols); return 0; }
};

struct UnitsPerBlockF {
    int64_t *upb;
    template <class L>
    int operator()() { *upb = kPairBlock / PairLayout<L>::type::LPU; return 0; }
};

struct PairsLaunchF {
    PairsArgs *a;
    hipStream_t s;
    bool adaptive, backward;
    template <class L0>
    int operator()() {
        using L = typename PairLayout<L0>::type;
        if (a->n_neg <= 5) return run<L, 5>();
        return run<L, kNMax>();
    }
    template <class L, int NMAX>
    int run() {
        const int64_t nb = pairs_blocks<L>(a->cols);
        if (!adaptive) {
            if (backward)
                hipLaunchKernelGGL((mf_pairs_kernel<L, kFused, NMAX>), dim3(nb), dim3(kPairBlock), 0, s, *a);
            else
                hipLaunchKernelGGL((mf_pairs_kernel<L, kLossOnly, NMAX>), dim3(nb), dim3(kPairBlock), 0, s, *a);
            return check_launch("rg_mf_pairs");
        }
        if (hipMemsetAsync(a->max_key, 0, sizeof(unsigned long long), s) != hipSuccess ||
            hipMemsetAsync(a->active_count, 0, sizeof(int32_t), s) != hipSuccess)
            return check_launch("rg_mf_pairs(adaptive memset)");
        hipLaunchKernelGGL((mf_pairs_kernel<L, kAdaptFwd, NMAX>), dim3(nb), dim3(kPairBlock), 0, s, *a);
        if (backward) {
            hipLaunchKernelGGL((mf_pairs_kernel<L, kAdaptBwd, NMAX>), dim3(nb), dim3(kPairBlock), 0, s, *a);
            hipLaunchKernelGGL((mf_adapt_max_kernel<L>), dim3(1), dim3(kWave), 0, s, *a);
        } else {
            hipLaunchKernelGGL((mf_pairs_kernel<L, kAdaptLoss, NMAX>), dim3(nb), dim3(kPairBlock), 0, s, *a);
        }
        return check_launch("rg_mf_pairs(adaptive)");
    }
};

struct ApplyLaunchF {
    ApplyArgs *a;
    hipStream_t s;
    int mode;
    template <class L>
    int operator()() {
        // MF rows (not NCF's contribution rows) on the dense pass's layout: the item gradient and
        // item update of the data-parallel steps, element-wise like the dense pass
        using LB = typename BackLayout<L>::type;
        if constexpr (!std::is_same<LB, L>::value) {
            if (a->contrib == nullptr) return run<LB>();
        }
        return run<L>();
    }
    template <class L>
    int run() {
        const int64_t rows = a->row_end - a->row_begin;
        if (rows <= 0 && a->loss_out == nullptr) return RG_OK;
        const int64_t waves = (rows + L::UPW - 1) / L::UPW;
        int64_t nb = (waves + kBlock / kWave - 1) / (kBlock / kWave);
        if (nb < 1) nb = 1;
#if RG_AB
        // A/B build only (measured no faster): non-temporal stores, the list loaded
        // beside the count
        static const int nt = [] { const char *e = getenv("RG_APPLY_NT"); return e ? atoi(e) : 0; }();
        static const int spec = [] { const char *e = getenv("RG_APPLY_SPEC"); return e ? atoi(e) : 0; }();
        if (mode == kApplyPull && spec && nt == 1)
            hipLaunchKernelGGL((mf_apply_kernel<L, kApplyPull, 1, true>), dim3(nb), dim3(kBlock), 0, s, *a);
        else if (mode == kApplyPull && spec)
            hipLaunchKernelGGL((mf_apply_kernel<L, kApplyPull, 0, true>), dim3(nb), dim3(kBlock), 0, s, *a);
        else if (mode == kApplyPull && nt == 1)
            hipLaunchKernelGGL((mf_apply_kernel<L, kApplyPull, 1>), dim3(nb), dim3(kBlock), 0, s, *a);
        else if (mode == kApplyPull && nt >= 2)
            hipLaunchKernelGGL((mf_apply_kernel<L, kApplyPull, 2>), dim3(nb), dim3(kBlock), 0, s, *a);
        else
#endif
        if (mode == kApplyPull)
            hipLaunchKernelGGL((mf_apply_kernel<L, kApplyPull>), dim3(nb), dim3(kBlock), 0, s, *a);
        else if (mode == kGradOnly)   // list and slot range loaded beside the count
            hipLaunchKernelGGL((mf_apply_kernel<L, kGradOnly, 0, true>), dim3(nb), dim3(kBlock), 0, s, *a);
        else
            hipLaunchKernelGGL((mf_apply_kernel<L, kApplyDense>), dim3(nb), dim3(kBlock), 0, s, *a);
        return check_launch("rg_mf_apply");
    }
};

struct ScoresLaunchF {
    const float *uw, *iw, *ub, *ib;
    int dim;
    const int64_t *users, *items;
    int64_t n;
    float *out;
    hipStream_t s;
    template <class L>
    int operator()() {
        const int64_t waves = (n + L::UPW - 1) / L::UPW;
        const int64_t nb = (waves + kBlock / kWave - 1) / (kBlock / kWave);
        hipLaunchKernelGGL((mf_scores_kernel<L>), dim3(nb), dim3(kBlock), 0, s, uw, iw, ub, ib, dim, users, items,
                           n, out);
        return check_launch("rg_mf_scores");
    }
};
}  // namespace

extern "C" int64_t rg_mf_pairs_len(int64_t cols, int32_t n_neg) {
    if (cols <= 0 || n_neg < 1 || n_neg > kNMax) return -1;
    return 2 * (int64_t)pair_stride(n_neg) * cols;
}

extern "C" int64_t rg_mf_partials_len(int64_t cols, int32_t dim) {
    int64_t nb = -1;
    PartialsLenF f{cols, &nb};
    if (dispatch_dim(dim, f) != 0) return -1;
    return 2 * nb;
}

extern "C" int64_t rg_mf_plan_units_per_block(int32_t dim) {
    int64_t upb = -1;
    UnitsPerBlockF f{&upb};
    if (dispatch_dim(dim, f) != 0) return -1;
    return upb;
}

static int check_tables(const rg_mf_tables_t *t) {
    if (t == nullptr) return fail_arg("null tables");
    if (!t->user_w || !t->item_w || !t->user_b || !t->item_b) return fail_arg("null parameter table");
    if (t->num_users <= 0 || t->num_items <= 0) return fail_arg("empty table");
    if (t->num_users + t->num_items >= (int64_t)1 << 31) return fail_arg("num_users + num_items must be < 2^31");
    if (t->dim < 1 || t->dim > 256) return fail_arg("dim must be in [1, 256]");
    return RG_OK;
}

static int pairs_args(const rg_mf_tables_t *t, const rg_mf_batch_t *b, const rg_mf_work_t *w, int32_t backward,
                      PairsArgs &a) {
    int rc = check_tables(t);
    if (rc) return rc;
    if (b == nullptr || w == nullptr) return fail_arg("rg_mf_pairs: null batch/work");
    if (b->n_neg < 1 || b->n_neg > kNMax) return fail_arg("rg_mf_pairs: n_neg must be in [1, 8]");
    if (b->cols <= 0 || b->n_pos < 0 || b->n_pos > b->cols) return fail_arg("rg_mf_pairs: bad n_pos/cols");
    if (b->col_offset < 0 || b->col_offset + b->cols > b->global_cols) return fail_arg("rg_mf_pairs: bad column slice");
    if (b->global_pos <= 0 && b->loss != RG_LOSS_POINTWISE && b->loss != RG_LOSS_POINTWISE_POS)
        return fail_arg("rg_mf_pairs: empty global batch");
    if (b->pool_len <= 0 || !b->pool || !b->words) return fail_arg("rg_mf_pairs: empty pool / no words");
    if (b->n_pos > 0 && (!b->pos_user || !b->pos_item)) return fail_arg("rg_mf_pairs: null positives");
    if (b->loss < 0 || b->loss > RG_LOSS_POINTWISE_POS) return fail_arg("rg_mf_pairs: bad loss kind");
    if (!w->loss_partials) return fail_arg("rg_mf_pairs: null loss_partials");
    if (backward && (!w->row_count || !w->row_list || !w->hot_grad || !w->hot_bias_grad))
        return fail_arg("rg_mf_pairs: null backward scratch");
    const bool adaptive = b->loss == RG_LOSS_ADAPTIVE_HINGE;
    if (adaptive && (!w->scores || !w->max_key || !w->active_count))
        return fail_arg("rg_mf_pairs: adaptive hinge needs scores/max_key/active_count");
    if (w->plan_perm && (!w->plan_pos_slot || !w->part_row || !w->part_bias || !w->plan_item_slot_off))
        return fail_arg("rg_mf_pairs: incomplete plan");

    a = PairsArgs{};
    a.user_w = t->user_w; a.item_w = t->item_w; a.user_b = t->user_b; a.item_b = t->item_b;
    a.num_users = t->num_users; a.dim = t->dim;
    a.pos_user = b->pos_user; a.pos_item = b->pos_item;
    a.n_pos = b->n_pos; a.cols = b->cols; a.col_offset = b->col_offset; a.global_cols = b->global_cols;
    a.words = reinterpret_cast<const uint2 *>(b->words);
    a.pool = reinterpret_cast<const int2 *>(b->pool);
    a.pool_len = b->pool_len; a.n_neg = b->n_neg; a.loss = b->loss;
    switch (b->loss) {
        case RG_LOSS_POINTWISE:
            a.n_a = (float)b->global_pos;
            a.n_b = (float)((int64_t)b->n_neg * (b->neg_cols > 0 ? b->neg_cols : b->global_cols));
            break;
        case RG_LOSS_BPR:
        case RG_LOSS_HINGE:
            a.n_a = (float)((int64_t)b->n_neg * b->global_pos);
            a.n_b = 1.0f;
            break;
        default:
            a.n_a = (float)b->global_pos;
            a.n_b = 1.0f;
    }
    a.row_count = w->row_count;
    a.row_list = reinterpret_cast<int2 *>(w->row_list);
    a.hot_grad = reinterpret_cast<long long *>(w->hot_grad);
    a.hot_bias_grad = reinterpret_cast<long long *>(w->hot_bias_grad);
    a.partials = w->loss_partials; a.scores = w->scores;
    a.max_key = reinterpret_cast<unsigned long long *>(w->max_key);
    a.active_count = w->active_count;
    if (!b->pairs) return fail_arg("rg_mf_pairs: batch->pairs not prepared (rg_mf_prepare)");
    a.pairs = reinterpret_cast<const int2 *>(b->pairs);
    a.perm = w->plan_perm;
    a.pos_slot = backward ? w->plan_pos_slot : nullptr;   // partials only in the backward pass
    a.part_row = w->part_row; a.part_bias = w->part_bias;
    if (w->claim_num_users > 0) {
        if (w->claim_num_users != t->num_users || t->num_users >= kClaimIdMask || t->num_items >= kClaimIdMask)
            return fail_arg("rg_mf_pairs: claimed slots need claim_num_users == num_users and ids < 2^27");
        if (adaptive) return fail_arg("rg_mf_pairs: no claimed slots for the adaptive hinge");
        a.claimed = 1;
    }
    return RG_OK;
}

extern "C" int rg_mf_pairs(void *stream, const rg_mf_tables_t *t, const rg_mf_batch_t *b, rg_mf_work_t *w,
                           int32_t backward) {
    PairsArgs a;
    int rc = pairs_args(t, b, w, backward, a);
    if (rc) return rc;
    PairsLaunchF f{&a, (hipStream_t)stream, b->loss == RG_LOSS_ADAPTIVE_HINGE, backward != 0};
    return dispatch_dim(t->dim, f);
}

static int prepare_args(const rg_mf_batch_t *b, const rg_mf_work_t *w, const rg_mf_mark_t *mark, PairsArgs &a) {
    if (!b || !b->pairs) return fail_arg("rg_mf_prepare: null batch/pairs");
    if (b->n_neg < 1 || b->n_neg > kNMax) return fail_arg("rg_mf_prepare: n_neg must be in [1, 8]");
    if (b->cols <= 0 || b->n_pos < 0 || b->n_pos > b->cols) return fail_arg("rg_mf_prepare: bad n_pos/cols");
    if (b->col_offset < 0 || b->col_offset + b->cols > b->global_cols) return fail_arg("rg_mf_prepare: bad slice");
    if (b->pool_len <= 0 || !b->pool || !b->words) return fail_arg("rg_mf_prepare: empty pool / no words");
    if (b->n_pos > 0 && (!b->pos_user || !b->pos_item)) return fail_arg("rg_mf_prepare: null positives");
    if (mark && (!mark->stamp || mark->serial == 0 || mark->num_users <= 0))
        return fail_arg("rg_mf_prepare: bad row marks (stamp, serial != 0, num_users)");
    a = PairsArgs{};
    a.pos_user = b->pos_user; a.pos_item = b->pos_item;
    a.n_pos = b->n_pos; a.cols = b->cols; a.col_offset = b->col_offset; a.global_cols = b->global_cols;
    a.words = reinterpret_cast<const uint2 *>(b->words);
    a.pool = reinterpret_cast<const int2 *>(b->pool);
    a.pool_len = b->pool_len; a.n_neg = b->n_neg;
    a.perm = w ? w->plan_perm : nullptr;
    a.pos_slot = w ? w->plan_pos_slot : nullptr;
    a.loss = b->loss;
    if (mark) {
        a.stamp = mark->stamp;
        a.serial = mark->serial;
        a.num_users = mark->num_users;
    }
    if (w && w->claim_num_users > 0) {
        if (mark) return fail_arg("rg_mf_prepare: claimed slots and row marks are exclusive");
        if (!w->row_count) return fail_arg("rg_mf_prepare: claimed slots need row_count");
        if (b->loss == RG_LOSS_ADAPTIVE_HINGE)
            return fail_arg("rg_mf_prepare: no claimed slots for the adaptive hinge (its lists follow the max)");
        a.claimed = 1;
        a.row_count = w->row_count;
        if (w->claim_num_users >= kClaimIdMask) return fail_arg("rg_mf_prepare: claimed slots need ids < 2^27");
        a.num_users = w->claim_num_users;
    }
    return RG_OK;
}

extern "C" int rg_mf_prepare_marked(void *stream, const rg_mf_batch_t *b, const rg_mf_work_t *w,
                                    const rg_mf_mark_t *mark) {
    PairsArgs a;
    int rc = prepare_args(b, w, mark, a);
    if (rc) return rc;
    const int64_t total = prepare_threads(b->cols, b->n_neg);
#if RG_AB
    static const int prio = [] { const char *e = getenv("RG_PREP_PRIO"); return e ? atoi(e) : 1; }();
#else
    constexpr int prio = 1;
#endif
    hipLaunchKernelGGL(mf_prepare_kernel, dim3((total + kBlock - 1) / kBlock), dim3(kBlock), 0,
                       (hipStream_t)stream, a, reinterpret_cast<int2 *>(b->pairs), prio);
    return check_launch("rg_mf_prepare");
}

extern "C" int rg_mf_prepare(void *stream, const rg_mf_batch_t *b, const rg_mf_work_t *w) {
    return rg_mf_prepare_marked(stream, b, w, nullptr);
}

extern "C" int rg_mf_prepare_hot(void *stream, const rg_mf_batch_t *b, const rg_mf_work_t *w, int32_t *hot_out,
                                 int32_t *nhot_out) {
    PairsArgs a;
    int rc = prepare_args(b, w, nullptr, a);
    if (rc) return rc;
    if (!a.claimed || !hot_out || !nhot_out) return fail_arg("rg_mf_prepare_hot: needs claimed slots and a hot list");
    a.hot_out = hot_out;
    a.nhot_out = nhot_out;
    const int64_t total = prepare_threads(b->cols, b->n_neg);
    hipLaunchKernelGGL(mf_prepare_kernel, dim3((total + kBlock - 1) / kBlock), dim3(kBlock), 0, (hipStream_t)stream, a,
                       reinterpret_cast<int2 *>(b->pairs), 0);
    return check_launch("rg_mf_prepare_hot");
}

static int apply_args(const rg_mf_tables_t *t, const rg_mf_work_t *w, const float *grad_in, float *grad_out,
                      const rg_opt_t *opt, int64_t row_begin, int64_t row_end, const rg_mf_loss_t *loss,
                      float *dense_loss_out, int mode, ApplyArgs &a) {
    int rc = check_tables(t);
    if (rc) return rc;
    const int64_t nrows = t->num_users + t->num_items;
    if (row_begin < 0) row_begin = 0;
    if (row_end < 0 || row_end > nrows) row_end = nrows;
    if (row_begin > row_end) return fail_arg("rg_mf_apply: row_begin > row_end");
    if (mode != kGradOnly) {
        if (!opt) return fail_arg("rg_mf_apply: null opt");
        if (!t->user_w_out || !t->item_w_out || !t->user_b_out || !t->item_b_out)
            return fail_arg("rg_mf_apply: null output tables");
        if ((mode == kApplyPull || mode == kApplyCold) && (t->user_w_out == t->user_w || t->item_w_out == t->item_w ||
                                   t->user_b_out == t->user_b || t->item_b_out == t->item_b))
            return fail_arg("rg_mf_apply: output tables must not alias the inputs (ping-pong)");
        if (opt->kind < RG_OPT_ADAM || opt->kind > RG_OPT_RMSPROP) return fail_arg("rg_mf_apply: bad optimizer");
        if (opt->kind == RG_OPT_ADAM && (!t->user_w_m || !t->item_w_m || !t->user_b_m || !t->item_b_m))
            return fail_arg("rg_mf_apply: Adam needs m state");
        if (opt->kind != RG_OPT_SGD && (!t->user_w_v || !t->item_w_v || !t->user_b_v || !t->item_b_v))
            return fail_arg("rg_mf_apply: optimizer needs v state");
    }
    if (mode != kApplyDense && mode != kApplyCold) {
        if (!w || !w->row_count || !w->row_list || !w->hot_grad || !w->hot_bias_grad)
            return fail_arg("rg_mf_apply: null scratch");
        if (loss && loss->out && !w->loss_partials) return fail_arg("rg_mf_apply: loss needs partials");
    }
    if (mode != kApplyPull && mode != kApplyCold && !(grad_in || grad_out))
        return fail_arg("rg_mf_apply: null gradient buffer");
    a = ApplyArgs{};
    a.w_in[0] = t->user_w; a.w_in[1] = t->item_w; a.b_in[0] = t->user_b; a.b_in[1] = t->item_b;
    a.w_out[0] = t->user_w_out; a.w_out[1] = t->item_w_out; a.b_out[0] = t->user_b_out; a.b_out[1] = t->item_b_out;
    a.w_m[0] = t->user_w_m; a.w_m[1] = t->item_w_m; a.w_v[0] = t->user_w_v; a.w_v[1] = t->item_w_v;
    a.b_m[0] = t->user_b_m; a.b_m[1] = t->item_b_m; a.b_v[0] = t->user_b_v; a.b_v[1] = t->item_b_v;
    a.num_users = t->num_users; a.num_items = t->num_items; a.dim = t->dim;
    a.row_begin = row_begin; a.row_end = row_end;
    if (w) {
        a.row_count = w->row_count; a.row_list = reinterpret_cast<const int2 *>(w->row_list);
        a.hot_grad = reinterpret_cast<long long *>(w->hot_grad);
    a.hot_bias_grad = reinterpret_cast<long long *>(w->hot_bias_grad);
        a.partials = w->loss_partials;
        if (w->plan_perm) {
            a.item_slot_off = w->plan_item_slot_off;
            a.part_row = w->part_row; a.part_bias = w->part_bias;
        }
    }
    if (opt) a.opt = *opt;
    if (mode == kApplyDense) {
        a.loss_out = dense_loss_out;
    } else if (loss) {
        a.n_partials = loss->n_partials; a.inv_a = loss->inv_a; a.inv_b = loss->inv_b;
        a.loss_out = loss->out;
    }
    a.grad = grad_out ? grad_out : const_cast<float *>(grad_in);
    a.has_bias = true;
    return RG_OK;
}

static int apply_common(void *stream, const rg_mf_tables_t *t, rg_mf_work_t *w, const float *grad_in,
                        float *grad_out, const rg_opt_t *opt, int64_t row_begin, int64_t row_end,
                        const rg_mf_loss_t *loss, float *dense_loss_out, int mode) {
    ApplyArgs a;
    int rc = apply_args(t, w, grad_in, grad_out, opt, row_begin, row_end, loss, dense_loss_out, mode, a);
    if (rc) return rc;
    ApplyLaunchF f{&a, (hipStream_t)stream, mode};
    return dispatch_dim(t->dim, f);
}

namespace {
struct FrontLaunchF {
    PairsArgs *pa, *prep;
    ApplyArgs *aa;
    FrontArgs f;
    hipStream_t s;
    template <class L>
    int operator()() {
        f.pair_blocks = pairs_blocks<L>(pa->cols);
        const int64_t cold_rows = aa->row_end - aa->row_begin;
        const int64_t cold_waves = (cold_rows + L::UPW - 1) / L::UPW;
        const int64_t cold_blocks = (cold_waves + kBlock / kWave - 1) / (kBlock / kWave);
        const dim3 grid((unsigned)(f.pair_blocks + f.prep_blocks + cold_blocks));
        if (pa->n_neg <= 5)
            hipLaunchKernelGGL((mf_front_kernel<L, 5>), grid, dim3(kBlock), 0, s, *pa, *prep, *aa, f);
        else
            hipLaunchKernelGGL((mf_front_kernel<L, kNMax>), grid, dim3(kBlock), 0, s, *pa, *prep, *aa, f);
        return check_launch("rg_mf_step_front");
    }
};

struct HotLaunchF {
    ApplyArgs *a;
    const int2 *pairs;
    int64_t n_slots;
    int stride, np_;
    const rg_mf_mark_t *mark;
    hipStream_t s;
    template <class L>
    int operator()() {
        if (mark) {
            const int64_t rows = a->row_end - a->row_begin;
            const int64_t waves = (rows + L::UPW - 1) / L::UPW;
            const int64_t nb = (waves + kBlock / kWave - 1) / (kBlock / kWave);
            hipLaunchKernelGGL((mf_hot_scan_kernel<L>), dim3(nb < 1 ? 1 : nb), dim3(kBlock), 0, s, *a, mark->stamp,
                               mark->serial);
            return check_launch("rg_mf_step_hot");
        }
        const int64_t waves = (n_slots + L::UPW - 1) / L::UPW;
        const int64_t nb = (waves + kBlock / kWave - 1) / (kBlock / kWave);
        hipLaunchKernelGGL((mf_hot_kernel<L>), dim3(nb < 1 ? 1 : nb), dim3(kBlock), 0, s, *a, pairs, n_slots, stride,
                           np_);
        return check_launch("rg_mf_step_hot");
    }
};
}  // namespace

#ifndef RG_BACK_V_NCF
#define RG_BACK_V_NCF 1
#endif
namespace {
struct BackLaunchF {
    ApplyArgs *a;
    PairsArgs *prep;
    int2 *prep_out;
    int64_t prep_blocks;
    MtGenArgs gen;
    hipStream_t s;
    const OwnerArgs *own = nullptr;   // owner-sharded DP: the next step's owner prepare
    bool lazy = false;                // lazy dense pass (rg_mf_apply_lazy)
    const MlpUpdArgs *upd = nullptr;  // NCF step: the MLP update in the same launch (rg_ncf_tail)
    template <class L>
    int operator()() {
        using LB = typename BackLayout<L>::type;
        if constexpr (!std::is_same<LB, L>::value) {
            // the dense pass (MF single-GPU, an owner rank's user rows, the NCF tail's embedding
            // tables pulling their per-example gradient rows) on its own row layout (RG_BACK_V64 /
            // _V128); element-wise arithmetic, so the same bits as the dispatch layout
            constexpr bool pairs = !LB::VEC;   // RowLayoutP: float2 pairs, even dims only
            if (!lazy && (a->contrib == nullptr || RG_BACK_V_NCF) && (!pairs || a->dim % 2 == 0))
                return run<LB, true>();
        }
        return run<L, false>();
    }
    // V: the dense-pass layout of a plain MF launch (no owner / NCF / lazy / A/B variants)
    template <class L, bool V>
    int run() {
        const int64_t rows = a->row_end - a->row_begin;
        const int64_t waves = (rows + L::UPW - 1) / L::UPW;
        int64_t nb = (waves + kBlock / kWave - 1) / (kBlock / kWave);
        if (nb < 1) nb = 1;
#if RG_AB
        // A/B build only (each measured slower or no faster): prepare blocks after the
        // dense blocks, the XCD-aware dense mapping, non-temporal stores, the list read after the
        // count, the persistent pipelined dense kernel
        static const int prep_first = [] { const char *e = getenv("RG_PREP_FIRST"); return e ? atoi(e) : 1; }();
        static const int xcd_map = [] { const char *e = getenv("RG_XCD_MAP"); return e ? atoi(e) : 0; }();
        static const int nt = [] { const char *e = getenv("RG_APPLY_NT"); return e ? atoi(e) : 0; }();
        static const int spec = [] { const char *e = getenv("RG_APPLY_SPEC"); return e ? atoi(e) : 1; }();
        static const int lazy_spec = [] { const char *e = getenv("RG_LAZY_SPEC"); return e ? atoi(e) : 0; }();
        static const int dense_v2 = [] { const char *e = getenv("RG_DENSE_PIPE"); return e ? atoi(e) : 0; }();
#else
        constexpr int prep_first = 1, xcd_map = 0;
#endif
        if (upd && !prep_first) return fail_arg("rg_ncf_tail: the MLP update workgroups need the prepare-first grid");
        const int64_t upd_blocks = upd ? ((int64_t)upd->P + 63) / 64 : 0;
        BackGrid bg{prep_blocks, 0, 0, prep_first, prep_first ? xcd_map : 0, upd_blocks};
        const int64_t head = prep_blocks + upd_blocks + (gen.nwords > 0 ? 1 : 0);
        int64_t total = nb + head;
        if (prep_first) {
            bg.apply_start = (head + 7) / 8 * 8;
            bg.apply_padded = (nb + 7) / 8 * 8;
            total = bg.apply_start + bg.apply_padded;
        }
        const dim3 grid((unsigned)total);
        const OwnerArgs oa = own ? *own : OwnerArgs{};
        const MlpUpdArgs ua = upd ? *upd : MlpUpdArgs{};
        LaunchEvents &le = launch_events();
        const hipEvent_t e0 = le.start, e1 = le.stop;
        le = LaunchEvents{};
        auto go = [&](auto kernel) {
            if (e0 || e1)
                hipExtLaunchKernelGGL(kernel, grid, dim3(kBlock), 0, s, e0, e1, 0, *a, *prep, prep_out, nb, gen, bg, oa,
                                      ua);
            else
                hipLaunchKernelGGL(kernel, grid, dim3(kBlock), 0, s, *a, *prep, prep_out, nb, gen, bg, oa, ua);
        };
        if constexpr (V) {
#ifndef RG_BACK_NT   // timing experiments: store policy of the V-layout dense pass (apply_row's NT)
#define RG_BACK_NT 0
#endif
#ifdef RG_BACK_PIPE   // timing experiments: the persistent software-pipelined dense kernel (mf_dense_kernel)
            if (!own) {
                int64_t db = (int64_t)num_cus() * RG_BACK_PIPE;
                const int64_t groups = (rows + L::UPW - 1) / L::UPW;
                const int64_t need = (groups + kBlock / kWave - 1) / (kBlock / kWave);
                if (db > need) db = need;
                BackGrid dg{prep_blocks, 0, 0, 1, 0};
                dg.apply_start = (head + 7) / 8 * 8;
                const dim3 dgrid((unsigned)(dg.apply_start + db));
                if (e0 || e1)
                    hipExtLaunchKernelGGL(mf_dense_kernel<L>, dgrid, dim3(kBlock), 0, s, e0, e1, 0, *a, *prep, prep_out, db,
                                          gen, dg);
                else
                    hipLaunchKernelGGL(mf_dense_kernel<L>, dgrid, dim3(kBlock), 0, s, *a, *prep, prep_out, db, gen, dg);
                return check_launch("rg_mf_apply_prepare");
            }
#endif
            if (own) go(mf_back_kernel<L, 0, true, true>);
            else go(mf_back_kernel<L, RG_BACK_NT, true>);
            return check_launch("rg_mf_apply_prepare");
        } else {
        if (own) {
            go(mf_back_kernel<L, 0, true, true>);
            return check_launch("rg_mf_apply_prepare");
        }
#if RG_AB
        if constexpr (L::LPU >= kCap) {
            if (!lazy && dense_v2 && a->contrib == nullptr && upd == nullptr) {
                // a few workgroups per CU, each wave walking a chunk of row groups (mf_dense_kernel)
                static const int per_cu = [] { const char *e = getenv("RG_DENSE_PER_CU"); return e ? atoi(e) : 4; }();
                int64_t db = (int64_t)num_cus() * per_cu;
                const int64_t groups = (rows + L::UPW - 1) / L::UPW;
                const int64_t need = (groups + kBlock / kWave - 1) / (kBlock / kWave);
                if (db > need) db = need;
                if (db < 1) db = 1;
                BackGrid dg{prep_blocks, 0, 0, 1, 0};
                dg.apply_start = (head + 7) / 8 * 8;
                const dim3 dgrid((unsigned)(dg.apply_start + db));
                if (e0 || e1)
                    hipExtLaunchKernelGGL(mf_dense_kernel<L>, dgrid, dim3(kBlock), 0, s, e0, e1, 0, *a, *prep, prep_out, db,
                                          gen, dg);
                else
                    hipLaunchKernelGGL(mf_dense_kernel<L>, dgrid, dim3(kBlock), 0, s, *a, *prep, prep_out, db, gen, dg);
                return check_launch("rg_mf_apply_prepare");
            }
        }
        if (lazy && lazy_spec) go(mf_back_kernel<L, 0, true, false, true, true>);
        else if (lazy) go(mf_back_kernel<L, 0, true, false, true>);
        else if (spec && nt == 1) go(mf_back_kernel<L, 1, true>);
        else if (spec && nt == 3) go(mf_back_kernel<L, 3, true>);
        else if (spec) go(mf_back_kernel<L, 0, true>);
        else if (nt == 1) go(mf_back_kernel<L, 1>);
        else if (nt >= 2) go(mf_back_kernel<L, 2>);
        else go(mf_back_kernel<L, 0>);
#else
        if (lazy) return fail_arg("the lazy dense pass is an A/B build (build.py --variant lazy -DRG_AB=1)");
        go(mf_back_kernel<L, 0, true>);   // the list loaded beside the count
#endif
        return check_launch("rg_mf_apply_prepare");
        }
    }
};
}  // namespace

namespace {
struct PipeLaunchF {
    ApplyArgs *a;
    PairsArgs *pa, *prep;
    int2 *prep_out;
    PipeArgs pp;
    MtGenArgs gen;
    int64_t pair_cols, pair_users;
    hipStream_t s;
    template <class L>
    int operator()() {
        if constexpr (L::LPU < kCap) {
            return fail_arg("rg_mf_pipe_step: dim must be a multiple of 4 and >= 32");
        } else {
            const int64_t rpb = (kBlock / kWave) * L::UPW;
            pp.item_blocks = (a->num_items + rpb - 1) / rpb;
            const int64_t hu = pair_users < a->num_users ? pair_users : a->num_users;
            pp.huser_blocks = (hu + rpb - 1) / rpb;
            const int64_t cold = (a->num_users + rpb - 1) / rpb;
            // cold rows ahead of the pair workgroups: about one chip's worth, so the hot rows are
            // mostly done when the pair workgroups start waiting
            static const int64_t c1 = [] { const char *e = getenv("RG_PIPE_COLD1"); return e ? atoll(e) : 2048LL; }();
            pp.cold1_blocks = cold < c1 ? cold : c1;
            pp.cold2_blocks = cold - pp.cold1_blocks;
            pp.pair_blocks = pairs_blocks<L>(pair_cols);
            const int64_t total = (gen.nwords > 0 ? 1 : 0) + pp.prep_blocks + pp.item_blocks + pp.huser_blocks +
                                  pp.cold1_blocks + pp.pair_blocks + pp.cold2_blocks;
            LaunchEvents &le = launch_events();
            const hipEvent_t e0 = le.start, e1 = le.stop;
            le = LaunchEvents{};
            auto go = [&](auto kernel) {
                if (e0 || e1)
                    hipExtLaunchKernelGGL(kernel, dim3((unsigned)total), dim3(kBlock), 0, s, e0, e1, 0, *a, *pa, *prep,
                                          prep_out, pp, gen);
                else
                    hipLaunchKernelGGL(kernel, dim3((unsigned)total), dim3(kBlock), 0, s, *a, *pa, *prep, prep_out, pp,
                                       gen);
            };
            if (pa->n_neg <= 5) go(mf_pipe_kernel<L, 5>);
            else go(mf_pipe_kernel<L, kNMax>);
            return check_launch("rg_mf_pipe_step");
        }
    }
};
}  // namespace

extern "C" int rg_mf_pipe_step(void *stream, const rg_mf_tables_t *t, rg_mf_work_t *w, const rg_opt_t *opt,
                               const rg_mf_loss_t *loss, const rg_mf_batch_t *pair_b, rg_mf_work_t *pair_w,
                               const rg_mf_batch_t *next, const rg_mf_work_t *next_w, const rg_mf_pipe_t *pipe,
                               const rg_mt_gen_t *gen) {
#if !RG_AB
    (void)stream; (void)t; (void)w; (void)opt; (void)loss; (void)pair_b; (void)pair_w; (void)next; (void)next_w;
    (void)pipe; (void)gen;
    // measured 4x slower than the split step: carried by the A/B build only
    return fail_arg("rg_mf_pipe_step: the pipelined step is an A/B build (build.py --variant NAME -DRG_AB=1)");
#else
    if (kPairBlock != kBlock) return fail_arg("rg_mf_pipe_step: built with a pair-pass workgroup != 256 threads");
    if (!pipe || !pipe->hot_users || !pipe->nhot || !pipe->counts_next || !pipe->gate || !pipe->gate_next ||
        !pipe->nhot_free || !pipe->err)
        return fail_arg("rg_mf_pipe_step: incomplete rg_mf_pipe_t");
    if (!pair_b || !pair_w) return fail_arg("rg_mf_pipe_step: null pair batch / work");
    if (pair_b->loss != RG_LOSS_POINTWISE && pair_b->loss != RG_LOSS_BPR && pair_b->loss != RG_LOSS_HINGE)
        return fail_arg("rg_mf_pipe_step: pointwise, bpr or hinge only (the adaptive hinge needs the max first)");
    if (pair_w->claim_num_users <= 0) return fail_arg("rg_mf_pipe_step: the paired step must carry claimed slots");
    if ((t->num_users > t->num_items ? t->num_users : t->num_items) * (int64_t)t->dim * 4 >= ((int64_t)1 << 31))
        return fail_arg("rg_mf_pipe_step: tables of 2 GiB or more (32-bit write-through offsets)");
    if (pair_w->row_list == w->row_list || pair_w->hot_grad == w->hot_grad || pair_w->loss_partials == w->loss_partials ||
        (w->part_row && pair_w->part_row == w->part_row))
        return fail_arg("rg_mf_pipe_step: the paired step's scratch must not alias this step's");
    ApplyArgs a;
    int rc = apply_args(t, w, nullptr, nullptr, opt, 0, -1, loss, nullptr, kApplyPull, a);
    if (rc) return rc;
    // the pair pass reads the tables this launch writes
    rg_mf_tables_t pt = *t;
    pt.user_w = t->user_w_out; pt.item_w = t->item_w_out; pt.user_b = t->user_b_out; pt.item_b = t->item_b_out;
    PairsArgs pa;
    if ((rc = pairs_args(&pt, pair_b, pair_w, 1, pa))) return rc;
    PairsArgs prep{};
    int2 *prep_out = nullptr;
    PipeArgs pp{};
    if (next) {
        if ((rc = prepare_args(next, next_w, nullptr, prep))) return rc;
        if (!prep.claimed || !pipe->hot_out || !pipe->nhot_out)
            return fail_arg("rg_mf_pipe_step: the prepared step needs claimed slots and a hot list");
        if (next->pairs == pair_b->pairs) return fail_arg("rg_mf_pipe_step: prepared pairs alias the paired step's");
        prep.hot_out = pipe->hot_out;
        prep.nhot_out = pipe->nhot_out;
        prep_out = reinterpret_cast<int2 *>(next->pairs);
        pp.prep_blocks = (prepare_threads(next->cols, next->n_neg) + kBlock - 1) / kBlock;
    } else {
        pp.prep_blocks = 1;   // block 0 still resets the counters and finalizes the loss
        prep.cols = 0;
    }
    MtGenArgs g{};
    if (gen && gen->nwords > 0) {
        if (!gen->state || !gen->out) return fail_arg("rg_mf_pipe_step: null MT state / output");
        g.state = gen->state; g.out = gen->out; g.state_before = gen->state_before; g.nwords = gen->nwords;
    }
    pp.hot_users = pipe->hot_users; pp.nhot = pipe->nhot; pp.counts_next = pipe->counts_next;
    pp.gate = pipe->gate; pp.gate_next = pipe->gate_next; pp.nhot_free = pipe->nhot_free; pp.err = pipe->err;
    static const uint32_t spin = [] { const char *e = getenv("RG_PIPE_SPIN"); return e ? (uint32_t)atoll(e) : 4000000u; }();
    pp.spin_limit = spin;
    PipeLaunchF f{&a, &pa, &prep, prep_out, pp, g, pair_b->cols, (int64_t)(1 + pair_b->n_neg) * pair_b->cols,
                  (hipStream_t)stream};
    return dispatch_dim(t->dim, f);
#endif
}

namespace {
struct Pipe2HotF {
    ApplyArgs *a;
    Pipe2Args p;
    MtGenArgs gen;
    int64_t hot_cap;
    hipStream_t s;
    template <class L>
    int operator()() {
        using LD = typename BackLayout<L>::type;
        constexpr int64_t rpb = (kBlock / kWave) * LD::UPW;
        p.item_blocks = (a->num_items + rpb - 1) / rpb;
        p.hot_blocks = (hot_cap + rpb - 1) / rpb;
        int64_t total = p.item_blocks + p.hot_blocks + (gen.nwords > 0 ? 1 : 0);
        if (total < 1) total = 1;
        LaunchEvents &le = launch_events();
        const hipEvent_t e0 = le.start, e1 = le.stop;
        le = LaunchEvents{};
        if (e0 || e1)
            hipExtLaunchKernelGGL(mf_pipe2_hot_kernel<LD>, dim3((unsigned)total), dim3(kBlock), 0, s, e0, e1, 0, *a, p,
                                  gen);
        else
            hipLaunchKernelGGL(mf_pipe2_hot_kernel<LD>, dim3((unsigned)total), dim3(kBlock), 0, s, *a, p, gen);
        return check_launch("rg_mf_pipe2_hot");
    }
};

struct Pipe2ColdF {
    ApplyArgs *a;
    PairsArgs *pa, *prep;
    int2 *prep_out;
    Pipe2Args p;
    MtGenArgs gen;
    hipStream_t s;
    template <class L>
    int operator()() {
        if (pa->n_neg <= 5) return run<L, 5>();
        return run<L, kNMax>();
    }
    template <class L, int NMAX>
    int run() {
        using LD = typename BackLayout<L>::type;
        constexpr int64_t rpb = (kBlock / kWave) * LD::UPW;
        p.pair_blocks = pairs_blocks<L>(pa->cols);
        p.cold_blocks = (a->num_users + rpb - 1) / rpb;
        const int64_t total = p.pair_blocks + (gen.nwords > 0 ? 1 : 0) + p.prep_blocks + p.cold_blocks;
        LaunchEvents &le = launch_events();
        const hipEvent_t e0 = le.start, e1 = le.stop;
        le = LaunchEvents{};
        if (e0 || e1)
            hipExtLaunchKernelGGL((mf_pipe2_cold_kernel<L, LD, NMAX>), dim3((unsigned)total), dim3(kBlock), 0, s, e0,
                                  e1, 0, *a, *pa, *prep, prep_out, p, gen);
        else
            hipLaunchKernelGGL((mf_pipe2_cold_kernel<L, LD, NMAX>), dim3((unsigned)total), dim3(kBlock), 0, s, *a, *pa,
                               *prep, prep_out, p, gen);
        return check_launch("rg_mf_pipe2_cold");
    }
};
}  // namespace

static int gen_args(const rg_mt_gen_t *gen, MtGenArgs &g, const char *what) {
    g = MtGenArgs{};
    if (gen && gen->nwords > 0) {
        if (!gen->state || !gen->out) return fail_arg(std::string(what) + ": null MT state / output");
        g.state = gen->state; g.out = gen->out; g.state_before = gen->state_before; g.nwords = gen->nwords;
    }
    return RG_OK;
}

extern "C" int rg_mf_pipe2_hot(void *stream, const rg_mf_tables_t *t, rg_mf_work_t *w, const rg_opt_t *opt,
                               const rg_mf_loss_t *loss, const int32_t *hot_users, const int32_t *nhot,
                               int64_t hot_cap, int32_t *nhot_clear, const rg_mt_gen_t *gen) {
    if (!hot_users || !nhot || hot_cap < 0) return fail_arg("rg_mf_pipe2_hot: null hot list");
    ApplyArgs a;
    int rc = apply_args(t, w, nullptr, nullptr, opt, 0, -1, loss, nullptr, kApplyPull, a);
    if (rc) return rc;
    MtGenArgs g;
    if ((rc = gen_args(gen, g, "rg_mf_pipe2_hot"))) return rc;
    Pipe2Args p{};
    p.hot = hot_users;
    p.nhot = nhot;
    p.nhot_clear = nhot_clear;
    Pipe2HotF f{&a, p, g, hot_cap < t->num_users ? hot_cap : t->num_users, (hipStream_t)stream};
    return dispatch_dim(t->dim, f);
}

extern "C" int rg_mf_pipe2_cold(void *stream, const rg_mf_tables_t *t, rg_mf_work_t *w, const rg_opt_t *opt,
                                const rg_mf_batch_t *pair_b, rg_mf_work_t *pair_w, const int32_t *counts_next,
                                const rg_mf_batch_t *next, const rg_mf_work_t *next_w, int32_t *hot_out,
                                int32_t *nhot_out, const rg_mt_gen_t *gen) {
    if (kPairBlock != kBlock) return fail_arg("rg_mf_pipe2_cold: built with a pair-pass workgroup != 256 threads");
    if (!pair_b || !pair_w || !counts_next) return fail_arg("rg_mf_pipe2_cold: null pair batch / work / counts");
    if (pair_b->loss != RG_LOSS_POINTWISE && pair_b->loss != RG_LOSS_BPR && pair_b->loss != RG_LOSS_HINGE)
        return fail_arg("rg_mf_pipe2_cold: pointwise, bpr or hinge only (the adaptive hinge needs the max first)");
    if (pair_w->claim_num_users <= 0 || pair_w->row_count != counts_next)
        return fail_arg("rg_mf_pipe2_cold: the paired step must carry claimed slots in counts_next");
    if (pair_w->row_list == w->row_list || pair_w->hot_grad == w->hot_grad || pair_w->loss_partials == w->loss_partials ||
        (w->part_row && pair_w->part_row == w->part_row) || pair_w->row_count == w->row_count)
        return fail_arg("rg_mf_pipe2_cold: the paired step's scratch must not alias this step's");
    ApplyArgs a;
    int rc = apply_args(t, w, nullptr, nullptr, opt, 0, t->num_users, nullptr, nullptr, kApplyPull, a);
    if (rc) return rc;
    // the pair pass of step t+1 reads the tables this step writes (their rows the hot launch wrote)
    rg_mf_tables_t pt = *t;
    pt.user_w = t->user_w_out; pt.item_w = t->item_w_out; pt.user_b = t->user_b_out; pt.item_b = t->item_b_out;
    PairsArgs pa;
    if ((rc = pairs_args(&pt, pair_b, pair_w, 1, pa))) return rc;
    PairsArgs prep{};
    int2 *prep_out = nullptr;
    a.guard = counts_next;
    Pipe2Args p{};
    p.counts_next = counts_next;
    if (next) {
        if ((rc = prepare_args(next, next_w, nullptr, prep))) return rc;
        if (!prep.claimed || !hot_out || !nhot_out)
            return fail_arg("rg_mf_pipe2_cold: the prepared step needs claimed slots and a hot list");
        if (next->pairs == pair_b->pairs) return fail_arg("rg_mf_pipe2_cold: prepared pairs alias the paired step's");
        if (next_w->row_count == counts_next || next_w->row_count == w->row_count)
            return fail_arg("rg_mf_pipe2_cold: the prepared step's claims alias a live count array");
        prep.hot_out = hot_out;
        prep.nhot_out = nhot_out;
        prep_out = reinterpret_cast<int2 *>(next->pairs);
        p.prep_blocks = (prepare_threads(next->cols, next->n_neg) + kBlock - 1) / kBlock;
    }
    MtGenArgs g;
    if ((rc = gen_args(gen, g, "rg_mf_pipe2_cold"))) return rc;
    Pipe2ColdF f{&a, &pa, &prep, prep_out, p, g, (hipStream_t)stream};
    return dispatch_dim(t->dim, f);
}


extern "C" int rg_mf_apply_prepare(void *stream, const rg_mf_tables_t *t, rg_mf_work_t *w, const rg_opt_t *opt,
                                   int64_t row_begin, int64_t row_end, const rg_mf_loss_t *loss,
                                   const rg_mf_batch_t *next, const rg_mf_work_t *next_w) {
    return rg_mf_apply_prepare_gen(stream, t, w, opt, row_begin, row_end, loss, next, next_w, nullptr);
}

extern "C" int rg_mf_apply_prepare_gen(void *stream, const rg_mf_tables_t *t, rg_mf_work_t *w, const rg_opt_t *opt,
                                       int64_t row_begin, int64_t row_end, const rg_mf_loss_t *loss,
                                       const rg_mf_batch_t *next, const rg_mf_work_t *next_w,
                                       const rg_mt_gen_t *gen) {
    MtGenArgs g{};
    if (gen && gen->nwords > 0) {
        if (!gen->state || !gen->out) return fail_arg("rg_mf_apply_prepare_gen: null MT state / output");
        g.state = gen->state; g.out = gen->out; g.state_before = gen->state_before; g.nwords = gen->nwords;
    }
    ApplyArgs a;
    int rc = apply_args(t, w, nullptr, nullptr, opt, row_begin, row_end, loss, nullptr, kApplyPull, a);
    if (rc) return rc;
    PairsArgs prep{};
    int64_t prep_blocks = 0;
    int2 *prep_out = nullptr;
    if (next) {
        if ((rc = prepare_args(next, next_w, nullptr, prep))) return rc;
        prep_out = reinterpret_cast<int2 *>(next->pairs);
        prep_blocks = (prepare_threads(next->cols, next->n_neg) + kBlock - 1) / kBlock;
    }
    BackLaunchF f{&a, &prep, prep_out, prep_blocks, g, (hipStream_t)stream};
    return dispatch_dim(t->dim, f);
}

namespace {
struct PairsPrepLaunchF {
    PairsArgs *a, *prep;
    int2 *prep_out;
    int64_t prep_blocks;
    hipStream_t s;
    template <class L>
    int operator()() {
        const int64_t nb = pairs_blocks<L>(a->cols);
        const dim3 grid((unsigned)(nb + prep_blocks));
        if (a->n_neg <= 5)
            hipLaunchKernelGGL((mf_pairs_prep_kernel<L, 5>), grid, dim3(kPairBlock), 0, s, *a, *prep, prep_out, nb);
        else
            hipLaunchKernelGGL((mf_pairs_prep_kernel<L, kNMax>), grid, dim3(kPairBlock), 0, s, *a, *prep, prep_out, nb);
        return check_launch("rg_mf_pairs_prepare");
    }
};

struct FlushLaunchF {
    ApplyArgs *a;
    hipStream_t s;
    template <class L>
    int operator()() {
        const int64_t waves = (a->num_users + L::UPW - 1) / L::UPW;
        const int64_t nb = (waves + kBlock / kWave - 1) / (kBlock / kWave);
        hipLaunchKernelGGL((mf_lazy_flush_kernel<L>), dim3(nb < 1 ? 1 : nb), dim3(kBlock), 0, s, *a);
        return check_launch("rg_mf_lazy_flush");
    }
};

int lazy_args(const rg_mf_lazy_t *lz, const rg_opt_t *opt, ApplyArgs &a) {
    if (!lz || !lz->last_rel) return fail_arg("lazy dense pass: null rg_mf_lazy_t / last_rel");
    if (lz->step < 1 || lz->base < 0 || lz->base > lz->step || lz->step >= ((int64_t)1 << 31))
        return fail_arg("lazy dense pass: bad step / base");
    if (opt && opt->kind == RG_OPT_ADAM && (!lz->step_consts || lz->n_consts <= lz->step))
        return fail_arg("lazy dense pass: Adam needs the per-step constants up to this step");
    a.last_rel = lz->last_rel;
    a.umark = lz->umark;
    a.step_consts = reinterpret_cast<const float2 *>(lz->step_consts);
    a.lazy_base = lz->base;
    a.lazy_t = (int32_t)lz->step;
    a.lazy_full = lz->full;
    a.lazy_rows = reinterpret_cast<unsigned long long *>(lz->rows_done);
#if RG_AB
    static const int dbg = [] { const char *e = getenv("RG_LAZY_DBG"); return e ? atoi(e) : 0; }();
    static const int cap = [] { const char *e = getenv("RG_LAZY_CAP"); return e ? atoi(e) : 0; }();
    a.lazy_dbg = dbg;
    a.lazy_cap = cap;
#else
    a.lazy_dbg = 0;
    a.lazy_cap = 0;
#endif
    return RG_OK;
}
}  // namespace

extern "C" int rg_mf_pairs_prepare(void *stream, const rg_mf_tables_t *t, const rg_mf_batch_t *b, rg_mf_work_t *w,
                                   const rg_mf_batch_t *next, const rg_mf_work_t *next_w, int32_t *umark,
                                   int32_t umark_step) {
    if (!next) return rg_mf_pairs(stream, t, b, w, 1);
    PairsArgs prep{};
    int rc = prepare_args(next, next_w, nullptr, prep);
    if (rc) return rc;
    prep.umark = umark;
    prep.umark_step = umark_step;
    prep.num_users = t ? t->num_users : 0;
    const int64_t total = prepare_threads(next->cols, next->n_neg);
    if (b && b->loss == RG_LOSS_ADAPTIVE_HINGE) {   // several launches: the global max first
        if ((rc = rg_mf_pairs(stream, t, b, w, 1))) return rc;
        hipLaunchKernelGGL(mf_prepare_kernel, dim3((total + kBlock - 1) / kBlock), dim3(kBlock), 0,
                           (hipStream_t)stream, prep, reinterpret_cast<int2 *>(next->pairs), 0);
        return check_launch("rg_mf_pairs_prepare(prepare)");
    }
    if (kPairBlock != kBlock) return fail_arg("rg_mf_pairs_prepare: built with a pair-pass workgroup != 256 threads");
    PairsArgs a;
    if ((rc = pairs_args(t, b, w, 1, a))) return rc;
    PairsPrepLaunchF f{&a, &prep, reinterpret_cast<int2 *>(next->pairs), (total + kBlock - 1) / kBlock,
                       (hipStream_t)stream};
    return dispatch_dim(t->dim, f);
}

extern "C" int rg_mf_apply_lazy(void *stream, const rg_mf_tables_t *t, rg_mf_work_t *w, const rg_opt_t *opt,
                                const rg_mf_loss_t *loss, const rg_mf_lazy_t *lazy, const rg_mt_gen_t *gen) {
    MtGenArgs g{};
    if (gen && gen->nwords > 0) {
        if (!gen->state || !gen->out) return fail_arg("rg_mf_apply_lazy: null MT state / output");
        g.state = gen->state; g.out = gen->out; g.state_before = gen->state_before; g.nwords = gen->nwords;
    }
    ApplyArgs a;
    int rc = apply_args(t, w, nullptr, nullptr, opt, 0, -1, loss, nullptr, kApplyPull, a);
    if (rc) return rc;
    if ((rc = lazy_args(lazy, opt, a))) return rc;
    if (!lazy->full && !lazy->umark) return fail_arg("rg_mf_apply_lazy: a partial pass needs the user marks");
    PairsArgs prep{};
    BackLaunchF f{&a, &prep, nullptr, 0, g, (hipStream_t)stream};
    f.lazy = true;
    return dispatch_dim(t->dim, f);
}

extern "C" int rg_mf_lazy_flush(void *stream, const rg_mf_tables_t *t, const rg_opt_t *opt, const rg_mf_lazy_t *lazy) {
    int rc = check_tables(t);
    if (rc) return rc;
    if (!opt || opt->kind < RG_OPT_ADAM || opt->kind > RG_OPT_RMSPROP) return fail_arg("rg_mf_lazy_flush: bad opt");
    if (!t->user_w_out || !t->user_b_out) return fail_arg("rg_mf_lazy_flush: null other-set user tables");
    ApplyArgs a{};
    a.w_in[0] = t->user_w; a.b_in[0] = t->user_b; a.w_out[0] = t->user_w_out; a.b_out[0] = t->user_b_out;
    a.w_m[0] = t->user_w_m; a.w_v[0] = t->user_w_v; a.b_m[0] = t->user_b_m; a.b_v[0] = t->user_b_v;
    if (opt->kind == RG_OPT_ADAM && (!a.w_m[0] || !a.b_m[0])) return fail_arg("rg_mf_lazy_flush: Adam needs m");
    if (opt->kind != RG_OPT_SGD && (!a.w_v[0] || !a.b_v[0])) return fail_arg("rg_mf_lazy_flush: needs v");
    a.num_users = t->num_users; a.num_items = t->num_items; a.dim = t->dim;
    a.opt = *opt;
    a.has_bias = true;
    if ((rc = lazy_args(lazy, opt, a))) return rc;
    FlushLaunchF f{&a, (hipStream_t)stream};
    return dispatch_dim(t->dim, f);
}

namespace rg {
int apply_prepare_owner(void *stream, const rg_mf_tables_t *t, rg_mf_work_t *w, const rg_opt_t *opt,
                        int64_t row_begin, int64_t row_end, const rg_mf_loss_t *loss,
                        const rg_mf_owner_batch_t *next) {
    ApplyArgs a;
    int rc = apply_args(t, w, nullptr, nullptr, opt, row_begin, row_end, loss, nullptr, kApplyPull, a);
    if (rc) return rc;
    PairsArgs prep{};
    OwnerArgs oa{};
    int64_t prep_blocks = 0;
    if (next) {
        if ((rc = owner_args(next, oa))) return rc;
        prep_blocks = oa.segs;
    }
    BackLaunchF f{&a, &prep, nullptr, prep_blocks, MtGenArgs{}, (hipStream_t)stream, next ? &oa : nullptr};
    return dispatch_dim(t->dim, f);
}
}  // namespace rg

extern "C" int rg_mf_step_front(void *stream, const rg_mf_tables_t *t, const rg_mf_batch_t *cur, rg_mf_work_t *w,
                                const rg_mf_mark_t *cur_mark, const rg_opt_t *opt, int64_t cold_begin,
                                int64_t cold_end, const rg_mf_batch_t *next, const rg_mf_work_t *next_w,
                                const rg_mf_mark_t *next_mark) {
    if (kPairBlock != kBlock) return fail_arg("rg_mf_step_front: built with a pair-pass workgroup != 256 threads");
    if (!cur_mark || !cur_mark->stamp || cur_mark->serial == 0)
        return fail_arg("rg_mf_step_front: the current step's pairs must be prepared with row marks");
    if (cur && cur->loss == RG_LOSS_ADAPTIVE_HINGE)
        return fail_arg("rg_mf_step_front: adaptive hinge needs the global max first (use rg_mf_pairs)");
    PairsArgs pa, prep{};
    int rc = pairs_args(t, cur, w, 1, pa);
    if (rc) return rc;
    ApplyArgs aa;
    if ((rc = apply_args(t, w, nullptr, nullptr, opt, cold_begin, cold_end, nullptr, nullptr, kApplyPull, aa)))
        return rc;
    FrontArgs f{};
    f.cold_stamp = cur_mark->stamp;
    f.cold_serial = cur_mark->serial;
    if (next) {
        if (!next_mark || next_mark->stamp == cur_mark->stamp || next_mark->serial == cur_mark->serial)
            return fail_arg("rg_mf_step_front: the next step needs its own stamp array and serial");
        if ((rc = prepare_args(next, next_w, next_mark, prep))) return rc;
        if (next->pairs == cur->pairs) return fail_arg("rg_mf_step_front: next pairs buffer aliases the current");
        f.prep_out = reinterpret_cast<int2 *>(next->pairs);
        f.prep_blocks = (prepare_threads(next->cols, next->n_neg) + kBlock - 1) / kBlock;
    }
    FrontLaunchF fl{&pa, &prep, &aa, f, (hipStream_t)stream};
    return dispatch_dim(t->dim, fl);
}

namespace {
struct ColdLaunchF {
    ApplyArgs *a;
    const rg_mf_mark_t *mark;
    hipStream_t s;
    template <class L>
    int operator()() {
        const int64_t rows = a->row_end - a->row_begin;
        if (rows <= 0) return RG_OK;
        const int64_t waves = (rows + L::UPW - 1) / L::UPW;
        const int64_t nb = (waves + kBlock / kWave - 1) / (kBlock / kWave);
        hipLaunchKernelGGL((mf_cold_kernel<L>), dim3(nb), dim3(kBlock), 0, s, *a, mark->stamp, mark->serial);
        return check_launch("rg_mf_step_cold");
    }
};
}  // namespace

extern "C" int rg_mf_step_cold(void *stream, const rg_mf_tables_t *t, const rg_mf_mark_t *mark, const rg_opt_t *opt,
                               int64_t row_begin, int64_t row_end) {
    if (!mark || !mark->stamp || mark->serial == 0) return fail_arg("rg_mf_step_cold: bad mark");
    ApplyArgs a;
    int rc = apply_args(t, nullptr, nullptr, nullptr, opt, row_begin, row_end, nullptr, nullptr, kApplyCold, a);
    if (rc) return rc;
    ColdLaunchF f{&a, mark, (hipStream_t)stream};
    return dispatch_dim(t->dim, f);
}

extern "C" int rg_mf_step_hot(void *stream, const rg_mf_tables_t *t, const rg_mf_batch_t *cur, rg_mf_work_t *w,
                              const rg_mf_mark_t *mark, const rg_opt_t *opt, int64_t row_begin, int64_t row_end,
                              const rg_mf_loss_t *loss) {
    if (!cur || !cur->pairs) return fail_arg("rg_mf_step_hot: null batch/pairs");
    if (mark && (!mark->stamp || mark->serial == 0)) return fail_arg("rg_mf_step_hot: bad mark");
    ApplyArgs a;
    int rc = apply_args(t, w, nullptr, nullptr, opt, row_begin, row_end, loss, nullptr, kApplyPull, a);
    if (rc) return rc;
    HotLaunchF f{&a, reinterpret_cast<const int2 *>(cur->pairs), 2 * (int64_t)pair_stride(cur->n_neg) * cur->cols,
                 pair_stride(cur->n_neg), 1 + cur->n_neg, mark,
                 (hipStream_t)stream};
    return dispatch_dim(t->dim, f);
}

static int ncf_apply_args(const rg_ncf_model_t *m, rg_mf_work_t *w, const float *contrib, const rg_opt_t *opt,
                          int64_t row_begin, int64_t row_end, ApplyArgs &a);
static int neumf_gmf_pass(void *stream, const rg_ncf_model_t *m, rg_mf_work_t *w, const rg_ncf_work_t *nw,
                          const rg_opt_t *opt, int64_t row_begin, int64_t row_end, const MtGenArgs &gen);

extern "C" int rg_ncf_apply(void *stream, const rg_ncf_model_t *m, rg_mf_work_t *w, const float *contrib,
                            const rg_opt_t *opt, int64_t row_begin, int64_t row_end) {
    ApplyArgs a{};
    const int rc = ncf_apply_args(m, w, contrib, opt, row_begin, row_end, a);
    if (rc) return rc;
    ApplyLaunchF f{&a, (hipStream_t)stream, kApplyPull};
    return dispatch_dim(m->dim, f);
}

// The tail of a single-GPU NCF step in one launch (mf_back_kernel's grid): the next step's
// prepare (next = NULL: none), the MLP update from the pair kernel's weight-gradient partials
// (rg_ncf_update's reduction and optimizer, the same sums) with the step's loss, and the
// embedding rows' update (rg_ncf_apply) -- three launches and their tails in one; the three
// parts touch disjoint data.  NeuMF (mf_dim > 0): the GMF tables' pass runs first, in a launch
// of its own (it keeps the per-row counts the MLP tables' pass then consumes), as rg_neumf_apply.
// gen (optional, rg_mf_stepper_tail_gen): workgroup 0 walks a later step's MT words, as in the
// MF split step's dense pass -- no generator-stream kernel beside the pair kernel.
// every check of rg_ncf_tail that does not depend on the stepper's outputs (next batch, MT walk):
// the engine runs it BEFORE the stepper bookkeeping calls (rg_mf_stepper_prefetch_args /
// rg_mf_stepper_tail_gen commit the next unit and the ring slot), so a refused tail never
// leaves the stepper believing a prepare or a walk was launched
static int ncf_tail_checks(const rg_ncf_model_t *m, rg_mf_work_t *w, const rg_ncf_work_t *nw, int64_t nparts,
                           const rg_opt_t *opt, const float *loss_partials, const rg_mf_loss_t *loss, ApplyArgs &a,
                           int64_t &P) {
    if (!m || !w || !nw || !opt || !nw->contrib || !nw->mlp_partials || !m->mlp)
        return fail_arg("rg_ncf_tail: null argument");
    if (opt->kind == RG_OPT_ADAM && !m->mlp_m) return fail_arg("rg_ncf_tail: Adam needs m state");
    if (opt->kind != RG_OPT_SGD && !m->mlp_v) return fail_arg("rg_ncf_tail: optimizer needs v state");
    P = m->mf_dim == 0 ? rg_ncf_mlp_len(m->dim) : rg_neumf_param_len(m->dim, m->mf_dim);
    if (P < 0 || nparts < 1) return fail_arg("rg_ncf_tail: bad dim / mf_dim / partial count");
    if (loss && loss->out && !loss_partials) return fail_arg("rg_ncf_tail: loss needs partials");
    if (m->dim < 1 || m->dim > 256) return fail_arg("rg_ncf_tail: dim must be in [1, 256]");
    return ncf_apply_args(m, w, nw->contrib, opt, 0, -1, a);
}

extern "C" int rg_ncf_tail_validate(const rg_ncf_model_t *m, rg_mf_work_t *w, const rg_ncf_work_t *nw,
                                    int64_t nparts, const rg_opt_t *opt, const float *loss_partials,
                                    const rg_mf_loss_t *loss) {
    ApplyArgs a{};
    int64_t P = 0;
    return ncf_tail_checks(m, w, nw, nparts, opt, loss_partials, loss, a, P);
}

extern "C" int rg_ncf_tail(void *stream, const rg_ncf_model_t *m, rg_mf_work_t *w, const rg_ncf_work_t *nw,
                           int64_t nparts, const rg_opt_t *opt, const float *loss_partials, const rg_mf_loss_t *loss,
                           const rg_mf_batch_t *next, const rg_mf_work_t *next_w, const rg_mt_gen_t *gen) {
    ApplyArgs a{};
    int64_t P = 0;
    int rc = ncf_tail_checks(m, w, nw, nparts, opt, loss_partials, loss, a, P);
    if (rc) return rc;
    MtGenArgs g{};
    if (gen && gen->nwords > 0) {
        if (!gen->state || !gen->out) return fail_arg("rg_ncf_tail: null MT state / output");
        g.state = gen->state; g.out = gen->out; g.state_before = gen->state_before; g.nwords = gen->nwords;
    }
    // NeuMF: the GMF tables' pass first; the walk (if any) rides in that launch -- the longer of
    // the two passes at the reference's sizes (mf 50 vs mlp 16 floats per row)
    if (m->mf_dim != 0) {
        if ((rc = neumf_gmf_pass(stream, m, w, nw, opt, 0, -1, g))) return rc;
        g = MtGenArgs{};
    }
    if (loss && loss->out) {   // finalized by the dense blocks' first workgroup (rg_ncf_update's sums)
        a.partials = loss_partials;
        a.n_partials = loss->n_partials;
        a.inv_a = loss->inv_a;
        a.inv_b = loss->inv_b;
        a.loss_out = loss->out;
    }
    MlpUpdArgs u{};
    u.mlp = m->mlp;
    u.m = opt->kind == RG_OPT_ADAM ? m->mlp_m : nullptr;
    u.v = opt->kind == RG_OPT_SGD ? nullptr : m->mlp_v;
    u.wpart = nw->mlp_partials;
    u.nparts = (int)nparts;
    u.P = (int)P;
    u.opt = *opt;
    u.mode = 0;
    PairsArgs prep{};
    int2 *prep_out = nullptr;
    int64_t prep_blocks = 0;
    if (next) {
        if ((rc = prepare_args(next, next_w, nullptr, prep))) return rc;
        if (next->pairs == nullptr) return fail_arg("rg_ncf_tail: null next pairs");
        prep_out = reinterpret_cast<int2 *>(next->pairs);
        prep_blocks = (prepare_threads(next->cols, next->n_neg) + kBlock - 1) / kBlock;
    }
    BackLaunchF f{&a, &prep, prep_out, prep_blocks, g, (hipStream_t)stream};
    f.upd = &u;
    return dispatch_dim(m->dim, f);
}

static int ncf_apply_args(const rg_ncf_model_t *m, rg_mf_work_t *w, const float *contrib, const rg_opt_t *opt,
                          int64_t row_begin, int64_t row_end, ApplyArgs &a) {
    if (!m || !w || !opt || !contrib || !m->user_w || !m->item_w) return fail_arg("rg_ncf_apply: null argument");
    if (!w->row_count || !w->row_list || !w->hot_grad) return fail_arg("rg_ncf_apply: null scratch");
    if (opt->kind == RG_OPT_ADAM && (!m->user_w_m || !m->item_w_m)) return fail_arg("rg_ncf_apply: Adam needs m");
    if (opt->kind != RG_OPT_SGD && (!m->user_w_v || !m->item_w_v)) return fail_arg("rg_ncf_apply: needs v");
    if (w->plan_perm && !w->part_row) return fail_arg("rg_ncf_apply: plan needs part_row");
    const int64_t nrows = m->num_users + m->num_items;
    if (row_begin < 0) row_begin = 0;
    if (row_end < 0 || row_end > nrows) row_end = nrows;
    if (row_begin > row_end) return fail_arg("rg_ncf_apply: row_begin > row_end");
    a = ApplyArgs{};
    a.w_in[0] = m->user_w; a.w_in[1] = m->item_w;
    a.w_out[0] = m->user_w; a.w_out[1] = m->item_w;          // in place: no partner rows are read
    a.w_m[0] = m->user_w_m; a.w_m[1] = m->item_w_m; a.w_v[0] = m->user_w_v; a.w_v[1] = m->item_w_v;
    a.num_users = m->num_users; a.num_items = m->num_items; a.dim = m->dim;
    a.row_begin = row_begin; a.row_end = row_end;
    a.row_count = w->row_count; a.row_list = reinterpret_cast<const int2 *>(w->row_list);
    a.hot_grad = reinterpret_cast<long long *>(w->hot_grad);
    if (w->plan_perm) { a.item_slot_off = w->plan_item_slot_off; a.part_row = w->part_row; }
    a.opt = *opt;
    a.contrib = contrib;
    a.contrib_stride = 2 * (int64_t)m->dim;
    a.has_bias = false;
    return RG_OK;
}

// Data-parallel NCF / NeuMF step (replicated, reference-exact): the embedding rows' data
// gradient pulled from the lists into the flat buffer (before the exchange), and the
// in-place update of every row from the summed buffer (after it).  gmf: the NeuMF GMF tables
// (their rows from ncf_work->mf_contrib; the lists are kept for the MLP tables' pass).
static int ncf_table_args(const rg_ncf_model_t *m, rg_mf_work_t *w, const rg_ncf_work_t *nw, int gmf,
                          int64_t row_begin, int64_t row_end, ApplyArgs &a) {
    if (!m) return fail_arg("rg_ncf_grads: null model");
    if (gmf && (m->mf_dim < 1 || !m->mf_user_w || !m->mf_item_w)) return fail_arg("rg_ncf_grads: no GMF tables");
    const int64_t nrows = m->num_users + m->num_items;
    if (row_begin < 0) row_begin = 0;
    if (row_end < 0 || row_end > nrows) row_end = nrows;
    if (row_begin > row_end) return fail_arg("rg_ncf_grads: row_begin > row_end");
    a = ApplyArgs{};
    a.w_in[0] = gmf ? m->mf_user_w : m->user_w;
    a.w_in[1] = gmf ? m->mf_item_w : m->item_w;
    a.w_out[0] = const_cast<float *>(a.w_in[0]);
    a.w_out[1] = const_cast<float *>(a.w_in[1]);
    a.w_m[0] = gmf ? m->mf_user_m : m->user_w_m; a.w_m[1] = gmf ? m->mf_item_m : m->item_w_m;
    a.w_v[0] = gmf ? m->mf_user_v : m->user_w_v; a.w_v[1] = gmf ? m->mf_item_v : m->item_w_v;
    a.num_users = m->num_users; a.num_items = m->num_items; a.dim = gmf ? m->mf_dim : m->dim;
    a.row_begin = row_begin; a.row_end = row_end;
    if (w) {
        if (!w->row_count || !w->row_list || !nw) return fail_arg("rg_ncf_grads: null scratch");
        a.row_count = w->row_count; a.row_list = reinterpret_cast<const int2 *>(w->row_list);
        a.hot_grad = reinterpret_cast<long long *>(gmf ? nw->mf_hot_grad : w->hot_grad);
        a.contrib = gmf ? nw->mf_contrib : nw->contrib;
        a.contrib_stride = 2 * (int64_t)a.dim;
        a.keep_count = gmf != 0;
        if (w->plan_perm) {
            a.item_slot_off = w->plan_item_slot_off;
            a.part_row = gmf ? nw->mf_part_row : w->part_row;
        }
        if (!a.hot_grad || !a.contrib) return fail_arg("rg_ncf_grads: null contribution rows / overflow rows");
    }
    a.has_bias = false;
    return RG_OK;
}

extern "C" int rg_ncf_grads(void *stream, const rg_ncf_model_t *m, rg_mf_work_t *w, const rg_ncf_work_t *nw,
                            float *grad, int64_t row_begin, int64_t row_end, int32_t gmf) {
    if (!w || !nw || !grad) return fail_arg("rg_ncf_grads: null argument");
    ApplyArgs a;
    int rc = ncf_table_args(m, w, nw, gmf, row_begin, row_end, a);
    if (rc) return rc;
    a.grad = grad;
    ApplyLaunchF f{&a, (hipStream_t)stream, kGradOnly};
    return dispatch_dim(a.dim, f);
}

extern "C" int rg_ncf_apply_dense(void *stream, const rg_ncf_model_t *m, const float *grad, const rg_opt_t *opt,
                                  int64_t row_begin, int64_t row_end, int32_t gmf) {
    if (!grad || !opt) return fail_arg("rg_ncf_apply_dense: null argument");
    ApplyArgs a;
    int rc = ncf_table_args(m, nullptr, nullptr, gmf, row_begin, row_end, a);
    if (rc) return rc;
    if (opt->kind == RG_OPT_ADAM && (!a.w_m[0] || !a.w_m[1])) return fail_arg("rg_ncf_apply_dense: Adam needs m");
    if (opt->kind != RG_OPT_SGD && (!a.w_v[0] || !a.w_v[1])) return fail_arg("rg_ncf_apply_dense: needs v");
    a.opt = *opt;
    a.grad = const_cast<float *>(grad);
    ApplyLaunchF f{&a, (hipStream_t)stream, kApplyDense};
    return dispatch_dim(a.dim, f);
}

// NeuMF (spotlight/dnn_models/neuMF.py:7-55): the GMF tables take their gradient rows
// from ncf_work->mf_contrib through the same per-row lists (kept), then the MLP tables
// pull theirs and reset the lists (rg_ncf_apply).
// NeuMF's GMF tables: pull + optimizer through the same per-row lists, keeping the counts for
// the MLP tables' pass that follows (rg_ncf_apply or rg_ncf_tail resets them)
static int neumf_gmf_pass(void *stream, const rg_ncf_model_t *m, rg_mf_work_t *w, const rg_ncf_work_t *nw,
                          const rg_opt_t *opt, int64_t row_begin, int64_t row_end, const MtGenArgs &gen) {
    if (!m || !w || !nw || !opt) return fail_arg("rg_neumf_apply: null argument");
    if (m->mf_dim < 1 || m->mf_dim > RG_NEUMF_MAX_MF_DIM) return fail_arg("rg_neumf_apply: mf_dim out of range");
    if (!m->mf_user_w || !m->mf_item_w || !nw->mf_contrib || !nw->mf_hot_grad)
        return fail_arg("rg_neumf_apply: null GMF table / scratch");
    if (w->plan_perm && !nw->mf_part_row) return fail_arg("rg_neumf_apply: plan needs mf_part_row");
    if (opt->kind == RG_OPT_ADAM && (!m->mf_user_m || !m->mf_item_m)) return fail_arg("rg_neumf_apply: Adam needs m");
    if (opt->kind != RG_OPT_SGD && (!m->mf_user_v || !m->mf_item_v)) return fail_arg("rg_neumf_apply: needs v");
    if (!w->row_count || !w->row_list) return fail_arg("rg_neumf_apply: null scratch");
    const int64_t nrows = m->num_users + m->num_items;
    int64_t rb = row_begin < 0 ? 0 : row_begin, re = row_end < 0 || row_end > nrows ? nrows : row_end;
    if (rb > re) return fail_arg("rg_neumf_apply: row_begin > row_end");
    ApplyArgs a{};
    a.w_in[0] = m->mf_user_w; a.w_in[1] = m->mf_item_w;
    a.w_out[0] = m->mf_user_w; a.w_out[1] = m->mf_item_w;
    a.w_m[0] = m->mf_user_m; a.w_m[1] = m->mf_item_m; a.w_v[0] = m->mf_user_v; a.w_v[1] = m->mf_item_v;
    a.num_users = m->num_users; a.num_items = m->num_items; a.dim = m->mf_dim;
    a.row_begin = rb; a.row_end = re;
    a.row_count = w->row_count; a.row_list = reinterpret_cast<const int2 *>(w->row_list);
    a.hot_grad = reinterpret_cast<long long *>(nw->mf_hot_grad);
    if (w->plan_perm) { a.item_slot_off = w->plan_item_slot_off; a.part_row = nw->mf_part_row; }
    a.opt = *opt;
    a.contrib = nw->mf_contrib;
    a.contrib_stride = 2 * (int64_t)m->mf_dim;
    a.has_bias = false;
    a.keep_count = true;
    if (gen.nwords > 0) {   // with an MT walk: mf_back_kernel's grid (walk block + the same pull)
        PairsArgs prep{};
        BackLaunchF f{&a, &prep, nullptr, 0, gen, (hipStream_t)stream};
        return dispatch_dim(m->mf_dim, f);
    }
    ApplyLaunchF f{&a, (hipStream_t)stream, kApplyPull};
    return dispatch_dim(m->mf_dim, f);
}

extern "C" int rg_neumf_apply(void *stream, const rg_ncf_model_t *m, rg_mf_work_t *w, const rg_ncf_work_t *nw,
                              const rg_opt_t *opt, int64_t row_begin, int64_t row_end) {
    const int rc = neumf_gmf_pass(stream, m, w, nw, opt, row_begin, row_end, MtGenArgs{});
    if (rc) return rc;
    return rg_ncf_apply(stream, m, w, nw->contrib, opt, row_begin, row_end);
}

extern "C" int rg_mf_apply(void *stream, const rg_mf_tables_t *t, rg_mf_work_t *w, const rg_opt_t *opt,
                           int64_t row_begin, int64_t row_end, const rg_mf_loss_t *loss) {
    return apply_common(stream, t, w, nullptr, nullptr, opt, row_begin, row_end, loss, nullptr, kApplyPull);
}

extern "C" int rg_mf_grads(void *stream, const rg_mf_tables_t *t, rg_mf_work_t *w, float *grad_dev,
                           int64_t row_begin, int64_t row_end, const rg_mf_loss_t *loss) {
    if (!grad_dev) return fail_arg("rg_mf_grads: null grad");
    return apply_common(stream, t, w, nullptr, grad_dev, nullptr, row_begin, row_end, loss, nullptr, kGradOnly);
}

extern "C" int rg_mf_apply_dense(void *stream, const rg_mf_tables_t *t, const float *grad_dev, const rg_opt_t *opt,
                                 int64_t row_begin, int64_t row_end, float *loss_out_dev) {
    if (!grad_dev) return fail_arg("rg_mf_apply_dense: null grad");
    return apply_common(stream, t, nullptr, grad_dev, nullptr, opt, row_begin, row_end, nullptr, loss_out_dev,
                        kApplyDense);
}

extern "C" int64_t rg_mf_grad_chunk(int64_t shard_users, int64_t shard_items, int32_t dim) {
    if (shard_users < 1 || shard_items < 1 || dim < 1) return -1;
    return ((shard_users + shard_items) * (int64_t)(dim + 1) + 1 + 3) / 4 * 4;
}

static int shard_args(const rg_mf_tables_t *t, int64_t su, int64_t si, int32_t world, int32_t rank, ApplyArgs &a) {
    if (world < 1 || rank < 0 || rank >= world) return fail_arg("rg_mf sharded: bad rank / world");
    if (su < 1 || si < 1 || su * world < t->num_users || si * world < t->num_items)
        return fail_arg("rg_mf sharded: shards do not cover the tables");
    a.shard_users = su;
    a.shard_items = si;
    a.chunk = rg_mf_grad_chunk(su, si, t->dim);
    a.world = world;
    a.rank = rank;
    return RG_OK;
}

extern "C" int rg_mf_grads_sharded(void *stream, const rg_mf_tables_t *t, rg_mf_work_t *w, float *grad_dev,
                                   int64_t shard_users, int64_t shard_items, int32_t world, const rg_mf_loss_t *loss) {
    if (!grad_dev) return fail_arg("rg_mf_grads_sharded: null grad");
    ApplyArgs a;
    int rc = apply_args(t, w, nullptr, grad_dev, nullptr, 0, -1, loss, nullptr, kGradOnly, a);
    if (rc || (rc = shard_args(t, shard_users, shard_items, world, 0, a))) return rc;
    ApplyLaunchF f{&a, (hipStream_t)stream, kGradOnly};
    return dispatch_dim(t->dim, f);
}

extern "C" int rg_mf_apply_shard(void *stream, const rg_mf_tables_t *t, const float *grad_dev, const rg_opt_t *opt,
                                 int64_t shard_users, int64_t shard_items, int32_t world, int32_t rank,
                                 float *loss_out_dev) {
    if (!grad_dev) return fail_arg("rg_mf_apply_shard: null grad");
    ApplyArgs a;
    int rc = apply_args(t, nullptr, grad_dev, nullptr, opt, 0, -1, nullptr, loss_out_dev, kApplyDense, a);
    if (rc || (rc = shard_args(t, shard_users, shard_items, world, rank, a))) return rc;
    const int64_t u0 = rank * shard_users, i0 = rank * shard_items;
    const int64_t nu = u0 < t->num_users ? std::min(shard_users, t->num_users - u0) : 0;
    const int64_t ni = i0 < t->num_items ? std::min(shard_items, t->num_items - i0) : 0;
    a.row_begin = 0;
    a.row_end = nu + ni;            // rows of the shard, mapped in mf_apply_kernel
    ApplyLaunchF f{&a, (hipStream_t)stream, kApplyDense};
    return dispatch_dim(t->dim, f);
}

extern "C" int64_t rg_mf_item_grad_chunk(int64_t shard_items, int32_t dim) {
    if (shard_items < 1 || dim < 1) return -1;
    return (shard_items * (int64_t)(dim + 1) + 1 + 3) / 4 * 4;
}

static int item_shard_args(const rg_mf_tables_t *t, int64_t si, int32_t world, int32_t rank, ApplyArgs &a) {
    if (world < 1 || rank < 0 || rank >= world) return fail_arg("rg_mf item shard: bad rank / world");
    if (si < 1 || si * world < t->num_items) return fail_arg("rg_mf item shard: shards do not cover the items");
    a.shard_users = 0;
    a.shard_items = si;
    a.item_shard = 1;
    a.chunk = rg_mf_item_grad_chunk(si, t->dim);
    a.world = world;
    a.rank = rank;
    return RG_OK;
}

extern "C" int rg_mf_grads_item_shard(void *stream, const rg_mf_tables_t *t, rg_mf_work_t *w, float *grad_dev,
                                      int64_t shard_items, int32_t world, const rg_mf_loss_t *loss) {
    if (!grad_dev) return fail_arg("rg_mf_grads_item_shard: null grad");
    ApplyArgs a;
    int rc = apply_args(t, w, nullptr, grad_dev, nullptr, t->num_users, t->num_users + t->num_items, loss, nullptr,
                        kGradOnly, a);
    if (rc || (rc = item_shard_args(t, shard_items, world, 0, a))) return rc;
    ApplyLaunchF f{&a, (hipStream_t)stream, kGradOnly};
    return dispatch_dim(t->dim, f);
}

extern "C" int rg_mf_apply_item_shard(void *stream, const rg_mf_tables_t *t, const float *grad_dev,
                                      const rg_opt_t *opt, int64_t shard_items, int32_t world, int32_t rank,
                                      float *loss_out_dev) {
    if (!grad_dev) return fail_arg("rg_mf_apply_item_shard: null grad");
    ApplyArgs a;
    int rc = apply_args(t, nullptr, grad_dev, nullptr, opt, 0, -1, nullptr, loss_out_dev, kApplyDense, a);
    if (rc || (rc = item_shard_args(t, shard_items, world, rank, a))) return rc;
    const int64_t i0 = rank * shard_items;
    a.row_begin = 0;
    a.row_end = i0 < t->num_items ? std::min(shard_items, t->num_items - i0) : 0;   // mapped in mf_apply_kernel
    ApplyLaunchF f{&a, (hipStream_t)stream, kApplyDense};
    return dispatch_dim(t->dim, f);
}

extern "C" int rg_loss_finalize(void *stream, const float *partials, int64_t n_partials, double inv_a,
                                double inv_b, float *out) {
    if (!partials || !out || n_partials < 0) return fail_arg("rg_loss_finalize: bad args");
    hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(kWave), 0, (hipStream_t)stream, partials, n_partials,
                       inv_a, inv_b, out);
    return check_launch("rg_loss_finalize");
}

extern "C" int rg_mf_scores(void *stream, const float *uw, const float *iw, const float *ub, const float *ib,
                            int32_t dim, const int64_t *users, const int64_t *items, int64_t n, float *out) {
    if (!uw || !iw || !ub || !ib || !users || !items || !out) return fail_arg("rg_mf_scores: null pointer");
    if (n < 0) return fail_arg("rg_mf_scores: n < 0");
    if (n == 0) return RG_OK;
    ScoresLaunchF f{uw, iw, ub, ib, dim, users, items, n, out, (hipStream_t)stream};
    return dispatch_dim(dim, f);
}

#ifdef RG_DIAG_STAMPS
extern "C" int rg_diag_set_stamps(unsigned long long *dev_buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(rg::g_diag_stamps), &dev_buf, sizeof(dev_buf)) == hipSuccess ? RG_OK
                                                                                                  : RG_E_LAUNCH;
}
extern "C" int rg_diag_set_flags(int flags) {
    return hipMemcpyToSymbol(HIP_SYMBOL(rg::g_diag_flags), &flags, sizeof(flags)) == hipSuccess ? RG_OK : RG_E_LAUNCH;
}
#endif
