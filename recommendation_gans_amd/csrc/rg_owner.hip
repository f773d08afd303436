// Owner-sharded data-parallel MF step (dp_mode 2): the per-rank passes around the score
// exchange.  See rg_owner.h and include/rg_hip.h (rg_mf_owner_*) for the layout.
//
// Reference semantics (implicit.py:347-364 at batch R*B): the scores, the loss terms and
// dL/dz of every pair are computed exactly as the single-GPU pair pass computes them
// (rg_mf.hip pairs_body: same dot-product layout, the same BPR / hinge / pointwise
// arithmetic in the same order), only split between the rank that owns the pair's user
// (scores, gradient rows) and the exchange of the scalar scores (the loss couples a
// column's positive with its negatives).  Row gradients go to the same per-row
// contribution lists, planned item partials and overflow rows the dense pass pulls.
#include "rg_owner.h"

namespace rg {
namespace {

constexpr int kBlk = 256;
constexpr int kCapO = RG_MF_LIST_CAP;
constexpr int kLdsF = 1280;   // >= units per block * (dim + 1) for every row layout

struct OwnTables {
    const float *user_w, *item_w, *user_b, *item_b;
    int64_t num_users;        // this rank's local users
    int32_t dim;
};

struct OwnWork {
    int32_t *row_count;
    int2 *row_list;
    long long *hot_grad, *hot_bias;      // int64 fixed point (rg_common.h fix_add)
    float *partials;
    float *part_row, *part_bias;
};

template <class L>
__device__ __forceinline__ void overflow_row(long long *__restrict__ hot, int64_t row, int D, int sub, float dz,
                                             const float (&o)[L::EPL]) {
#pragma unroll
    for (int e = 0; e < L::EPL; ++e) {
        const int c = L::elem(sub, e);
        if (L::VEC || c < D) fix_add(hot + row * (int64_t)D + c, dz * o[e]);
    }
}

// append {other, dz} to row's contribution list (the unit's lane sub == 0 claims the slot);
// a row touched more than kCapO times this step adds dz * partner row into the overflow
// accumulators instead (partner gathered again: rare)
template <class L>
__device__ __forceinline__ void append(const OwnWork &w, const OwnTables &t, int64_t row, int other,
                                       const float *partner_table, float dz, int sub, int ubase) {
    int sl = 0;
    if (sub == 0) sl = atomicAdd(w.row_count + row, 1);
    sl = __shfl(sl, ubase);
    if (sl < kCapO) {
        if (sub == 0) store_entry(w.row_list + row * kCapO + sl, other, dz);
    } else {
        float o[L::EPL];
        L::load(o, partner_table, other, t.dim, sub);
        overflow_row<L>(w.hot_grad, row, t.dim, sub, dz, o);
        if (sub == 0) fix_add(w.hot_bias + row, dz);
    }
}

// append at a slot the prepare claimed (no atomic; the overflow path as append's)
template <class L>
__device__ __forceinline__ void append_at(const OwnWork &w, const OwnTables &t, int64_t row, int other,
                                          const float *partner_table, float dz, int sub, int sl) {
    if (sl < kCapO) {
        if (sub == 0) store_entry(w.row_list + row * kCapO + sl, other, dz);
    } else {
        float o[L::EPL];
        L::load(o, partner_table, other, t.dim, sub);
        overflow_row<L>(w.hot_grad, row, t.dim, sub, dz, o);
        if (sub == 0) fix_add(w.hot_bias + row, dz);
    }
}

template <class L>
__device__ __forceinline__ float score(const OwnTables &t, int lu, int i, int sub) {
    constexpr int EPL = L::EPL;
    float ur[EPL], ir[EPL];
    L::load(ur, t.user_w, lu, t.dim, sub);
    L::load(ir, t.item_w, i, t.dim, sub);
    const float ub = t.user_b[lu], ib = t.item_b[i];
    float d = 0.0f;
#pragma unroll
    for (int e = 0; e < EPL; ++e) d = fmaf(ur[e], ir[e], d);
    d = group_sum<L::LPU>(d);
    return sigmoidf_ref((d + ub) + ib);
}

// Grid: [pos_blocks: the planned positives, units_per_block positions each]
//       [segs * npass: negative records; block (seg, pass) takes entries pass*UPB + unit,
//        stepping npass*UPB, of the segment's seg_count[seg]]
template <class L>
__global__ __launch_bounds__(kBlk) void owner_scores_kernel(OwnerArgs a, OwnTables t, int64_t pos_blocks, int npass) {
    constexpr int LPU = L::LPU, UPB = kBlk / LPU;
    const int lane = threadIdx.x & (kWave - 1), sub = lane & (LPU - 1);
    const int ublk = threadIdx.x / LPU;
    const int64_t blk = blockIdx.x;
    if (blk < pos_blocks) {
        const int64_t s = blk * UPB + ublk;
        const bool has = s < a.n_planned;
        const int64_t c = has ? a.perm[s] : 0;
        const int lu = has ? (int)(a.pos_user[c] / a.world) : 0;
        const int i = has ? (int)a.pos_item[c] : 0;
        const float p = score<L>(t, lu, i, sub);
        if (has && sub == 0) a.scores[c] = p;
        return;
    }
    const int64_t q = blk - pos_blocks, seg = q / npass, pass = q - seg * npass;
    const int cnt = a.seg_count[seg];
    for (int e = (int)pass * UPB + ublk; e < cnt; e += npass * UPB) {
        const int4 r = a.rec[seg * kOwnSeg + e];
        const float p = score<L>(t, r.y, r.z, sub);
        if (sub == 0) a.scores[r.x] = p;
    }
}

template <class L, int NMAX>
__global__ __launch_bounds__(kBlk) void owner_back_kernel(OwnerArgs a, OwnTables t, OwnWork w, int64_t pos_blocks,
                                                          int npass) {
    constexpr int LPU = L::LPU, EPL = L::EPL, UPB = kBlk / LPU;
    __shared__ float red[2][kBlk / kWave];
    __shared__ float lrow[kLdsF];
    __shared__ int lslot[UPB];
    const int lane = threadIdx.x & (kWave - 1), sub = lane & (LPU - 1), ubase = lane & ~(LPU - 1);
    const int ublk = threadIdx.x / LPU;
    const int64_t blk = blockIdx.x;
    const int D = t.dim, n = a.n_neg;
    const int64_t U = t.num_users, gc = a.gc;
    const bool pairwise = (a.loss == RG_LOSS_BPR) || (a.loss == RG_LOSS_HINGE);
    const float g = 1.0f / a.n_a;
    float la = 0.0f, lb = 0.0f;
    if (blk < pos_blocks) {
        // ---- a planned positive: its column's scores -> dL/dp (pairs_body's arithmetic) ----
        const int64_t s = blk * UPB + ublk;
        const bool has = s < a.n_planned;
        const int64_t c = has ? a.perm[s] : 0;
        const int lu = has ? (int)(a.pos_user[c] / a.world) : 0;
        const int i = has ? (int)a.pos_item[c] : 0;
        const int myslot = has ? a.pos_slot[s] : -1;
        float ur[EPL];
        L::load(ur, t.user_w, lu, D, sub);          // the planned item-side partial: dz * user row
        const float p0 = a.scores[c];
        float dp0 = 0.0f;
        if (a.loss == RG_LOSS_ADAPTIVE_HINGE) {   // hinge against the global max negative (owner_adapt_kernel)
            const float x = (a.scores[adapt_slot(a)] - p0) + 1.0f;
            la = fmaxf(x, 0.0f);
            if (x >= 0.0f) dp0 = -(1.0f / a.n_a);
        } else if (pairwise) {
#pragma unroll
            for (int k = 0; k < NMAX; ++k) {
                if (k < n) {
                    const float pk = a.scores[(1 + k) * gc + c];
                    if (a.loss == RG_LOSS_BPR) {
                        const float sg = sigmoidf_ref(p0 - pk);
                        la += 1.0f - sg;
                        const float dx = (-g) * (1.0f - sg) * sg;
                        dp0 += dx;
                    } else {
                        const float x = (pk - p0) + 1.0f;
                        la += fmaxf(x, 0.0f);
                        dp0 -= x >= 0.0f ? g : 0.0f;
                    }
                }
            }
        } else {
            la = -fmaxf(logf(p0), -100.0f);
            dp0 = ((p0 - 1.0f) / fmaxf((1.0f - p0) * p0, 1e-12f)) / a.n_a;
        }
        if (!has) { la = 0.0f; dp0 = 0.0f; }
        const float dz = (dp0 * (1.0f - p0)) * p0;
        if (has) append<L>(w, t, lu, i, t.item_w, dz, sub, ubase);
        // block-level segmented sum of the item-side rows (positions sorted by item)
        const int stride = D + 1;
        if (has) {
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                const int cc = L::elem(sub, e);
                if (L::VEC || cc < D) lrow[ublk * stride + cc] = dz * ur[e];
            }
            if (sub == 0) lrow[ublk * stride + D] = dz;
        }
        if (sub == 0) lslot[ublk] = myslot;
        __syncthreads();
        if (has && (ublk == 0 || lslot[ublk - 1] != myslot)) {   // segment head
            float acc[EPL];
            float accb = 0.0f;
            L::zero(acc);
            for (int v = ublk; v < UPB && lslot[v] == myslot; ++v) {
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    const int cc = L::elem(sub, e);
                    if (L::VEC || cc < D) acc[e] += lrow[v * stride + cc];
                }
                accb += lrow[v * stride + D];
            }
            L::store(w.part_row, myslot, D, sub, acc);
            if (sub == 0) w.part_bias[myslot] = accb;
        }
    } else {
        // ---- negatives this rank owns ------------------------------------------------
        const int64_t q = blk - pos_blocks, seg = q / npass, pass = q - seg * npass;
        const int cnt = a.seg_count[seg];
        for (int e = (int)pass * UPB + ublk; e < cnt; e += npass * UPB) {
            const int4 r = a.rec[seg * kOwnSeg + e];
            const int64_t gp = r.x, k1 = gp / gc, c = gp - k1 * gc;
            const int lu = r.y, i = r.z;
            const float pk = a.scores[gp];
            float dpk;
            if (a.loss == RG_LOSS_ADAPTIVE_HINGE) {
                // only the global max negative has a gradient: the active positives' count / B
                const float *ex = a.scores + adapt_slot(a);
                if (gp != (int64_t)__float_as_int(ex[1])) continue;
                dpk = ex[2] * (1.0f / a.n_a);
            } else if (pairwise) {
                const float p0 = a.scores[c];
                if (a.loss == RG_LOSS_BPR) {
                    const float sg = sigmoidf_ref(p0 - pk);
                    const float dx = (-g) * (1.0f - sg) * sg;
                    dpk = -dx;
                } else {
                    const float x = (pk - p0) + 1.0f;
                    dpk = x >= 0.0f ? g : 0.0f;
                }
            } else {
                lb += -fmaxf(logf(1.0f - pk), -100.0f);
                dpk = (pk / fmaxf((1.0f - pk) * pk, 1e-12f)) / a.n_b;
            }
            const float dz = (dpk * (1.0f - pk)) * pk;
            if (a.claim != nullptr) {
                append_at<L>(w, t, lu, i, t.item_w, dz, sub, r.w & 0xff);
                append_at<L>(w, t, U + i, lu, t.user_w, dz, sub, (r.w >> 8) & 0xff);
            } else {
                append<L>(w, t, lu, i, t.item_w, dz, sub, ubase);
                append<L>(w, t, U + i, lu, t.user_w, dz, sub, ubase);
            }
        }
    }
    // ---- deterministic loss partials: wave DPP sum -> block -> partials[block] --------
    float va = sub == 0 ? la : 0.0f, vb = sub == 0 ? lb : 0.0f;
    va = group_sum<kWave>(va);
    vb = group_sum<kWave>(vb);
    const int wv = threadIdx.x >> 6;
    if (lane == 0) { red[0][wv] = va; red[1][wv] = vb; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float sa = 0.0f, sb = 0.0f;
#pragma unroll
        for (int k = 0; k < kBlk / kWave; ++k) { sa += red[0][k]; sb += red[1][k]; }
        w.partials[2 * blk] = sa;
        w.partials[2 * blk + 1] = sb;
    }
}

__global__ __launch_bounds__(kBlk) void owner_prepare_kernel(OwnerArgs a) { owner_prepare_block(a, blockIdx.x); }

// Adaptive hinge (implicit.py:194-199 'bpr' / 'adaptive_hinge', spotlight/losses.py:133-172)
// on the owner layout: after the exchange every rank holds every score, so each finds the
// global max negative (largest score, first draw on ties -- torch.max over the flat draw) and
// the count of active positives itself, identically, with no further exchange; stored in
// the score buffer's extra slots [(1 + n) * GC + {0, 1, 2}] = (max, its pair index gp, count)
__device__ __forceinline__ void block_max_first(float &v, int64_t &i, float *sv, int64_t *si) {
    const int tid = threadIdx.x;
    sv[tid] = v;
    si[tid] = i;
    __syncthreads();
    for (int w = blockDim.x >> 1; w > 0; w >>= 1) {
        if (tid < w && (sv[tid + w] > sv[tid] || (sv[tid + w] == sv[tid] && si[tid + w] < si[tid]))) {
            sv[tid] = sv[tid + w];
            si[tid] = si[tid + w];
        }
        __syncthreads();
    }
    v = sv[0];
    i = si[0];
    __syncthreads();
}

__global__ __launch_bounds__(1024) void owner_adapt_kernel(OwnerArgs a) {
    __shared__ float sv[1024];
    __shared__ int64_t si[1024];
    const int64_t gc = a.gc, end = (int64_t)(1 + a.n_neg) * gc;
    float best = -1.0f;
    int64_t bi = INT64_MAX;
    for (int64_t g = gc + threadIdx.x; g < end; g += 1024) {
        const float v = a.scores[g];
        if (v > best) { best = v; bi = g; }
    }
    block_max_first(best, bi, sv, si);
    float cnt = 0.0f;
    for (int64_t c = threadIdx.x; c < a.n_pos; c += 1024) cnt += ((best - a.scores[c]) + 1.0f >= 0.0f) ? 1.0f : 0.0f;
    sv[threadIdx.x] = cnt;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) sv[threadIdx.x] += sv[threadIdx.x + w];   // integers: exact in any order
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        float *ex = a.scores + end;
        ex[0] = best;
        ex[1] = __int_as_float((int)bi);
        ex[2] = sv[0];
    }
}

// run_val_iteration's loss (implicit.py:366-379) from the exchanged score vector: every
// rank holds every score, so each computes the whole loss (one workgroup, fixed order,
// double accumulators) -- identical on every rank
__global__ __launch_bounds__(1024) void owner_loss_kernel(OwnerArgs a, double inv_a, double inv_b, float *out) {
    __shared__ double red[2][1024 / kWave];
    const int64_t gc = a.gc;
    const int n = a.n_neg;
    const bool pairwise = a.loss == RG_LOSS_BPR || a.loss == RG_LOSS_HINGE;
    double sa = 0.0, sb = 0.0;
    float mx = 0.0f;
    if (a.loss == RG_LOSS_ADAPTIVE_HINGE) {
        __shared__ float sv[1024];
        __shared__ int64_t si[1024];
        float best = -1.0f;
        int64_t bi = INT64_MAX;
        for (int64_t g = gc + threadIdx.x; g < (int64_t)(1 + n) * gc; g += 1024)
            if (a.scores[g] > best) { best = a.scores[g]; bi = g; }
        block_max_first(best, bi, sv, si);
        mx = best;
    }
    for (int64_t c = threadIdx.x; c < gc; c += 1024) {
        const bool has = c < a.n_pos;
        const float p0 = a.scores[c];
        if (a.loss == RG_LOSS_ADAPTIVE_HINGE) {
            if (has) sa += (double)fmaxf((mx - p0) + 1.0f, 0.0f);
        } else if (pairwise) {
            if (!has) continue;
            for (int k = 0; k < n; ++k) {
                const float pk = a.scores[(1 + k) * gc + c];
                if (a.loss == RG_LOSS_BPR) sa += (double)(1.0f - sigmoidf_ref(p0 - pk));
                else sa += (double)fmaxf((pk - p0) + 1.0f, 0.0f);
            }
        } else {
            if (has) sa += (double)(-fmaxf(logf(p0), -100.0f));
            for (int k = 0; k < n; ++k) sb += (double)(-fmaxf(logf(1.0f - a.scores[(1 + k) * gc + c]), -100.0f));
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        sa += __shfl_xor(sa, off);
        sb += __shfl_xor(sb, off);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & (kWave - 1)) == 0) { red[0][w] = sa; red[1][w] = sb; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double ta = 0.0, tb = 0.0;
        for (int k = 0; k < 1024 / kWave; ++k) { ta += red[0][k]; tb += red[1][k]; }
        *out = (float)(ta * inv_a + tb * inv_b);
    }
}

struct UpbF {
    int *upb;
    template <class L>
    int operator()() { *upb = kBlk / L::LPU; return 0; }
};

int upb_of(int dim) {
    int u = 0;
    UpbF f{&u};
    return dispatch_dim(dim, f) == 0 ? u : -1;
}

int64_t segs_of(int64_t gc, int n) { return ((int64_t)n * gc + kOwnSeg - 1) / kOwnSeg; }

int npass_of(int world, int upb) {
    const int p = (kOwnSeg + world * upb - 1) / (world * upb);
    return p < 1 ? 1 : p;
}

struct OwnLaunchF {
    OwnerArgs *a;
    OwnTables t;
    OwnWork w;
    bool back;
    hipStream_t s;
    template <class L>
    int operator()() {
        constexpr int UPB = kBlk / L::LPU;
        const int64_t pos_blocks = (a->n_planned + UPB - 1) / UPB;
        const int npass = npass_of(a->world, UPB);
        const int64_t grid = pos_blocks + a->segs * npass;
        if (grid <= 0) return RG_OK;
        if (!back) {
            hipLaunchKernelGGL((owner_scores_kernel<L>), dim3((unsigned)grid), dim3(kBlk), 0, s, *a, t, pos_blocks,
                               npass);
        } else if (a->n_neg <= 5) {
            hipLaunchKernelGGL((owner_back_kernel<L, 5>), dim3((unsigned)grid), dim3(kBlk), 0, s, *a, t, w,
                               pos_blocks, npass);
        } else {
            hipLaunchKernelGGL((owner_back_kernel<L, RG_MF_MAX_NEG>), dim3((unsigned)grid), dim3(kBlk), 0, s, *a, t,
                               w, pos_blocks, npass);
        }
        return check_launch(back ? "rg_mf_owner_back" : "rg_mf_owner_scores");
    }
};

OwnTables own_tables(const rg_mf_tables_t *t) {
    OwnTables o{};
    o.user_w = t->user_w; o.item_w = t->item_w; o.user_b = t->user_b; o.item_b = t->item_b;
    o.num_users = t->num_users; o.dim = t->dim;
    return o;
}

}  // namespace

int owner_args(const rg_mf_owner_batch_t *b, OwnerArgs &a) {
    if (!b) return fail_arg("rg_mf_owner: null batch");
    if (b->n_neg < 1 || b->n_neg > RG_MF_MAX_NEG) return fail_arg("rg_mf_owner: n_neg must be in [1, 8]");
    if (b->world < 1 || b->rank < 0 || b->rank >= b->world) return fail_arg("rg_mf_owner: bad rank / world");
    if (b->global_cols <= 0 || (int64_t)(1 + b->n_neg) * b->global_cols >= ((int64_t)1 << 31))
        return fail_arg("rg_mf_owner: bad global_cols");
    if (b->n_pos < 0 || b->n_pos > b->global_cols) return fail_arg("rg_mf_owner: bad n_pos");
    if (b->n_planned < 0 || b->n_planned > b->n_pos) return fail_arg("rg_mf_owner: bad n_planned");
    if (b->n_planned > 0 && (!b->plan_perm || !b->plan_pos_slot || !b->pos_user || !b->pos_item))
        return fail_arg("rg_mf_owner: null positives / plan");
    if (b->loss < 0 || b->loss > RG_LOSS_ADAPTIVE_HINGE) return fail_arg("rg_mf_owner: bad loss kind");
    if (b->loss != RG_LOSS_POINTWISE && b->n_pos <= 0) return fail_arg("rg_mf_owner: empty global batch");
    if (!b->words || !b->pool || b->pool_len <= 0) return fail_arg("rg_mf_owner: no words / empty pool");
    if (!b->neg_rec || !b->seg_count || !b->scores) return fail_arg("rg_mf_owner: null records / counts / scores");
    a = OwnerArgs{};
    a.pos_user = b->pos_user; a.pos_item = b->pos_item; a.n_pos = b->n_pos; a.gc = b->global_cols;
    a.perm = b->plan_perm; a.pos_slot = b->plan_pos_slot; a.n_planned = b->n_planned;
    a.words = reinterpret_cast<const uint2 *>(b->words);
    a.pool = reinterpret_cast<const int2 *>(b->pool);
    a.pool_len = b->pool_len; a.n_neg = b->n_neg; a.loss = b->loss; a.world = b->world; a.rank = b->rank;
    a.rec = reinterpret_cast<int4 *>(b->neg_rec);
    a.seg_count = b->seg_count;
    a.scores = b->scores;
    a.segs = segs_of(b->global_cols, b->n_neg);
    if (b->claim_count) {
        if (b->loss == RG_LOSS_ADAPTIVE_HINGE)
            return fail_arg("rg_mf_owner: no claimed slots for the adaptive hinge (only the max negative is listed)");
        if (b->claim_num_users <= 0) return fail_arg("rg_mf_owner: claimed slots need claim_num_users");
        a.claim = b->claim_count;
        a.claim_users = b->claim_num_users;
    }
    // mean denominators as the pair pass: BCE means over B and n*B, bpr / hinge over n*B
    if (b->loss == RG_LOSS_POINTWISE) {
        a.n_a = (float)(b->n_pos > 0 ? b->n_pos : 1);
        a.n_b = (float)((int64_t)b->n_neg * b->global_cols);
    } else if (b->loss == RG_LOSS_ADAPTIVE_HINGE) {
        a.n_a = (float)b->n_pos;
        a.n_b = 1.0f;
    } else {
        a.n_a = (float)((int64_t)b->n_neg * b->n_pos);
        a.n_b = 1.0f;
    }
    return RG_OK;
}

}  // namespace rg

using namespace rg;

extern "C" int64_t rg_mf_owner_segments(int64_t global_cols, int32_t n_neg) {
    if (global_cols <= 0 || n_neg < 1) return -1;
    return segs_of(global_cols, n_neg);
}

extern "C" int64_t rg_mf_owner_rec_len(int64_t global_cols, int32_t n_neg) {
    if (global_cols <= 0 || n_neg < 1) return -1;
    return segs_of(global_cols, n_neg) * kOwnSeg;
}

extern "C" int64_t rg_mf_owner_partials_used(int64_t global_cols, int32_t n_neg, int32_t dim, int32_t world,
                                             int64_t n_planned) {
    const int upb = upb_of(dim);
    if (upb <= 0 || global_cols <= 0 || n_neg < 1 || world < 1 || n_planned < 0) return -1;
    return 2 * ((n_planned + upb - 1) / upb + segs_of(global_cols, n_neg) * npass_of(world, upb));
}

extern "C" int64_t rg_mf_owner_partials_len(int64_t global_cols, int32_t n_neg, int32_t dim, int32_t world) {
    return rg_mf_owner_partials_used(global_cols, n_neg, dim, world, global_cols);
}

extern "C" int rg_mf_owner_prepare(void *stream, const rg_mf_owner_batch_t *b) {
    OwnerArgs a;
    int rc = owner_args(b, a);
    if (rc) return rc;
    hipLaunchKernelGGL(owner_prepare_kernel, dim3((unsigned)a.segs), dim3(kBlk), 0, (hipStream_t)stream, a);
    return check_launch("rg_mf_owner_prepare");
}

extern "C" int rg_mf_owner_loss(void *stream, const rg_mf_owner_batch_t *b, float *loss_out) {
    OwnerArgs a;
    int rc = owner_args(b, a);
    if (rc) return rc;
    if (!loss_out) return fail_arg("rg_mf_owner_loss: null output");
    const double gp = (double)(b->n_pos > 0 ? b->n_pos : 1), n = (double)b->n_neg;
    const double inv_a = (b->loss == RG_LOSS_POINTWISE || b->loss == RG_LOSS_ADAPTIVE_HINGE) ? 1.0 / gp : 1.0 / (n * gp);
    const double inv_b = b->loss == RG_LOSS_POINTWISE ? 1.0 / (n * (double)b->global_cols) : 0.0;
    hipLaunchKernelGGL(owner_loss_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, a, inv_a, inv_b, loss_out);
    return check_launch("rg_mf_owner_loss");
}

extern "C" int rg_mf_owner_adapt(void *stream, const rg_mf_owner_batch_t *b) {
    OwnerArgs a;
    int rc = owner_args(b, a);
    if (rc) return rc;
    if (b->loss != RG_LOSS_ADAPTIVE_HINGE) return fail_arg("rg_mf_owner_adapt: adaptive hinge only");
    hipLaunchKernelGGL(owner_adapt_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, a);
    return check_launch("rg_mf_owner_adapt");
}

extern "C" int rg_mf_owner_scores(void *stream, const rg_mf_tables_t *t, const rg_mf_owner_batch_t *b) {
    OwnerArgs a;
    int rc = owner_args(b, a);
    if (rc) return rc;
    if (!t || !t->user_w || !t->item_w || !t->user_b || !t->item_b) return fail_arg("rg_mf_owner_scores: null tables");
    OwnLaunchF f{&a, own_tables(t), OwnWork{}, false, (hipStream_t)stream};
    return dispatch_dim(t->dim, f);
}

extern "C" int rg_mf_owner_back(void *stream, const rg_mf_tables_t *t, const rg_mf_owner_batch_t *b,
                                rg_mf_work_t *w) {
    OwnerArgs a;
    int rc = owner_args(b, a);
    if (rc) return rc;
    if (!t || !t->user_w || !t->item_w) return fail_arg("rg_mf_owner_back: null tables");
    if (!w || !w->row_count || !w->row_list || !w->hot_grad || !w->hot_bias_grad || !w->loss_partials)
        return fail_arg("rg_mf_owner_back: null scratch");
    if (a.n_planned > 0 && (!w->part_row || !w->part_bias || !w->plan_item_slot_off))
        return fail_arg("rg_mf_owner_back: planned positives need part_row / part_bias / plan_item_slot_off");
    if (a.claim && (a.claim != w->row_count || a.claim_users != t->num_users))
        return fail_arg("rg_mf_owner_back: claimed slots need the claim array as row_count and claim_num_users == "
                        "num_users");
    OwnWork ow{};
    ow.row_count = w->row_count;
    ow.row_list = reinterpret_cast<int2 *>(w->row_list);
    ow.hot_grad = reinterpret_cast<long long *>(w->hot_grad);
    ow.hot_bias = reinterpret_cast<long long *>(w->hot_bias_grad);
    ow.partials = w->loss_partials;
    ow.part_row = w->part_row; ow.part_bias = w->part_bias;
    OwnLaunchF f{&a, own_tables(t), ow, true, (hipStream_t)stream};
    return dispatch_dim(t->dim, f);
}
