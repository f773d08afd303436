// Owner-sharded data-parallel MF step (dp_mode 2): device pieces shared by rg_owner.hip
// (the score / backward passes) and rg_mf.hip (the dense pass that runs the NEXT step's
// owner prepare in extra workgroups).
//
// Rank r of R owns the users u with u % R == r (local row u / R: embedding, bias,
// optimizer state) and holds every item.  Every rank walks the ONE global CPython
// stream of the step (n * GC draws, GC = B * R global columns, implicit.py:351-354) and
// keeps the pairs whose user it owns: draw j of negative slot k = j / GC, column
// c = j % GC, is pair gp = (1 + k) * GC + c of the global step (gp = c: the positive).
#pragma once
#include "rg_common.h"

namespace rg {

constexpr int kOwnSeg = 256;   // draws per prepare workgroup = record segment capacity

struct OwnerArgs {
    const int64_t *pos_user, *pos_item;   // the global batch (global ids)
    int64_t n_pos, gc;
    const int32_t *perm, *pos_slot;       // this rank's planned positives
    int64_t n_planned;
    const uint2 *words;
    const int2 *pool;
    int64_t pool_len;
    int32_t n_neg, loss, world, rank;
    int4 *rec;                            // [segs * kOwnSeg] {gp, local user, item, 0}
    int32_t *seg_count;                   // [segs]
    float *scores;                        // [(1 + n) * gc]
    int64_t segs;
    float n_a, n_b;                       // loss mean denominators (global batch)
    // claimed list slots (rg_mf_owner_batch_t claim_count): the prepare claims both row sides of
    // every kept draw and stores them in rec.w (user slot | item slot << 8, each min(slot, cap))
    int32_t *claim;
    int64_t claim_users;
};

// One prepare workgroup: draws [b * kOwnSeg, (b + 1) * kOwnSeg) -> pool pairs (CPython
// random.choices arithmetic, choice_index) -> the ones this rank owns, compacted in draw
// order (wave ballots: deterministic), plus this workgroup's share of zeroing the score
// buffer the exchange sums.  Pairwise losses drop the draws of columns without a positive
// (they pair with nothing, spotlight/losses.py neg.view(n, B)[:, :Bp]).
__device__ __forceinline__ void owner_prepare_block(const OwnerArgs &a, int64_t b) {
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid >> 6;
    const int64_t j = b * kOwnSeg + tid;
    const int64_t total = (int64_t)a.n_neg * a.gc;
    const bool pairwise = a.loss == RG_LOSS_BPR || a.loss == RG_LOSS_HINGE;
    bool own = false;
    int4 r = make_int4(0, 0, 0, 0);
    if (j < total) {
        const int64_t k = j / a.gc, c = j - k * a.gc;
        if (!pairwise || c < a.n_pos) {
            const uint2 wd = a.words[j];
            const int2 pr = a.pool[choice_index(wd.x, wd.y, a.pool_len)];
            own = (pr.x % a.world) == a.rank;
            r = make_int4((int)((1 + k) * a.gc + c), pr.x / a.world, pr.y, 0);
            if (own && a.claim != nullptr) {
                const int su = atomicAdd(a.claim + r.y, 1);
                const int si = atomicAdd(a.claim + a.claim_users + r.z, 1);
                r.w = (su < RG_MF_LIST_CAP ? su : RG_MF_LIST_CAP) | ((si < RG_MF_LIST_CAP ? si : RG_MF_LIST_CAP) << 8);
            }
        }
    }
    __shared__ int wcount[kOwnSeg / kWave];
    const uint64_t m = __ballot(own);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wcount[w] = __popcll(m);
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int q = 0; q < kOwnSeg / kWave; ++q) {
        base += q < w ? wcount[q] : 0;
        tot += wcount[q];
    }
    if (own) a.rec[b * kOwnSeg + base + before] = r;
    if (tid == 0) a.seg_count[b] = tot;
    const int64_t len = (int64_t)(1 + a.n_neg) * a.gc;
    const int64_t z = (len + a.segs - 1) / a.segs;
    const int64_t z1 = (b + 1) * z < len ? (b + 1) * z : len;
    for (int64_t i = b * z + tid; i < z1; i += kOwnSeg) a.scores[i] = 0.0f;
}

// adaptive hinge: the score buffer's extra slots after the exchanged (1 + n) * GC scores
__device__ __forceinline__ int64_t adapt_slot(const OwnerArgs &a) { return (int64_t)(1 + a.n_neg) * a.gc; }

// host: validated device view of a batch (rg_owner.hip)
int owner_args(const rg_mf_owner_batch_t *b, OwnerArgs &a);
// rg_mf_apply_prepare with the NEXT step's owner prepare in the extra workgroups (rg_mf.hip)
int apply_prepare_owner(void *stream, const rg_mf_tables_t *t, rg_mf_work_t *w, const rg_opt_t *opt,
                        int64_t row_begin, int64_t row_end, const rg_mf_loss_t *loss,
                        const rg_mf_owner_batch_t *next);

}  // namespace rg
