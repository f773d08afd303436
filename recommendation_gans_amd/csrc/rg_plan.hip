// Item-sorted per-batch plans for the MF / NCF step (rg_hip.h rg_mf_work_t plan_*), built
// on the device for every batch of a fit in ONE launch (one workgroup per batch).
//
// The reference shuffles the training set once per fit (implicit.py:262, torch_utils.py
// shuffle) and then cuts it into the same contiguous batches every epoch (minibatch,
// implicit.py:290), so a batch's plan is loop-invariant: it is built once per fit.
//
// Per batch (1024 threads):
//   1. the batch's positives (those whose user this rank owns, owner-sharded DP) are
//      compacted in column order into 64-bit keys (item << 32 | column): block scan of
//      per-thread counts;
//   2. bitonic sort of the keys (LDS when they fit, 128 KB; else device scratch): the
//      order is (item, column), i.e. a stable sort by item;
//   3. partial slots: a new slot starts where the item changes or a pair-kernel block of
//      units_per_block positions begins (block scan of the head flags) -> perm, pos_slot,
//      and the item of every slot;
//   4. item_slot_off[i] = first slot whose item is >= i (binary search per item).
#include "rg_common.h"

namespace rg {
namespace {

constexpr int kPT = 1024;               // threads per plan workgroup
constexpr int kPW = kPT / kWave;        // waves
constexpr int kLdsKeys = 16384;         // keys sorted in LDS (128 KB)
constexpr int kChunk = kLdsKeys / kPT;  // positions per thread per round of step 3

struct PlanArgs {
    const int64_t *users, *items;
    int64_t n, offset, stride, batch_len, cols, num_items;
    int32_t upb, world, rank, pad_;
    int32_t *perm, *pos_slot, *item_slot_off, *counts;
    uint64_t *scratch;                  // per batch: scratch_stride uint64
    int64_t scratch_stride;
};

__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int t = __shfl_up(v, o);
        if (lane >= o) v += t;
    }
    return v;
}

// exclusive block scan of one int per thread; *total = the block's sum (every thread)
__device__ __forceinline__ int block_excl_scan(int v, int *sh, int *total) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & (kWave - 1);
    const int inc = wave_incl_scan(v);
    __syncthreads();                    // sh may still be read by a previous scan
    if (lane == kWave - 1) sh[w] = inc;
    __syncthreads();
    int before = 0, all = 0;
#pragma unroll
    for (int k = 0; k < kPW; ++k) {
        const int x = sh[k];
        before += k < w ? x : 0;
        all += x;
    }
    *total = all;
    return before + inc - v;
}

__device__ __forceinline__ bool owned(const PlanArgs &a, int64_t g) {
    return a.world <= 1 || (int32_t)(a.users[g] % a.world) == a.rank;
}

template <bool kLds>
__device__ void plan_body(const PlanArgs &a, int64_t k, int64_t lo, int64_t m, int n_own, uint64_t *lds_keys,
                          int *sh) {
    const int tid = threadIdx.x;
    uint64_t *keys = kLds ? lds_keys : a.scratch + k * a.scratch_stride;
    int P = 1;
    while (P < n_own) P <<= 1;
    int *segitem = kLds ? reinterpret_cast<int *>(lds_keys) : reinterpret_cast<int *>(keys + P);

    // ---- 1. compact the planned positives in column order -------------------------
    {
        const int64_t C = (m + kPT - 1) / kPT;
        const int64_t j0 = tid * C, j1 = j0 + C < m ? j0 + C : m;
        int c = 0;
        for (int64_t j = j0; j < j1; ++j) c += owned(a, lo + j) ? 1 : 0;
        int tot;
        int pos = block_excl_scan(c, sh, &tot);
        for (int64_t j = j0; j < j1; ++j) {
            if (!owned(a, lo + j)) continue;
            keys[pos++] = ((uint64_t)(uint32_t)a.items[lo + j] << 32) | (uint64_t)(uint32_t)j;
        }
        for (int s = n_own + tid; s < P; s += kPT) keys[s] = ~0ull;
    }
    __syncthreads();

    // ---- 2. bitonic sort (keys are unique: the column breaks item ties) ---------------
    for (int kk = 2; kk <= P; kk <<= 1) {
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int t = tid; t < (P >> 1); t += kPT) {
                const int i = 2 * j * (t / j) + (t % j), l = i + j;
                const uint64_t x = keys[i], y = keys[l];
                const bool up = (i & kk) == 0;
                if ((x > y) == up) { keys[i] = y; keys[l] = x; }
            }
            __syncthreads();
        }
    }

    // ---- 3. slots, perm, pos_slot (rounds of kLdsKeys positions) --------------------
    int32_t *perm = a.perm + k * a.cols, *pslot = a.pos_slot + k * a.cols;
    int carry = 0;
    for (int base = 0; base < n_own; base += kLdsKeys) {
        int it[kChunk], col[kChunk];
        int prev_item = -1;
        const int s0 = base + tid * kChunk;
        int heads = 0;
#pragma unroll
        for (int e = 0; e < kChunk; ++e) {
            const int s = s0 + e;
            it[e] = -1;
            col[e] = 0;
            if (s < n_own) {
                const uint64_t x = keys[s];
                it[e] = (int)(x >> 32);
                col[e] = (int)(uint32_t)x;
            }
        }
        if (s0 > 0 && s0 < n_own) prev_item = (int)(keys[s0 - 1] >> 32);
        int pi = prev_item;
#pragma unroll
        for (int e = 0; e < kChunk; ++e) {
            const int s = s0 + e;
            if (s < n_own) {
                const bool head = s == 0 || it[e] != pi || (s % a.upb) == 0;
                heads += head ? 1 : 0;
                pi = it[e];
            }
        }
        int tot;
        int slot = carry + block_excl_scan(heads, sh, &tot) - 1;   // the scan's barriers end the key reads
        pi = prev_item;
#pragma unroll
        for (int e = 0; e < kChunk; ++e) {
            const int s = s0 + e;
            if (s < n_own) {
                const bool head = s == 0 || it[e] != pi || (s % a.upb) == 0;
                if (head) {
                    ++slot;
                    segitem[slot] = it[e];
                }
                perm[s] = col[e];
                pslot[s] = slot;
                pi = it[e];
            }
        }
        carry += tot;
        __syncthreads();
    }
    const int nslots = carry;
    // the remaining positions: the batch's other columns (single rank), else -1
    for (int64_t s = n_own + tid; s < a.cols; s += kPT) {
        perm[s] = a.world <= 1 ? (int32_t)s : -1;
        pslot[s] = -1;
    }
    __syncthreads();

    // ---- 4. item -> first slot ------------------------------------------------------
    int32_t *off = a.item_slot_off + k * (a.num_items + 1);
    for (int64_t i = tid; i <= a.num_items; i += kPT) {
        int lo_ = 0, hi = nslots;
        while (lo_ < hi) {
            const int mid = (lo_ + hi) >> 1;
            if ((int64_t)segitem[mid] < i) lo_ = mid + 1; else hi = mid;
        }
        off[i] = lo_;
    }
    if (tid == 0) {
        a.counts[2 * k] = n_own;
        a.counts[2 * k + 1] = nslots;
    }
}

__global__ __launch_bounds__(kPT) void plan_kernel(PlanArgs a) {
    __shared__ uint64_t lds_keys[kLdsKeys];
    __shared__ int sh[kPW];
    const int64_t k = blockIdx.x;
    const int64_t lo = a.offset + k * a.stride;
    int64_t m = lo < a.n ? a.n - lo : 0;
    if (m > a.batch_len) m = a.batch_len;
    // planned positives of this batch (block-uniform)
    int n_own;
    {
        const int64_t C = (m + kPT - 1) / kPT;
        const int64_t j0 = threadIdx.x * C, j1 = j0 + C < m ? j0 + C : m;
        int c = 0;
        for (int64_t j = j0; j < j1; ++j) c += owned(a, lo + j) ? 1 : 0;
        block_excl_scan(c, sh, &n_own);
    }
    if (n_own <= kLdsKeys) {
        plan_body<true>(a, k, lo, m, n_own, lds_keys, sh);
    } else if (a.scratch == nullptr) {   // owner filter without scratch: refused per batch (host retries)
        if (threadIdx.x == 0) {
            a.counts[2 * k] = -1;
            a.counts[2 * k + 1] = -1;
        }
    } else {
        plan_body<false>(a, k, lo, m, n_own, lds_keys, sh);
    }
}

}  // namespace
}  // namespace rg

using namespace rg;

extern "C" int64_t rg_mf_plans_scratch_len(int64_t cols, int64_t n_batches) {
    if (cols <= 0 || n_batches < 0) return -1;
    if (cols <= kLdsKeys) return 0;
    int64_t P = 1;
    while (P < cols) P <<= 1;
    return n_batches * (P + (cols + 1) / 2 + 1);
}

extern "C" int rg_mf_plans_build(void *stream, const int64_t *users, const int64_t *items, int64_t n, int64_t offset,
                                 int64_t stride, int64_t batch_len, int64_t n_batches, int64_t cols,
                                 int32_t units_per_block, int64_t num_items, int32_t owner_world, int32_t owner_rank,
                                 int32_t *perm, int32_t *pos_slot, int32_t *item_slot_off, int32_t *counts,
                                 uint64_t *scratch) {
    if (n_batches == 0) return RG_OK;
    if ((!items && n > 0) || !perm || !pos_slot || !item_slot_off || !counts) return fail_arg("rg_mf_plans_build: null pointer");
    if (n < 0 || offset < 0 || stride <= 0 || batch_len <= 0 || n_batches < 0 || units_per_block <= 0)
        return fail_arg("rg_mf_plans_build: bad batch layout");
    if (num_items <= 0 || num_items >= ((int64_t)1 << 31)) return fail_arg("rg_mf_plans_build: bad num_items");
    if (owner_world < 1 || owner_rank < 0 || owner_rank >= owner_world || (owner_world > 1 && !users))
        return fail_arg("rg_mf_plans_build: bad owner rank / world (users required when world > 1)");
    if (batch_len > cols) return fail_arg("rg_mf_plans_build: batch_len > cols (the output stride)");
    if (cols >= ((int64_t)1 << 31)) return fail_arg("rg_mf_plans_build: cols too large");
    const int64_t need = rg_mf_plans_scratch_len(cols, n_batches);
    // owner filter (world > 1): a rank plans ~cols / world positives per batch, almost always
    // within the LDS path, so scratch may be omitted; a batch that needs it then reports
    // counts = -1 and the caller rebuilds with scratch
    if (need > 0 && !scratch && owner_world <= 1)
        return fail_arg("rg_mf_plans_build: batches over 16384 planned positives need scratch");
    PlanArgs a{};
    a.users = users; a.items = items; a.n = n; a.offset = offset; a.stride = stride; a.batch_len = batch_len;
    a.cols = cols; a.num_items = num_items; a.upb = units_per_block; a.world = owner_world; a.rank = owner_rank;
    a.perm = perm; a.pos_slot = pos_slot; a.item_slot_off = item_slot_off; a.counts = counts;
    a.scratch = scratch;
    a.scratch_stride = n_batches > 0 && need > 0 && scratch ? need / n_batches : 0;
    hipLaunchKernelGGL(plan_kernel, dim3((unsigned)n_batches), dim3(kPT), 0, (hipStream_t)stream, a);
    return check_launch("rg_mf_plans_build");
}
