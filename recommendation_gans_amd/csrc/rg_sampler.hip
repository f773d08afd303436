// MT19937 word stream of CPython's `random` module on the GPU.
//
// Replaces the host-side `random.choices(pool, k=n*batch_size)` draw of
// implicit.py:352 (66 % of the reference's CPU step).  The state is
// exactly CPython's getstate()[1]: 624 words + the position of the next word.
//
// Seen as one infinite word stream x[] whose first 624 words are the state
// block, CPython's in-place block twist is the recurrence
//     x[n] = x[n-227] ^ mix(x[n-624], x[n-623]),   mix(a,b) = twist(a_hi | b_lo)
// so ONE workgroup produces 227 consecutive words per round ("chunk", lane p owns
// position p of every chunk).  x[n-227] is the same lane's previous output (kept
// in a register); x[n-624] / x[n-623] lie two or three chunks back in an LDS
// ring, written by other lanes, so a barrier is needed only every second round
// (and both rounds' LDS reads are issued together right after it).
// Raw (untempered) words are stored coalesced -- the consumer tempers them; the state
// written back is the 624-word block holding the last emitted word (CPython
// twists lazily, so position 624 means "block exhausted").
#include <cstdlib>

#include "rg_mt.h"

namespace rg {

__global__ __launch_bounds__(kGenThreads) void mt_generate_kernel(uint32_t *__restrict__ state,
                                                                  uint32_t *__restrict__ out,
                                                                  int64_t nwords,
                                                                  uint32_t *__restrict__ state_before, int prio) {
    __shared__ uint32_t X[kRing + 2];
    if (prio) __builtin_amdgcn_s_setprio(3);
    mt_generate_block(X, state, out, nwords, state_before);
}

// ---------------------------------------------------------------- jump-ahead path
// One step's words as head + jump + parallel tail segments (rg_mtjump.cpp has the
// algebra): the head walks the first H >= 19,937 + 623 words sequentially; the
// jump kernel XORs windows of them into the window-form states where the tail
// segments (and the next step) start; the tail segments are walked concurrently.

// head: state_before copy, zero the jump accumulators, walk H words
template <bool BOUNDED>
__global__ __launch_bounds__(kGenThreads) void mt_head_kernel(const uint32_t *__restrict__ state,
                                                              uint32_t *__restrict__ out, int64_t H,
                                                              uint32_t *__restrict__ state_before,
                                                              uint32_t *__restrict__ raw, int nraw) {
    __shared__ uint32_t X[kRing + 2];
    const int p = threadIdx.x;
    mt_load(X, p, state);
    const int64_t pos0 = (int64_t)state[kMtN];
    if (state_before != nullptr)
        for (int i = p; i <= kMtN; i += kGenThreads) state_before[i] = state[i];
    for (int i = p; i < nraw; i += kGenThreads) raw[i] = 0U;
    __syncthreads();
    mt_walk<BOUNDED>(X, p, pos0, H, out);
}

// the other ranks' slices of `units` units ([R][L] words each), hashed (local stand-in of the
// owner step's word all-gather: the words are random, the draws they make are not the stream's)
__global__ __launch_bounds__(256) void mt_fill_slices_kernel(uint32_t *__restrict__ words, int64_t units, int64_t W,
                                                             int64_t L, int rank, uint32_t seed) {
    const int64_t n = units * W;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        if ((i % W) / L == rank) continue;
        uint32_t h = (uint32_t)i * 0x9E3779B1u ^ seed;
        h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
        words[i] = h;
    }
}

int mt_fill_other_slices(hipStream_t stream, uint32_t *words, int64_t units, int64_t W, int64_t L, int rank,
                         int world, uint32_t seed) {
    if (!words || units < 0 || L <= 0 || W != L * world) return fail_arg("mt_fill_other_slices: bad geometry");
    hipLaunchKernelGGL(mt_fill_slices_kernel, dim3(1024), dim3(256), 0, stream, words, units, W, L, rank, seed);
    return check_launch("mt_fill_other_slices");
}

// raw[j][k] ^= XOR over this block's share of jump j's terms i of x[i + k].
// The stream words x[0 .. nx) (80 KB) and the block's term indices are staged in
// LDS, so the XOR loop is LDS-only (broadcast term read + three conflict-free
// word reads per term) and unrolled to keep several reads in flight.
constexpr int kJumpMaxTerms = 1024;   // per block (chunks chosen on the host to fit)
__global__ __launch_bounds__(kGenThreads) void mt_jump_kernel(const uint32_t *__restrict__ x, int nx,
                                                              const int32_t *__restrict__ terms,
                                                              const int32_t *__restrict__ term_off,
                                                              uint32_t *__restrict__ raw) {
    extern __shared__ uint32_t sx[];                 // [nx] stream words
    __shared__ int32_t st[kJumpMaxTerms];
    const int j = blockIdx.y, c = blockIdx.x, chunks = gridDim.x;
    const int t0 = term_off[j], t1 = term_off[j + 1];
    const int per = (t1 - t0 + chunks - 1) / chunks;
    const int a = t0 + c * per, b = min(t1, a + per);
    const int nt = b > a ? b - a : 0;
    const int k0 = threadIdx.x;
    for (int i = k0; i < (nx >> 2); i += kGenThreads)
        reinterpret_cast<uint4 *>(sx)[i] = reinterpret_cast<const uint4 *>(x)[i];
    for (int i = (nx & ~3) + k0; i < nx; i += kGenThreads) sx[i] = x[i];
    for (int i = k0; i < nt; i += kGenThreads) st[i] = terms[a + i];
    __syncthreads();
    if (nt == 0) return;
    const bool third = k0 + 2 * kGenThreads < kMtN;
    uint32_t acc0 = 0U, acc1 = 0U, acc2 = 0U;       // words k0, k0 + 256, k0 + 512
    int t = 0;
    for (; t + 4 <= nt; t += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t *w = sx + st[t + u] + k0;
            acc0 ^= w[0];
            acc1 ^= w[kGenThreads];
            if (third) acc2 ^= w[2 * kGenThreads];
        }
    }
    for (; t < nt; ++t) {
        const uint32_t *w = sx + st[t] + k0;
        acc0 ^= w[0];
        acc1 ^= w[kGenThreads];
        if (third) acc2 ^= w[2 * kGenThreads];
    }
    uint32_t *r = raw + (int64_t)j * kMtN;
    atomicXor(r + k0, acc0);
    atomicXor(r + k0 + kGenThreads, acc1);
    if (third) atomicXor(r + k0 + 2 * kGenThreads, acc2);
}

// window-form state x[D .. D+624) from the XOR of windows with exponent D - 1
__device__ __forceinline__ uint32_t mt_fixup(const uint32_t *r, int i) {
    return i < kMtN - 1 ? r[i + 1] : r[kMtM] ^ mt_mix(r[0], r[1]);
}

// blocks 0..n-1: tail segment j from window state raw[j]; block n: next step's state
__global__ __launch_bounds__(kGenThreads) void mt_tail_kernel(const uint32_t *__restrict__ raw,
                                                              MtTailSegs segs, uint32_t *__restrict__ out,
                                                              uint32_t *__restrict__ state) {
    __shared__ uint32_t X[kRing + 2];
    const int p = threadIdx.x, j = blockIdx.x;
    const uint32_t *r = raw + (int64_t)j * kMtN;
    if (j == segs.n) {
        for (int i = p; i < kMtN; i += kGenThreads) state[i] = mt_fixup(r, i);
        if (p == 0) state[kMtN] = kMtN;
        return;
    }
    for (int i = p; i < kMtN; i += kGenThreads) X[i] = mt_fixup(r, i);
    if (p == 0) X[kRing] = mt_fixup(r, 0);
    __syncthreads();
    mt_walk<true>(X, p, kMtN, segs.len[j], out + segs.start[j]);
}

int mt_produce_jump(hipStream_t stream, const MtJumpPlan &plan, uint32_t *state, uint32_t *out,
                    uint32_t *state_before, int64_t walk) {
    const int nslots = plan.segs.n + 1;
    if (walk > 0) {
        if (plan.segs.n != 0 || walk < plan.head) return fail_arg("mt_produce_jump: a slice walk needs a jump-only plan");
        hipLaunchKernelGGL(mt_head_kernel<true>, dim3(1), dim3(kGenThreads), 0, stream, state, out, walk, state_before,
                           plan.raw, nslots * kMtN);
    } else {
        hipLaunchKernelGGL(mt_head_kernel<false>, dim3(1), dim3(kGenThreads), 0, stream, state, out, plan.head,
                           state_before, plan.raw, nslots * kMtN);
    }
    const int nx = (int)plan.head;
    const size_t lds = (size_t)nx * sizeof(uint32_t);
    static const bool attr = [&] {
        return hipFuncSetAttribute(reinterpret_cast<const void *>(mt_jump_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
    }();
    if (!attr) return fail_arg("mt_jump_kernel: cannot reserve LDS for the stream window");
    hipLaunchKernelGGL(mt_jump_kernel, dim3(plan.chunks, nslots), dim3(kGenThreads), lds, stream, out, nx,
                       plan.terms, plan.term_off, plan.raw);
    hipLaunchKernelGGL(mt_tail_kernel, dim3(nslots), dim3(kGenThreads), 0, stream, plan.raw, plan.segs, out, state);
    return check_launch("mt_produce_jump");
}

}  // namespace rg

extern "C" int rg_mt_generate(void *stream, uint32_t *state_dev, uint32_t *out_words_dev, int64_t nwords,
                              uint32_t *state_before_dev) {
    if (state_dev == nullptr) return rg::fail_arg("rg_mt_generate: null state");
    if (nwords < 0) return rg::fail_arg("rg_mt_generate: nwords < 0");
    if (nwords > 0 && out_words_dev == nullptr) return rg::fail_arg("rg_mt_generate: null output");
#if RG_AB
    static const int prio = [] { const char *e = getenv("RG_MT_PRIO"); return e ? atoi(e) : 0; }();
#else
    constexpr int prio = 0;
#endif
    hipLaunchKernelGGL(rg::mt_generate_kernel, dim3(1), dim3(rg::kGenThreads), 0, (hipStream_t)stream,
                       state_dev, out_words_dev, nwords, state_before_dev, prio);
    return rg::check_launch("rg_mt_generate");
}
