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
#include "rg_common.h"

namespace rg {

constexpr int kMtN = 624;
constexpr int kMtM = 397;
constexpr int kChunk = kMtN - kMtM;     // 227
constexpr int kRing = 2048;             // words of stream kept in LDS (power of two)
constexpr uint32_t kMatrixA = 0x9908b0dfU;
constexpr int kGenThreads = 256;

__device__ __forceinline__ uint32_t mt_mix(uint32_t hi_src, uint32_t lo_src) {
    const uint32_t y = (hi_src & 0x80000000U) | (lo_src & 0x7fffffffU);
    return (y >> 1) ^ ((y & 1U) ? kMatrixA : 0U);
}

// 4 waves (one per SIMD), lane p owns position p of every 227-word
// chunk, two chunks per LDS-only barrier.
__global__ __launch_bounds__(kGenThreads) void mt_generate_kernel(uint32_t *__restrict__ state,
                                                                  uint32_t *__restrict__ out,
                                                                  int64_t nwords,
                                                                  uint32_t *__restrict__ state_before) {
    // X[kRing] mirrors X[0] so that x[n-624], x[n-623] are always adjacent (one ds_read2);
    // X[kRing + 1] is a dummy that takes the mirror write of every other lane (no branch)
    __shared__ uint32_t X[kRing + 2];
    __builtin_amdgcn_s_setprio(3);   // one workgroup on a CU shared with HBM-streaming kernels
    const int p = threadIdx.x;
    for (int i = p; i < kMtN; i += kGenThreads) X[i] = state[i];
    if (p == 0) X[kRing] = state[0];
    const int64_t pos0 = (int64_t)state[kMtN];
    if (state_before != nullptr)
        for (int i = p; i <= kMtN; i += kGenThreads) state_before[i] = state[i];
    if (nwords <= 0) return;
    __syncthreads();
    const int64_t end = pos0 + nwords;               // emit stream positions [pos0, end)
    for (int64_t q = pos0 + p; q < kMtN && q < end; q += kGenThreads) out[q - pos0] = X[q];
    const int64_t last = end - 1;
    const int64_t fb = last / kMtN;                  // block holding the last emitted word
    const int64_t need = kMtN * fb + (kMtN - 1);     // generate through the end of that block
    const int64_t nchunks = need >= kMtN ? (need - (kMtN - 1) + kChunk - 1) / kChunk : 0;
    const int64_t niter = (nchunks + 1) / 2;         // two chunks per iteration (output is padded)
    const bool act = p < kChunk;
    constexpr uint32_t M = kRing - 1;
    uint32_t prev = act ? X[kMtM + p] : 0U;          // x[624 + p - 227]
    uint32_t base = (uint32_t)p;                     // (n0 - 624) & M of this lane's chunk-c word
    uint32_t *o = out + (kMtN - pos0) + p;           // out index of stream position 624 + p
    for (int64_t it = 0; it < niter; ++it) {
        if (act) {
            // chunk c reads chunks c-2 / c-3, chunk c+1 reads c-1 / c-2: all written before
            // the last barrier, so the four words come from two ds_read2 issued together
            const uint32_t b1 = (base + kChunk) & M;
            const uint32_t a0 = X[base], c0 = X[base + 1];
            const uint32_t a1 = X[b1], c1 = X[b1 + 1];
            const uint32_t x0 = prev ^ mt_mix(a0, c0);
            const uint32_t x1 = x0 ^ mt_mix(a1, c1);
            const uint32_t w0 = (base + kMtN) & M, w1 = (b1 + kMtN) & M;
            X[w0] = x0;
            X[w1] = x1;
            X[w0 == 0 ? kRing : kRing + 1] = x0;
            X[w1 == 0 ? kRing : kRing + 1] = x1;
            o[0] = x0;                                // raw words; consumers temper
            o[kChunk] = x1;
            o += 2 * kChunk;
            prev = x1;
            base = (b1 + kChunk) & M;
        }
        lds_barrier();                                // every wave, every iteration
    }
    __syncthreads();
    for (int i = p; i < kMtN; i += kGenThreads) state[i] = X[(kMtN * fb + i) & (kRing - 1)];
    if (p == 0) state[kMtN] = (uint32_t)(last - kMtN * fb + 1);
}

}  // namespace rg

extern "C" int rg_mt_generate(void *stream, uint32_t *state_dev, uint32_t *out_words_dev, int64_t nwords,
                              uint32_t *state_before_dev) {
    if (state_dev == nullptr) return rg::fail_arg("rg_mt_generate: null state");
    if (nwords < 0) return rg::fail_arg("rg_mt_generate: nwords < 0");
    if (nwords > 0 && out_words_dev == nullptr) return rg::fail_arg("rg_mt_generate: null output");
    hipLaunchKernelGGL(rg::mt_generate_kernel, dim3(1), dim3(rg::kGenThreads), 0, (hipStream_t)stream,
                       state_dev, out_words_dev, nwords, state_before_dev);
    return rg::check_launch("rg_mt_generate");
}
