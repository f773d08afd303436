// NumPy legacy RandomState.randint(low, high, size) (int64 output) on the GPU: the
// uniform item sampler of spotlight/sampling.py:9-35 (`sample_items`,
// random_state.randint(0, num_items, shape)).
//
// NumPy's algorithm (random/_bounded_integers.pyx `_rand_int64` ->
// distributions.c `random_bounded_uint64_fill`, legacy masked rejection): with
// rng = high - 1 - low and 0 < rng <= 0xFFFFFFFF, every output draws 32-bit MT19937
// words, keeps word & mask (mask = the smallest 2^k - 1 >= rng) and redraws while
// that exceeds rng; out = low + value.  rng == 0xFFFFFFFF takes every word as is;
// rng == 0 draws nothing (the caller fills `low`).
//
// On the device the words are generated ahead (rg_mt_generate, raw state words), and
// the rejection becomes an ordered stream compaction: count the accepted words of
// each 2,048-word block, one workgroup turns the counts into exclusive offsets, and
// each block scatters its accepted values to offset + in-block rank.  The thread
// holding the n-th accepted word reports how many words the draw consumed, which
// the caller uses to advance the generator state exactly as NumPy would.
#include "rg_common.h"

namespace rg {

namespace {

constexpr int kUThreads = 256;
constexpr int kUPer = 8;                         // consecutive words per thread
constexpr int kUWords = kUThreads * kUPer;       // words per block
constexpr int kScanThreads = 1024;

__device__ __forceinline__ bool accept(uint32_t raw, uint32_t mask, uint32_t rng, uint32_t &v) {
    v = mt_temper(raw) & mask;
    return v <= rng;
}

// block sum of `x` (all threads get it); `red` holds kUThreads / 64 entries
__device__ __forceinline__ int block_exclusive(int x, int *red, int &total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    if (lane == 63) red[w] = incl;
    __syncthreads();
    int before = 0;
    total = 0;
#pragma unroll
    for (int k = 0; k < kUThreads / 64; ++k) {
        if (k < w) before += red[k];
        total += red[k];
    }
    return before + incl - x;
}

__global__ __launch_bounds__(kUThreads) void uniform_count_kernel(const uint32_t *__restrict__ words, int64_t nwords,
                                                                  uint32_t mask, uint32_t rng,
                                                                  int32_t *__restrict__ counts) {
    __shared__ int red[kUThreads / 64];
    const int64_t w0 = (int64_t)blockIdx.x * kUWords + (int64_t)threadIdx.x * kUPer;
    int c = 0;
#pragma unroll
    for (int j = 0; j < kUPer; ++j) {
        uint32_t v;
        if (w0 + j < nwords && accept(words[w0 + j], mask, rng, v)) ++c;
    }
    int total;
    block_exclusive(c, red, total);
    if (threadIdx.x == 0) counts[blockIdx.x] = total;
}

// exclusive offsets of the block counts, in place (one workgroup; chunked per thread)
__global__ __launch_bounds__(kScanThreads) void uniform_scan_kernel(int32_t *__restrict__ counts, int nblocks,
                                                                    int64_t *__restrict__ offsets) {
    __shared__ int64_t part[kScanThreads];
    const int t = threadIdx.x, per = (nblocks + kScanThreads - 1) / kScanThreads;
    const int b0 = t * per, b1 = min(nblocks, b0 + per);
    int64_t s = 0;
    for (int b = b0; b < b1; ++b) s += counts[b];
    part[t] = s;
    __syncthreads();
    for (int off = 1; off < kScanThreads; off <<= 1) {   // Hillis-Steele inclusive scan
        const int64_t y = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += y;
        __syncthreads();
    }
    int64_t run = part[t] - s;
    for (int b = b0; b < b1; ++b) {
        offsets[b] = run;
        run += counts[b];
    }
    if (t == kScanThreads - 1) offsets[nblocks] = part[t];   // total accepted
}

__global__ __launch_bounds__(kUThreads) void uniform_scatter_kernel(const uint32_t *__restrict__ words, int64_t nwords,
                                                                    uint32_t mask, uint32_t rng, int64_t low,
                                                                    const int64_t *__restrict__ offsets, int64_t n_out,
                                                                    int64_t *__restrict__ out,
                                                                    int64_t *__restrict__ consumed) {
    __shared__ int red[kUThreads / 64];
    const int64_t base = offsets[blockIdx.x];
    if (base >= n_out) return;   // uniform over the block
    const int64_t w0 = (int64_t)blockIdx.x * kUWords + (int64_t)threadIdx.x * kUPer;
    uint32_t v[kUPer];
    bool ok[kUPer];
    int c = 0;
#pragma unroll
    for (int j = 0; j < kUPer; ++j) {
        ok[j] = w0 + j < nwords && accept(words[w0 + j], mask, rng, v[j]);
        c += ok[j] ? 1 : 0;
    }
    int total;
    int64_t r = base + block_exclusive(c, red, total);
#pragma unroll
    for (int j = 0; j < kUPer; ++j) {
        if (!ok[j]) continue;
        if (r < n_out) out[r] = low + (int64_t)v[j];
        if (r == n_out - 1) *consumed = w0 + j + 1;
        ++r;
    }
}

uint32_t gen_mask(uint32_t rng) {   // smallest 2^k - 1 >= rng
    uint32_t m = rng;
    m |= m >> 1;
    m |= m >> 2;
    m |= m >> 4;
    m |= m >> 8;
    m |= m >> 16;
    return m;
}

}  // namespace

}  // namespace rg

using namespace rg;

extern "C" int64_t rg_uniform_scratch_len(int64_t n_words) {
    if (n_words < 0) return -1;
    const int64_t nb = (n_words + kUWords - 1) / kUWords;
    return nb + 2 * (nb + 1) + 2;   // int32 counts, then int64 offsets (8-byte aligned)
}

extern "C" int rg_uniform_int64(void *stream, const uint32_t *words, int64_t n_words, int64_t low, int64_t high,
                                int64_t n_out, int64_t *out, int32_t *scratch, int64_t *consumed) {
    const int64_t span = high - low;
    if (!words || !out || !scratch || !consumed || n_words < 0 || n_out < 0)
        return fail_arg("rg_uniform_int64: bad argument");
    if (span < 2 || span - 1 > (int64_t)0xFFFFFFFFLL)
        return fail_arg("rg_uniform_int64: needs 2 <= high - low <= 2^32 (high - low == 1 draws nothing)");
    const int64_t nb = (n_words + kUWords - 1) / kUWords;
    if (nb < 1 || nb > (int64_t)1 << 30) return fail_arg("rg_uniform_int64: word count out of range");
    const uint32_t rng = (uint32_t)(span - 1), mask = gen_mask(rng);
    hipStream_t st = (hipStream_t)stream;
    int32_t *counts = scratch;
    int64_t *offsets = reinterpret_cast<int64_t *>(scratch + ((nb + 1) & ~(int64_t)1));
    hipMemsetAsync(consumed, 0, sizeof(int64_t), st);
    hipLaunchKernelGGL(uniform_count_kernel, dim3((unsigned)nb), dim3(kUThreads), 0, st, words, n_words, mask, rng,
                       counts);
    hipLaunchKernelGGL(uniform_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, counts, (int)nb, offsets);
    hipLaunchKernelGGL(uniform_scatter_kernel, dim3((unsigned)nb), dim3(kUThreads), 0, st, words, n_words, mask, rng,
                       low, offsets, n_out, out, consumed);
    return check_launch("rg_uniform_int64");
}
