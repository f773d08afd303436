// MT19937 word-stream walk shared by the sampler kernels (rg_sampler.hip) and the
// MF dense pass (rg_mf.hip), which hosts the walk of a later step's words in one of
// its workgroups.  See rg_sampler.hip for the recurrence and the LDS ring.
#pragma once

#include "rg_common.h"

namespace rg {

constexpr int kMtN = 624;
constexpr int kMtM = 397;
constexpr int kChunk = kMtN - kMtM;     // 227
constexpr int kRing = 2048;             // words of stream kept in LDS (power of two)
constexpr uint32_t kMatrixA = 0x9908b0dfU;
constexpr int kGenThreads = 256;
#ifndef RG_MT_WAVE_WALK
#define RG_MT_WAVE_WALK 0     // 1: mt_generate_block walks on one wave (mt_walk_wave; measured 3.4x slower: 127 vs 37 us)
#endif

__device__ __forceinline__ uint32_t mt_mix(uint32_t hi_src, uint32_t lo_src) {
    const uint32_t y = (hi_src & 0x80000000U) | (lo_src & 0x7fffffffU);
    return (y >> 1) ^ ((y & 1U) ? kMatrixA : 0U);
}

// 4 waves (one per SIMD), lane p owns position p of every 227-word chunk, two
// chunks per LDS-only barrier.  X[0 .. 624) holds the state block (X[kRing] mirrors
// X[0]); emits stream positions [pos0, pos0 + nwords) of that block's stream to
// out[0 ..).  BOUNDED: never store at out[nwords] or beyond (segments written
// side by side); otherwise up to two chunks past the end are written (padded
// output).  Returns the block index fb holding the last emitted word; that block
// is X[(624 fb + i) & (kRing - 1)] afterwards.
template <bool BOUNDED>
__device__ __forceinline__ int64_t mt_walk(uint32_t *X, int p, int64_t pos0, int64_t nwords, uint32_t *out) {
    const int64_t end = pos0 + nwords;               // emit stream positions [pos0, end)
    for (int64_t q = pos0 + p; q < kMtN && q < end; q += kGenThreads) out[q - pos0] = X[q];
    const int64_t last = end - 1;
    const int64_t fb = last / kMtN;                  // block holding the last emitted word
    const int64_t need = kMtN * fb + (kMtN - 1);     // generate through the end of that block
    const int64_t nchunks = need >= kMtN ? (need - (kMtN - 1) + kChunk - 1) / kChunk : 0;
    const int64_t niter = (nchunks + 1) / 2;         // two chunks per iteration
    const bool act = p < kChunk;
    constexpr uint32_t M = kRing - 1;
    uint32_t prev = act ? X[kMtM + p] : 0U;          // x[624 + p - 227]
    uint32_t base = (uint32_t)p;                     // (n0 - 624) & M of this lane's chunk-c word
    int64_t oi = (kMtN - pos0) + p;                  // out index of stream position 624 + p
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
            if (!BOUNDED || oi < nwords) out[oi] = x0;              // raw words; consumers temper
            if (!BOUNDED || oi + kChunk < nwords) out[oi + kChunk] = x1;
            oi += 2 * kChunk;
            prev = x1;
            base = (b1 + kChunk) & M;
        }
        lds_barrier();                                // every wave, every iteration
    }
    __syncthreads();
    return fb;
}

// The same walk by ONE wave (lanes 0..63 of the workgroup's first wave; the caller's other waves
// skip it and meet it at a __syncthreads after): lane l owns positions l, l + 64, l + 128 and
// l + 192 (< 227) of every chunk.  Every word an iteration reads was written in an earlier one
// (mt_walk's two-chunk argument), and a single wave's LDS operations complete in order, so no
// barrier is needed: one LDS round trip per two chunks instead of a read + a 4-wave barrier.  The
// stream and the state left in X are mt_walk's, word for word (the unbounded form).
__device__ __forceinline__ int64_t mt_walk_wave(uint32_t *X, int lane, int64_t pos0, int64_t nwords,
                                                uint32_t *out) {
    constexpr int kPer = (kChunk + kWave - 1) / kWave;   // 4 positions per lane (lanes >= 35: 3)
    const int64_t end = pos0 + nwords;
    for (int64_t q = pos0 + lane; q < kMtN && q < end; q += kWave) out[q - pos0] = X[q];
    const int64_t last = end - 1;
    const int64_t fb = last / kMtN;
    const int64_t need = kMtN * fb + (kMtN - 1);
    const int64_t nchunks = need >= kMtN ? (need - (kMtN - 1) + kChunk - 1) / kChunk : 0;
    const int64_t niter = (nchunks + 1) / 2;
    constexpr uint32_t M = kRing - 1;
    uint32_t prev[kPer], base[kPer];
    bool act[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int p = lane + j * kWave;
        act[j] = p < kChunk;
        prev[j] = act[j] ? X[kMtM + p] : 0U;
        base[j] = (uint32_t)p;
    }
    int64_t oi = (kMtN - pos0) + lane;
    for (int64_t it = 0; it < niter; ++it) {
        uint32_t a0[kPer], c0[kPer], a1[kPer], c1[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j) {          // every read of the iteration first: one round trip
            const uint32_t b1 = (base[j] + kChunk) & M;
            a0[j] = act[j] ? X[base[j]] : 0U;
            c0[j] = act[j] ? X[base[j] + 1] : 0U;
            a1[j] = act[j] ? X[b1] : 0U;
            c1[j] = act[j] ? X[b1 + 1] : 0U;
        }
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            if (!act[j]) continue;
            const uint32_t b1 = (base[j] + kChunk) & M;
            const uint32_t x0 = prev[j] ^ mt_mix(a0[j], c0[j]);
            const uint32_t x1 = x0 ^ mt_mix(a1[j], c1[j]);
            const uint32_t w0 = (base[j] + kMtN) & M, w1 = (b1 + kMtN) & M;
            X[w0] = x0;
            X[w1] = x1;
            if (w0 == 0) X[kRing] = x0;
            if (w1 == 0) X[kRing] = x1;
            const int64_t o = oi + j * kWave;
            out[o] = x0;
            out[o + kChunk] = x1;
            prev[j] = x1;
            base[j] = (b1 + kChunk) & M;
        }
        oi += 2 * kChunk;
    }
    return fb;
}

__device__ __forceinline__ void mt_load(uint32_t *X, int p, const uint32_t *state) {
    for (int i = p; i < kMtN; i += kGenThreads) X[i] = state[i];
    if (p == 0) X[kRing] = state[0];
}

// One workgroup of kGenThreads threads: CPython's stream from `state` (624 words +
// position, advanced in place) -> raw words out[0 .. nwords) (+ up to two chunks of
// padding), the entry state copied to state_before first (optional).  X: LDS ring of
// kRing + 2 words.  Every thread of the workgroup must call it.
__device__ __forceinline__ void mt_generate_block(uint32_t *X, uint32_t *__restrict__ state,
                                                  uint32_t *__restrict__ out, int64_t nwords,
                                                  uint32_t *__restrict__ state_before) {
    const int p = threadIdx.x;
    mt_load(X, p, state);
    const int64_t pos0 = (int64_t)state[kMtN];
    if (state_before != nullptr)
        for (int i = p; i <= kMtN; i += kGenThreads) state_before[i] = state[i];
    if (nwords <= 0) return;
    __syncthreads();
#if RG_MT_WAVE_WALK
    int64_t fb = 0;
    if (p < kWave) fb = mt_walk_wave(X, p, pos0, nwords, out);
    __syncthreads();
    fb = (pos0 + nwords - 1) / kMtN;                 // every thread: the block of the last word
#else
    const int64_t fb = mt_walk<false>(X, p, pos0, nwords, out);
#endif
    for (int i = p; i < kMtN; i += kGenThreads) state[i] = X[(kMtN * fb + i) & (kRing - 1)];
    if (p == 0) state[kMtN] = (uint32_t)(pos0 + nwords - 1 - kMtN * fb + 1);
}

}  // namespace rg
