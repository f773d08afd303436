// Shared device helpers for librg_hip.so (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/rg_hip.h"

// RG_AB=1 (build.py --variant NAME -DRG_AB=1): the measured-slower alternatives kept for
// same-box A/B runs, selected by RG_* environment switches.  The product library
// is built without them: one tested path per configuration, no environment switches on it.
#ifndef RG_AB
#define RG_AB 0
#endif

namespace rg {

constexpr int kWave = 64;
constexpr int kSc1 = 16;   // buffer-intrinsic cache-policy operand: sc1 (gfx940+ CPol::SC1)

// ---------------------------------------------------------------- errors
void set_error(const std::string &msg);
int fail_arg(const std::string &msg);
// Timing events for the next instrumented launch on this thread (the dense pass of the
// split step): recorded by the kernel dispatch itself (hipExtLaunchKernel), so they time
// the kernel alone and add no marker packets (and no bubbles) to the stream.  Consumed
// (reset) by the launch that uses them.
struct LaunchEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
LaunchEvents &launch_events();
int check_launch(const char *what);
// rg_comm.cpp: all-reduce of buf on the communicator stream, fenced against `stream`
int comm_begin(void *comm, hipStream_t stream, float *buf, int64_t n);
int comm_end(void *comm, hipStream_t stream);
int comm_reduce_scatter(void *comm, hipStream_t stream, float *buf, int64_t chunk);
int comm_allgather(void *comm, hipStream_t stream, int n, float *const *bufs, const int64_t *counts);
hipStream_t comm_stream(void *comm);   // the communicator's own stream
// the all-reduce enqueued on `stream` itself (no cross-stream events; host mode: begin + end)
int comm_allreduce_on(void *comm, hipStream_t stream, float *buf, int64_t n);
// the owner step's MT word exchange: `units` units of W = world * L words each, rank r having
// written words [k W + r L, k W + (r + 1) L) of unit k; afterwards every rank holds every unit's
// W words.  On `stream` (the generator stream), over a communicator of its own (RCCL: split off
// the step's, so it never orders against the step's collectives); host mode: synchronous, through
// the gather callback; local mode: the other slices hashed (a stand-in of the same shape)
int comm_words_prepare(void *comm);
int comm_words_allgather(void *comm, hipStream_t stream, uint32_t *words, int64_t units, int64_t W, int64_t L);
// 0: RCCL, 1: host-staged, 2: local copies
int comm_kind(void *comm);

// ---------------------------------------------------------------- MT jump-ahead
// One step's words as a sequential head + parallel tail segments (rg_mtjump.cpp,
// rg_sampler.hip).  Device buffers are owned by the plan.
constexpr int kMtMaxTail = 32;
struct MtTailSegs {
    int64_t start[kMtMaxTail], len[kMtMaxTail];
    int n;
};
struct MtJumpPlan {
    int64_t words = 0, head = 0;   // words per step, head length
    MtTailSegs segs{};
    int chunks = 0;                // blocks per jump in mt_jump_kernel
    int32_t *terms = nullptr;      // concatenated set bits of t^(D-1) mod chi, per slot
    int32_t *term_off = nullptr;   // [segs.n + 2]
    uint32_t *raw = nullptr;       // [(segs.n + 1) * 624] XOR accumulators
};
// nullptr if `words` is too short for the jump path (then use rg_mt_generate)
// tail < 0: segments of ~20k words; tail = 0: no segments, only the state `words` ahead (a jump)
MtJumpPlan *mt_jump_plan_create(int64_t words, int tail = -1);
// one rank's slices of `units` consecutive units of W words (L words at the start of each, the
// output's unit stride W): the head + parallel segments, the state then units * W ahead
MtJumpPlan *mt_slice_plan_create(int64_t W, int64_t L, int64_t units);
void mt_jump_plan_destroy(MtJumpPlan *plan);
// head -> jump -> tail on `stream`: out[0 .. words) and the next window-form state.  walk > 0
// (a plan without tail segments): the head walks exactly `walk` >= plan.head words into out
// (bounded: nothing past out[walk - 1]) -- one rank's slice of a step's stream, the state then
// jumping `plan.words` ahead of the slice's start
int mt_produce_jump(hipStream_t stream, const MtJumpPlan &plan, uint32_t *state, uint32_t *out,
                    uint32_t *state_before, int64_t walk = 0);
// the local (one-process) stand-in of the owner step's word all-gather: the slices of the other
// ranks, of each of `units` units of `W` words ([R][L] per unit), filled with hashed words
int mt_fill_other_slices(hipStream_t stream, uint32_t *words, int64_t units, int64_t W, int64_t L, int rank,
                         int world, uint32_t seed);

// ---------------------------------------------------------------- prepared pairs
// rg_mf_prepare's output: one record per batch column s (processing order) of
// kPairStride(n) int2 -- [q] = (user, item) of pair q (0: the positive, 1 + k: negative
// k), [n + 1] = (plan slot of the positive's item side, 0) when a plan is given, the rest
// zero -- so a column's ids and slot are one 64-B (n <= 6) or 128-B line.
__host__ __device__ constexpr int pair_stride(int n_neg) { return n_neg + 2 <= 8 ? 8 : 16; }

// ---------------------------------------------------------------- DPP
// Cross-lane moves inside a 16-lane DPP row (no LDS traffic, all lanes valid).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

// Sum over aligned groups of G lanes (G a power of two <= 64); every lane of the
// group ends with the bitwise-identical total (each step adds a value and its
// partner's, which commute exactly).
template <int G>
__device__ __forceinline__ float group_sum(float x) {
    if constexpr (G >= 2) x += dpp_mov<0xB1>(x);    // quad_perm [1,0,3,2]
    if constexpr (G >= 4) x += dpp_mov<0x4E>(x);    // quad_perm [2,3,0,1]
    if constexpr (G >= 8) x += dpp_mov<0x141>(x);   // row_half_mirror
    if constexpr (G >= 16) x += dpp_mov<0x140>(x);  // row_mirror
    if constexpr (G >= 32) x += __shfl_xor(x, 16);
    if constexpr (G >= 64) x += __shfl_xor(x, 32);
    return x;
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS operations
// (lgkmcnt) but leaves its global stores/atomics in flight.  __syncthreads() on
// gfx9 also emits s_waitcnt vmcnt(0), draining every outstanding global store
// before the barrier -- needless when no other thread of the block reads them.
// compute units of the current device (host; cached on first use)
inline int num_cus() {
    static const int n = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
            return 256;
        return v;
    }();
    return n;
}

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---------------------------------------------------------------- MT19937
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}

// CPython random.choices: pop[floor(random() * float(n))] with
// random() = ((a>>5)*2^26 + (b>>6)) / 2^53 on two tempered words (pass the
// raw state words: they are tempered here).  Every
// operation is exact except the final product, which is a single IEEE
// round-to-nearest multiply exactly as in CPython; no contraction is possible.
__device__ __forceinline__ int64_t choice_index(uint32_t w0, uint32_t w1, int64_t n) {
    w0 = mt_temper(w0);
    w1 = mt_temper(w1);
    const double r = ((double)(w0 >> 5) * 67108864.0 + (double)(w1 >> 6)) * (1.0 / 9007199254740992.0);
    return (int64_t)floor(r * (double)n);
}

__device__ __forceinline__ float sigmoidf_ref(float z) { return 1.0f / (1.0f + expf(-z)); }

// ---------------------------------------------------------------- overflow accumulators
// Rows touched more than RG_MF_LIST_CAP times in a step add their surplus contributions
// atomically.  The accumulators are int64 fixed point (2^-48 resolution, range +-32768):
// integer addition is associative, so the sum does not depend on the atomics' arrival
// order, and a row that overflowed sums ALL of its contributions (list and surplus) this
// way -- its gradient is then bit-reproducible whichever contributions the list took.
// Range (no run-time guard: a contribution or running sum of magnitude >= 32768 would wrap):
//  * MF: an element's gradient is sum dz * (partner embedding element), with sum |dz| <= 1
//    over a step (|dL/dp| <= 1/B per pair of a mean loss, |dp/dz| <= 1/4) and embeddings of
//    order 1/d at init, so |sum| stays below ~1 unless the tables themselves diverge;
//  * NCF / NeuMF: dz times the tower's back-propagated input vector (|W|-bounded products of
//    Xavier weights, order 1) or the GMF partner row (N(0,1) init): again sum |dz| <= 1 times
//    an order-one vector.
// Both leave > 4 orders of magnitude of headroom.  Resolution: 2^-49 rounding per
// contribution, below fp32's own rounding of the ~1e-6 contributions a step produces.
constexpr double kFixScale = 281474976710656.0;   // 2^48
__device__ __forceinline__ long long to_fix(float v) { return __double2ll_rn((double)v * kFixScale); }
__device__ __forceinline__ float from_fix(long long x) { return (float)((double)x * (1.0 / kFixScale)); }
__device__ __forceinline__ void fix_add(long long *p, float v) {
    atomicAdd(reinterpret_cast<unsigned long long *>(p), (unsigned long long)to_fix(v));
}

// A row-list entry {other, dz bits} (8 B, scattered over the list lines) stored write-through
// (global_store_dwordx2 sc1): the line leaves the XCD's L2 at once instead of staying dirty for
// the end-of-kernel write-back, which the kernel's end otherwise waits for (~98 k scattered
// entries per MF step).  Measured (profiles/r6/mf/attr_r6f_list_wt.txt): MF pair pass 11.6 ->
// 11.0 us, step 64.4 -> 63.4 us.  The next kernel reads them as before (kernel-boundary acquire).
__device__ __forceinline__ void store_entry(int2 *p, int other, float dz) {
    const uint64_t v = ((uint64_t)(uint32_t)__float_as_int(dz) << 32) | (uint32_t)other;
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), (unsigned long long)v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// torch.optim single-tensor update of one element, in the rounding torch's CPU
// kernels use (checked on the reference's AVX-512 build): add(alpha) and addcmul
// fuse their final multiply-add (FMA), addcdiv rounds (value * t1) / t2 then adds,
// lerp(w = 1 - beta1) takes ATen's two-branch form.  g is the data gradient.
__device__ __forceinline__ float opt_update(const rg_opt_t &o, float p, float gdata, float &m, float &v) {
    const float g = fmaf(o.weight_decay, p, gdata);         // grad.add(param, alpha=wd)
    if (o.kind == RG_OPT_ADAM) {
        const float w = o.one_minus_beta1;                  // exp_avg.lerp_(grad, 1 - beta1)
        m = (fabsf(w) < 0.5f) ? fmaf(w, g - m, m) : fmaf(w - 1.0f, g - m, g);
        v = fmaf(o.one_minus_beta2 * g, g, v * o.beta2);   // mul_(beta2).addcmul_(g, g, 1 - beta2)
        const float denom = sqrtf(v) / o.bias_correction2_sqrt + o.eps;
        return p + ((-o.step_size) * m) / denom;           // addcdiv_(m, denom, -step_size)
    }
    if (o.kind == RG_OPT_SGD) return fmaf(-o.lr, g, p);     // add_(g, alpha=-lr)
    v = fmaf(o.one_minus_alpha * g, g, v * o.alpha);        // RMSprop (centered = False)
    return p + ((-o.lr) * g) / (sqrtf(v) + o.eps);
}


// ---------------------------------------------------------------- row layouts
// A table row of D floats is spread over LPU lanes.  VEC: D == 4 * LPU and each
// lane owns one contiguous float4 (rows are 16-B aligned when D % 4 == 0).
// !VEC: lane l of the row's LPU owns elements l, l + LPU, ... (runtime D <= LPU * EPL);
// consecutive lanes read consecutive floats, so a row is LPU-float coalesced segments.
template <int LPU_, int EPL_, bool VEC_>
struct RowLayout {
    static constexpr int LPU = LPU_;
    static constexpr int EPL = EPL_;
    static constexpr bool VEC = VEC_;
    static constexpr int UPW = kWave / LPU;   // rows (units) per wave

    __device__ static __forceinline__ int elem(int sub, int e) { return VEC ? sub * 4 + e : sub + LPU * e; }

    __device__ static __forceinline__ void load(float (&v)[EPL], const float *__restrict__ base,
                                                int64_t row, int D, int sub) {
        if constexpr (VEC) {
            const float4 t = *reinterpret_cast<const float4 *>(base + row * (int64_t)(4 * LPU) + sub * 4);
            v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
        } else {
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                const int c = sub + LPU * e;
                v[e] = c < D ? base[row * (int64_t)D + c] : 0.0f;
            }
        }
    }

    // row of an array with an explicit row stride (floats; a multiple of 4 for VEC)
    __device__ static __forceinline__ void load_strided(float (&v)[EPL], const float *__restrict__ base,
                                                        int64_t row, int64_t stride, int D, int sub) {
        if constexpr (VEC) {
            const float4 t = *reinterpret_cast<const float4 *>(base + row * stride + sub * 4);
            v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
        } else {
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                const int c = sub + LPU * e;
                v[e] = c < D ? base[row * stride + c] : 0.0f;
            }
        }
    }

    __device__ static __forceinline__ void store(float *__restrict__ base, int64_t row, int D, int sub,
                                                 const float (&v)[EPL]) {
        if constexpr (VEC) {
            *reinterpret_cast<float4 *>(base + row * (int64_t)(4 * LPU) + sub * 4) =
                make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                const int c = sub + LPU * e;
                if (c < D) base[row * (int64_t)D + c] = v[e];
            }
        }
    }

    // streaming (non-temporal) store: the line is not kept dirty in L2, so the
    // end-of-kernel release has less to write back before the next kernel starts
    __device__ static __forceinline__ void store_nt(float *__restrict__ base, int64_t row, int D, int sub,
                                                    const float (&v)[EPL]) {
        if constexpr (VEC) {
            typedef float v4f __attribute__((ext_vector_type(4)));
            v4f t = {v[0], v[1], v[2], v[3]};
            __builtin_nontemporal_store(t, reinterpret_cast<v4f *>(base + row * (int64_t)(4 * LPU) + sub * 4));
        } else {
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                const int c = sub + LPU * e;
                if (c < D) __builtin_nontemporal_store(v[e], base + row * (int64_t)D + c);
            }
        }
    }

    // write-through store (sc1): the bytes go to memory and the line leaves the XCD's L2, so
    // the pass leaves no dirty lines for the end-of-kernel write-back (MI355X guide: "stores of
    // each flavour")
    // write-through store (sc1) of a row slice: one 16-byte buffer store per lane, so every
    // 128-byte row reaches memory as whole lines (two interleaved 8-byte halves would each write
    // half of every sector).  The table must be < 2 GiB (32-bit offsets; the one caller,
    // rg_mf_pipe_step's pipelined kernel (A/B build), checks).  The resource is built from the table's base, which is
    // wave-uniform: a resource per row would be a per-lane value, which buffer instructions take
    // only through a waterfall loop.
    __device__ static __forceinline__ void store_wt(float *__restrict__ base, int64_t row, int D, int sub,
                                                    const float (&v)[EPL]) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0xffffffff, 0x00020000);
        if constexpr (VEC) {
            typedef float v4f __attribute__((ext_vector_type(4)));
            const v4f t = {v[0], v[1], v[2], v[3]};
            __builtin_amdgcn_raw_buffer_store_b128(t, rs, (int)((row * (4 * LPU) + sub * 4) * 4), 0, kSc1);
        } else {
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                const int c = sub + LPU * e;
                if (c < D) __builtin_amdgcn_raw_buffer_store_b32(v[e], rs, (int)((row * D + c) * 4), 0, kSc1);
            }
        }
    }
    __device__ static __forceinline__ void store1_wt(float *p, float v) {
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // global_store_dword ... sc1
    }

    // load past the CU's L1 (sc1: served by L2 / memory): reads rows another workgroup of the
    // same launch wrote with write-through stores (the pipelined MF step's pair pass); < 2 GiB
    __device__ static __forceinline__ void load_sc1(float (&v)[EPL], const float *__restrict__ base,
                                                    int64_t row, int D, int sub) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(base), 0, 0xffffffff,
                                                                           0x00020000);
        if constexpr (VEC) {
            typedef float v4f __attribute__((ext_vector_type(4)));
            const v4f t = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((row * (4 * LPU) + sub * 4) * 4), 0, kSc1);
            v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
        } else {
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                const int c = sub + LPU * e;
                v[e] = c < D ? __builtin_amdgcn_raw_buffer_load_b32(rs, (int)((row * D + c) * 4), 0, kSc1) : 0.0f;
            }
        }
    }
    __device__ static __forceinline__ float load1_sc1(const float *p) {
        return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    __device__ static __forceinline__ void load_nt(float (&v)[EPL], const float *__restrict__ base,
                                                   int64_t row, int D, int sub) {
        if constexpr (VEC) {
            typedef float v4f __attribute__((ext_vector_type(4)));
            const v4f t = __builtin_nontemporal_load(reinterpret_cast<const v4f *>(base + row * (int64_t)(4 * LPU) + sub * 4));
            v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
        } else {
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                const int c = sub + LPU * e;
                v[e] = c < D ? __builtin_nontemporal_load(base + row * (int64_t)D + c) : 0.0f;
            }
        }
    }

    __device__ static __forceinline__ void zero(float (&v)[EPL]) {
#pragma unroll
        for (int e = 0; e < EPL; ++e) v[e] = 0.0f;
    }
};

// A row of D = 4 * LPU * K floats over LPU lanes, K float4 chunks per lane, chunk c of lane
// `sub` at floats (c * LPU + sub) * 4: each chunk is one fully coalesced wave instruction
// (LPU lanes x 16 B contiguous per row).  Used by the dense pass (mf_back_kernel), whose per-row
// arithmetic is element-wise, so any partition of a row over lanes gives the same bits: more
// rows per wave (64 / LPU) and K loads in flight per lane and array instead of one.
template <int LPU_, int K_>
struct RowLayoutV {
    static constexpr int LPU = LPU_;
    static constexpr int K = K_;
    static constexpr int EPL = 4 * K_;
    static constexpr bool VEC = true;
    static constexpr int UPW = kWave / LPU;
    static constexpr int D = 4 * LPU_ * K_;
    __device__ static __forceinline__ int elem(int sub, int e) { return ((e >> 2) * LPU + sub) * 4 + (e & 3); }
    __device__ static __forceinline__ void load(float (&v)[EPL], const float *__restrict__ base, int64_t row, int,
                                                int sub) {
        load_strided(v, base, row, D, 0, sub);
    }
    __device__ static __forceinline__ void load_strided(float (&v)[EPL], const float *__restrict__ base, int64_t row,
                                                        int64_t stride, int, int sub) {
#pragma unroll
        for (int c = 0; c < K; ++c) {
            const float4 t = *reinterpret_cast<const float4 *>(base + row * stride + (c * LPU + sub) * 4);
            v[4 * c] = t.x; v[4 * c + 1] = t.y; v[4 * c + 2] = t.z; v[4 * c + 3] = t.w;
        }
    }
    __device__ static __forceinline__ void store(float *__restrict__ base, int64_t row, int, int sub,
                                                 const float (&v)[EPL]) {
#pragma unroll
        for (int c = 0; c < K; ++c)
            *reinterpret_cast<float4 *>(base + row * (int64_t)D + (c * LPU + sub) * 4) =
                make_float4(v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]);
    }
    __device__ static __forceinline__ void store_nt(float *__restrict__ base, int64_t row, int, int sub,
                                                    const float (&v)[EPL]) {
        typedef float v4f __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int c = 0; c < K; ++c) {
            v4f t = {v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]};
            __builtin_nontemporal_store(t, reinterpret_cast<v4f *>(base + row * (int64_t)D + (c * LPU + sub) * 4));
        }
    }
    __device__ static __forceinline__ void load_nt(float (&v)[EPL], const float *__restrict__ base, int64_t row, int,
                                                   int sub) {
        typedef float v4f __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int c = 0; c < K; ++c) {
            const v4f t = __builtin_nontemporal_load(
                reinterpret_cast<const v4f *>(base + row * (int64_t)D + (c * LPU + sub) * 4));
            v[4 * c] = t.x; v[4 * c + 1] = t.y; v[4 * c + 2] = t.z; v[4 * c + 3] = t.w;
        }
    }
    __device__ static __forceinline__ void store_wt(float *__restrict__ base, int64_t row, int, int sub,
                                                    const float (&v)[EPL]) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0xffffffff, 0x00020000);
        typedef float v4f __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int c = 0; c < K; ++c) {
            const v4f t = {v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]};
            __builtin_amdgcn_raw_buffer_store_b128(t, rs, (int)((row * D + (c * LPU + sub) * 4) * 4), 0, kSc1);
        }
    }
    __device__ static __forceinline__ void store1_wt(float *p, float v) {
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ static __forceinline__ void zero(float (&v)[EPL]) {
#pragma unroll
        for (int e = 0; e < EPL; ++e) v[e] = 0.0f;
    }
};

// A row of an EVEN runtime D <= 2 * LPU * K floats over LPU lanes in float2 pairs: pair c of lane
// `sub` holds floats (c * LPU + sub) * 2 and + 1 (rows 8-B aligned when D is even), masked past D.
// The dense pass's layout for even dims that are not a power of two (NeuMF's GMF width 50): one
// 8-B load per lane and pair instead of a dword per element (element-wise arithmetic, same bits).
template <int LPU_, int K_>
struct RowLayoutP {
    static constexpr int LPU = LPU_;
    static constexpr int EPL = 2 * K_;
    static constexpr bool VEC = false;
    static constexpr int UPW = kWave / LPU;
    __device__ static __forceinline__ int elem(int sub, int e) { return ((e >> 1) * LPU + sub) * 2 + (e & 1); }
    __device__ static __forceinline__ void load_strided(float (&v)[EPL], const float *__restrict__ base, int64_t row,
                                                        int64_t stride, int D, int sub) {
#pragma unroll
        for (int c = 0; c < K_; ++c) {
            const int f = (c * LPU + sub) * 2;
            float2 t = make_float2(0.0f, 0.0f);
            if (f < D) t = *reinterpret_cast<const float2 *>(base + row * stride + f);
            v[2 * c] = t.x; v[2 * c + 1] = t.y;
        }
    }
    __device__ static __forceinline__ void load(float (&v)[EPL], const float *__restrict__ base, int64_t row, int D,
                                                int sub) {
        load_strided(v, base, row, D, D, sub);
    }
    __device__ static __forceinline__ void load_nt(float (&v)[EPL], const float *__restrict__ base, int64_t row, int D,
                                                   int sub) {
        load(v, base, row, D, sub);
    }
    __device__ static __forceinline__ void load_sc1(float (&v)[EPL], const float *__restrict__ base, int64_t row,
                                                    int D, int sub) {
        load(v, base, row, D, sub);   // only the pipelined step (A/B build, d = 64) reads past L1
    }
    __device__ static __forceinline__ void store(float *__restrict__ base, int64_t row, int D, int sub,
                                                 const float (&v)[EPL]) {
#pragma unroll
        for (int c = 0; c < K_; ++c) {
            const int f = (c * LPU + sub) * 2;
            if (f < D) *reinterpret_cast<float2 *>(base + row * (int64_t)D + f) = make_float2(v[2 * c], v[2 * c + 1]);
        }
    }
    __device__ static __forceinline__ void store_nt(float *__restrict__ base, int64_t row, int D, int sub,
                                                    const float (&v)[EPL]) {
        store(base, row, D, sub, v);
    }
    __device__ static __forceinline__ void store_wt(float *__restrict__ base, int64_t row, int D, int sub,
                                                    const float (&v)[EPL]) {
        store(base, row, D, sub, v);  // only the pipelined step (A/B build, d = 64) writes through
    }
    __device__ static __forceinline__ void store1_wt(float *p, float v) {
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ static __forceinline__ float load1_sc1(const float *p) {
        return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ static __forceinline__ void zero(float (&v)[EPL]) {
#pragma unroll
        for (int e = 0; e < EPL; ++e) v[e] = 0.0f;
    }
};

// The dense pass's layout for a dim's pair-pass layout L (mf_back_kernel, single-GPU MF):
// RG_BACK_V32 / _V64 / _V128 = lanes per row of a RowLayoutV for d = 32 / 64 / 128 (0: L itself).
// Measured (round 5, profiles/r5/attr/): d = 64 on 8 lanes x 2 float4 (8 rows per wave) instead of
// 16 lanes x 1 float4: 55.1 -> 51.2 us per dense pass; d = 128 on 16 lanes x 2 float4 instead of
// 32 x 1: 111.7 -> 104.3 us -- twice the bytes in flight per wave at a similar occupancy.
#ifndef RG_BACK_V64
#define RG_BACK_V64 8
#endif
#ifndef RG_BACK_V128
#define RG_BACK_V128 16
#endif
#ifndef RG_BACK_V16
#define RG_BACK_V16 0   // d = 16 on 2 lanes x 2 float4 / 1 x 4: 28.4-30.5 / 33.2-33.5 vs 26.7-28.9 us in the NeuMF
#endif                  // step (its tower's tables), not kept (profiles/r6/ncf/neumf_dense_layouts_r6.txt)
#ifndef RG_BACK_P
#define RG_BACK_P 0     // even dims 33..64 that are not 64 (NeuMF's GMF 50) on RowLayoutP<RG_BACK_P, 32 / RG_BACK_P>
                        // (float2 pairs; lanes per row): 8 lanes measured slower in the NeuMF step, 47.7-47.8 vs
                        // 45.8-46.2 us (profiles/r6/ncf/neumf_dense_layouts_r6.txt)
#endif
#ifndef RG_BACK_V32
#define RG_BACK_V32 4   // d = 32 on 4 lanes x 2 float4 (16 rows per wave) instead of 8 x 1: dense pass
#endif                  // 34.0-34.5 -> 31.5-32.0 us, 140.6-142.0 -> 146.5-146.8 M/s (profiles/r6/mf/attr_r6m_d32.txt)
template <class L>
struct BackLayout {
    using type = L;
};
#if RG_BACK_V64
template <>
struct BackLayout<RowLayout<16, 4, true>> {
    using type = RowLayoutV<RG_BACK_V64, 64 / (4 * RG_BACK_V64)>;
};
#endif
#if RG_BACK_V128
template <>
struct BackLayout<RowLayout<32, 4, true>> {
    using type = RowLayoutV<RG_BACK_V128, 128 / (4 * RG_BACK_V128)>;
};
#endif
#if RG_BACK_V16
template <>
struct BackLayout<RowLayout<4, 4, true>> {
    using type = RowLayoutV<RG_BACK_V16, 16 / (4 * RG_BACK_V16)>;
};
#endif
#if RG_BACK_P
template <>
struct BackLayout<RowLayout<16, 4, false>> {
    using type = RowLayoutP<RG_BACK_P, 32 / RG_BACK_P>;   // even D only: the caller checks (BackLaunchF)
};
#endif
#if RG_BACK_V32
template <>
struct BackLayout<RowLayout<8, 4, true>> {
    using type = RowLayoutV<RG_BACK_V32, 32 / (4 * RG_BACK_V32)>;
};
#endif

// The split step's pair pass on its own row layout (RG_PAIR_V64 / RG_PAIR_V128 lanes per row, 0:
// the dispatch layout): timing experiments of fewer lanes per row in the latency-bound gather
#ifndef RG_PAIR_V64
#define RG_PAIR_V64 0
#endif
#ifndef RG_PAIR_V128
#define RG_PAIR_V128 0
#endif
template <class L>
struct PairLayout {
    using type = L;
};
#if RG_PAIR_V64
template <>
struct PairLayout<RowLayout<16, 4, true>> {
    using type = RowLayoutV<RG_PAIR_V64, 64 / (4 * RG_PAIR_V64)>;
};
#endif
#if RG_PAIR_V128
template <>
struct PairLayout<RowLayout<32, 4, true>> {
    using type = RowLayoutV<RG_PAIR_V128, 128 / (4 * RG_PAIR_V128)>;
};
#endif

// Dispatch on dim: calls f.template operator()<Layout>() for the layout of `dim`.
template <typename F>
inline int dispatch_dim(int dim, F &&f) {
    switch (dim) {
        case 8: return f.template operator()<RowLayout<2, 4, true>>();
        case 16: return f.template operator()<RowLayout<4, 4, true>>();
        case 32: return f.template operator()<RowLayout<8, 4, true>>();
        case 64: return f.template operator()<RowLayout<16, 4, true>>();
        case 128: return f.template operator()<RowLayout<32, 4, true>>();
        case 256: return f.template operator()<RowLayout<64, 4, true>>();
        default: break;
    }
    // other dims <= 64: 16 lanes per row (4 rows per wave) instead of a wave per row
    if (dim >= 1 && dim <= 16) return f.template operator()<RowLayout<16, 1, false>>();
    if (dim <= 32) return f.template operator()<RowLayout<16, 2, false>>();
    if (dim <= 64) return f.template operator()<RowLayout<16, 4, false>>();
    if (dim <= 128) return f.template operator()<RowLayout<64, 2, false>>();
    if (dim <= 192) return f.template operator()<RowLayout<64, 3, false>>();
    if (dim <= 256) return f.template operator()<RowLayout<64, 4, false>>();
    return fail_arg("dim must be in [1, 256]");
}

}  // namespace rg
