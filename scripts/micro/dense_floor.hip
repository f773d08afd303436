// Microbenchmark (scripts only, never shipped): the floor of the MF dense pass and what the
// kernel boundary in front of the pair pass costs, by the dense pass's store flavour.
//   stream<ST>: every row of U + I = 156,785 rows x 64 floats, ping-pong p, in-place m, v,
//               the six bias arrays, the exact Adam arithmetic (rg_common.h opt_update);
//               ST 0 plain stores, 1 nontemporal, 2 write-through (sc1)
//   gather:     a pair-pass-shaped follower: 49,152 pairs, user row + item row + biases
//               gathered by 16 lanes each, dot, sigmoid, one score out
// Prints us per pass for: stream alone, gather alone, stream -> gather alternating.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));

struct Opt { float lr, beta1, beta2, eps, wd, omb1, omb2, step_size, bc2s; };
__device__ __forceinline__ float adam(const Opt &o, float p, float gdata, float &m, float &v) {
    const float g = fmaf(o.wd, p, gdata);
    const float w = o.omb1;
    m = (fabsf(w) < 0.5f) ? fmaf(w, g - m, m) : fmaf(w - 1.0f, g - m, g);
    v = fmaf(o.omb2 * g, g, v * o.beta2);
    const float denom = sqrtf(v) / o.bc2s + o.eps;
    return p + ((-o.step_size) * m) / denom;
}

template <int ST>
__device__ __forceinline__ void st4(float *p, v4f v) {
    if (ST == 0) *reinterpret_cast<v4f *>(p) = v;
    else if (ST == 1) __builtin_nontemporal_store(v, reinterpret_cast<v4f *>(p));
    else asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
template <int ST>
__device__ __forceinline__ void st1(float *p, float v) {
    if (ST == 0) *p = v;
    else if (ST == 1) __builtin_nontemporal_store(v, p);
    else asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

template <int ST>
__global__ __launch_bounds__(256) void stream(const float *__restrict__ pin, float *__restrict__ pout,
                                              float *__restrict__ m, float *__restrict__ v,
                                              const float *__restrict__ bin, float *__restrict__ bout,
                                              float *__restrict__ bm, float *__restrict__ bv, long rows, Opt o) {
    const long t = (long)blockIdx.x * 256 + threadIdx.x;
    const long r = t >> 4;
    const int sub = threadIdx.x & 15;
    if (r >= rows) return;
    v4f p = *reinterpret_cast<const v4f *>(pin + r * 64 + sub * 4);
    v4f a = *reinterpret_cast<const v4f *>(m + r * 64 + sub * 4);
    v4f b = *reinterpret_cast<const v4f *>(v + r * 64 + sub * 4);
    float pb = 0, mb = 0, vb = 0;
    if (sub == 0) { pb = bin[r]; mb = bm[r]; vb = bv[r]; }
#pragma unroll
    for (int e = 0; e < 4; ++e) { float mm = a[e], vv = b[e]; p[e] = adam(o, p[e], 0.0f, mm, vv); a[e] = mm; b[e] = vv; }
    st4<ST>(pout + r * 64 + sub * 4, p);
    st4<ST>(m + r * 64 + sub * 4, a);
    st4<ST>(v + r * 64 + sub * 4, b);
    if (sub == 0) {
        pb = adam(o, pb, 0.0f, mb, vb);
        st1<ST>(bout + r, pb); st1<ST>(bm + r, mb); st1<ST>(bv + r, vb);
    }
}

__global__ __launch_bounds__(256) void gather(const float *__restrict__ w, const float *__restrict__ b,
                                              const int2 *__restrict__ ids, float *__restrict__ out, long n,
                                              long users) {
    const long t = (long)blockIdx.x * 256 + threadIdx.x;
    const long q = t >> 4;
    const int sub = threadIdx.x & 15;
    if (q >= n) return;
    const int2 id = ids[q];
    const long ur = id.x, ir = users + id.y;
    const v4f x = *reinterpret_cast<const v4f *>(w + ur * 64 + sub * 4);
    const v4f y = *reinterpret_cast<const v4f *>(w + ir * 64 + sub * 4);
    float d = x[0] * y[0] + x[1] * y[1] + x[2] * y[2] + x[3] * y[3];
    for (int o = 8; o > 0; o >>= 1) d += __shfl_xor(d, o, 16);
    d += b[ur] + b[ir];
    if (sub == 0) out[q] = 1.0f / (1.0f + expf(-d));
}

// touches `lines` random 128-B lines of a large buffer (the pair pass's pool gathers and the
// rest of a step's traffic that competes with the tables for the Infinity Cache)
__global__ __launch_bounds__(256) void pollute(const float *__restrict__ buf, long nlines, long lines, unsigned seed,
                                               float *__restrict__ sink) {
    const long t = (long)blockIdx.x * 256 + threadIdx.x;
    if (t >= lines) return;
    unsigned x = (unsigned)t * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    const float v = buf[((long)x % nlines) * 32];
    if (v == 12345.0f) sink[0] = v;
}

int main(int argc, char **argv) {
    const int random_data = argc > 1 ? atoi(argv[1]) : 0;
    const long U = 136677, I = 20108, rows = U + I, npairs = 49152;
    const size_t tb = rows * 64 * 4;
    float *P[2], *m, *v, *B[2], *bm, *bv, *out;
    int2 *ids;
    hipMalloc(&P[0], tb); hipMalloc(&P[1], tb); hipMalloc(&m, tb); hipMalloc(&v, tb);
    for (int k = 0; k < 2; ++k) hipMalloc(&B[k], rows * 4);
    hipMalloc(&bm, rows * 4); hipMalloc(&bv, rows * 4); hipMalloc(&out, npairs * 4); hipMalloc(&ids, npairs * 8);
    hipMemset(P[0], 0, tb); hipMemset(P[1], 0, tb); hipMemset(m, 0, tb); hipMemset(v, 0, tb);
    hipMemset(B[0], 0, rows * 4); hipMemset(B[1], 0, rows * 4); hipMemset(bm, 0, rows * 4); hipMemset(bv, 0, rows * 4);
    if (random_data) {     // tables of N(0, 1/64)-like values, m ~ 1e-6, v ~ 1e-12, not zeros
        std::vector<float> hv(rows * 64);
        srand(3);
        for (auto &x : hv) x = ((rand() & 0xffff) - 32768) * (1.0f / 32768 / 64);
        hipMemcpy(P[0], hv.data(), tb, hipMemcpyHostToDevice);
        hipMemcpy(P[1], hv.data(), tb, hipMemcpyHostToDevice);
        for (auto &x : hv) x *= 1e-4f;
        hipMemcpy(m, hv.data(), tb, hipMemcpyHostToDevice);
        for (auto &x : hv) x = x * x + 1e-12f;
        hipMemcpy(v, hv.data(), tb, hipMemcpyHostToDevice);
    }
    const long big = 1l << 30;   // 1 GiB pollution buffer (pool + positives + plans + ring are ~0.5 GB)
    float *junk, *sink;
    hipMalloc(&junk, big); hipMemset(junk, 0, big); hipMalloc(&sink, 64);
    std::vector<int2> h(npairs);
    srand(7);
    for (long k = 0; k < npairs; ++k) h[k] = make_int2(rand() % (int)U, rand() % (int)I);
    hipMemcpy(ids, h.data(), npairs * 8, hipMemcpyHostToDevice);
    Opt o{1e-3f, 0.5f, 0.999f, 1e-8f, 1e-5f, 0.5f, 0.001f, 2e-3f, 0.03f};
    const int sg = (int)((rows * 16 + 255) / 256), gg = (int)((npairs * 16 + 255) / 256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    size_t lds = 0;                                           // dynamic LDS per block (occupancy sweep)
    auto launch = [&](int st, int s) {
        if (st == 0) hipLaunchKernelGGL(stream<0>, dim3(sg), dim3(256), lds, 0, P[s], P[1 - s], m, v, B[s], B[1 - s], bm, bv, rows, o);
        if (st == 1) hipLaunchKernelGGL(stream<1>, dim3(sg), dim3(256), 0, 0, P[s], P[1 - s], m, v, B[s], B[1 - s], bm, bv, rows, o);
        if (st == 2) hipLaunchKernelGGL(stream<2>, dim3(sg), dim3(256), 0, 0, P[s], P[1 - s], m, v, B[s], B[1 - s], bm, bv, rows, o);
    };
    long pl = 0;                                              // lines polluted per iteration
    unsigned seed = 1;
    auto polluter = [&]() {
        if (pl > 0) hipLaunchKernelGGL(pollute, dim3((unsigned)((pl + 255) / 256)), dim3(256), 0, 0, junk, big / 128, pl,
                                       seed++, sink);
    };
    auto timeit = [&](const char *what, int st, int mode) {   // mode 0 stream, 1 gather, 2 both
        const int it = 200;
        for (int k = 0; k < 20; ++k) {
            if (mode == 0 || mode == 2) launch(st, k & 1);
            if (mode == 1 || mode == 2) hipLaunchKernelGGL(gather, dim3(gg), dim3(256), 0, 0, P[(k + 1) & 1], B[(k + 1) & 1], ids, out, npairs, U);
        }
        hipEventRecord(e0, 0);
        for (int k = 0; k < it; ++k) {
            polluter();
            if (mode == 0 || mode == 2) launch(st, k & 1);
            if (mode == 1 || mode == 2) hipLaunchKernelGGL(gather, dim3(gg), dim3(256), 0, 0, P[(k + 1) & 1], B[(k + 1) & 1], ids, out, npairs, U);
        }
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / it;
        printf("%-28s store %d: %7.2f us/iter", what, st, us);
        if (mode == 0) printf("  %.2f TB/s algorithmic", 6.0 * rows * 65 * 4 / us / 1e6);
        printf("\n");
    };
    printf("random_data %d\n", random_data);
    timeit("gather alone", 0, 1);
    for (int st = 0; st < 3; st += 2) {
        timeit("stream alone", st, 0);
        timeit("stream -> gather", st, 2);
    }
    for (int per_cu : {6, 4, 3, 2}) {      // resident blocks per CU (waves per SIMD) by LDS
        lds = 160 * 1024 / per_cu - 1024;
        char what[64];
        snprintf(what, sizeof what, "stream, %d blocks/CU", per_cu);
        timeit(what, 0, 0);
    }
    lds = 0;
    for (long mb : {2, 8, 32, 64}) {      // MB of random lines pulled in per iteration
        pl = mb * (1l << 20) / 128;
        char what[64];
        snprintf(what, sizeof what, "pollute %ld MB + stream", mb);
        timeit(what, 0, 0);
        snprintf(what, sizeof what, "pollute %ld MB alone", mb);
        timeit(what, 0, 3);
    }
    pl = 0;
    hipError_t err = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(err));
    return err == hipSuccess ? 0 : 1;
}
