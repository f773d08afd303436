// Microbenchmark (scripts only, never shipped): does the table layout of the optimizer state
// move the MF dense pass's stream?  156,785 rows x 64 floats, the product's d = 64 dense layout
// (8 lanes x 2 float4 per row, RowLayoutV<8, 2>), exact Adam arithmetic, biases beside.
//   0: p ping-pong, m and v separate tables (the product)
//   1: p ping-pong, m and v interleaved per row ([m | v], 128 floats)
//   2: p, m, v interleaved per row ([p | m | v], 192 floats), updated in place
//   3: as 0 with p updated in place (no ping-pong)
//   4..7: 0..3 with 1 GB written between passes (untimed): nothing of the tables left in the MALL
// Prints us per pass (median of 40) for each.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));
struct Opt { float beta2, eps, wd, omb1, omb2, step_size, bc2s; };

__device__ __forceinline__ float adam(const Opt &o, float p, float gd, float &m, float &v) {
    const float g = fmaf(o.wd, p, gd);
    const float w = o.omb1;
    m = (fabsf(w) < 0.5f) ? fmaf(w, g - m, m) : fmaf(w - 1.0f, g - m, g);
    v = fmaf(o.omb2 * g, g, v * o.beta2);
    const float denom = sqrtf(v) / o.bc2s + o.eps;
    return p + ((-o.step_size) * m) / denom;
}

__device__ __forceinline__ v4f ld(const float *p) { return *reinterpret_cast<const v4f *>(p); }
__device__ __forceinline__ void st(float *p, v4f v) { *reinterpret_cast<v4f *>(p) = v; }

template <int MODE>
__global__ __launch_bounds__(256) void dense(const float *__restrict__ pin, float *__restrict__ pout,
                                             float *__restrict__ m, float *__restrict__ v, const float *__restrict__ bin,
                                             float *__restrict__ bout, float *__restrict__ bm, float *__restrict__ bv,
                                             const float *__restrict__ grad, long rows, Opt o, int rev) {
    long r = ((long)blockIdx.x * 256 + threadIdx.x) >> 3;
    if (rev) r = rows - 1 - r;     // this pass streams the rows last to first
    if (r < 0) return;
    const int sub = threadIdx.x & 7;
    if (r >= rows) return;
    const long o0 = (long)sub * 4, o1 = (long)(8 + sub) * 4;
    const float *P; float *PO; float *M; float *V;
    if (MODE == 0) { P = pin + r * 64; PO = pout + r * 64; M = m + r * 64; V = v + r * 64; }
    else if (MODE == 1) { P = pin + r * 64; PO = pout + r * 64; M = m + r * 128; V = M + 64; }
    else if (MODE == 2) { P = m + r * 192; PO = m + r * 192; M = m + r * 192 + 64; V = m + r * 192 + 128; }
    else { P = pout + r * 64; PO = pout + r * 64; M = m + r * 64; V = v + r * 64; }
    v4f p0 = ld(P + o0), p1 = ld(P + o1), m0 = ld(M + o0), m1 = ld(M + o1), v0 = ld(V + o0), v1 = ld(V + o1);
    const float gd = grad[r];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float a = m0[k], b = v0[k];
        p0[k] = adam(o, p0[k], gd * (float)(k + 1), a, b);
        m0[k] = a; v0[k] = b;
        a = m1[k]; b = v1[k];
        p1[k] = adam(o, p1[k], gd * (float)(k + 2), a, b);
        m1[k] = a; v1[k] = b;
    }
    st(PO + o0, p0); st(PO + o1, p1); st(M + o0, m0); st(M + o1, m1); st(V + o0, v0); st(V + o1, v1);
    if (sub == 0) {
        float a = bm[r], b = bv[r];
        bout[r] = adam(o, bin[r], gd, a, b);
        bm[r] = a; bv[r] = b;
    }
}

__global__ void fill(float *x, long n, unsigned seed) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        x[i] = (float)(h & 0xffffff) * (1.0f / 16777216.0f) * 0.02f + 1e-4f;   // positive (v under sqrt)
    }
}

int main(int argc, char **argv) {
    // argv[1]: row-count scale (the MALL knee: footprint 1056 B per row for mode 0)
    const double scale = argc > 1 ? atof(argv[1]) : 1.0;
    const int only = argc > 2 ? atoi(argv[2]) : -1;
    // argv[3]: waves per SIMD to allow (dynamic LDS per workgroup caps the workgroups per CU)
    const int occ = argc > 3 ? atoi(argv[3]) : 0;
    const size_t lds = occ > 0 ? (size_t)(160 * 1024 / occ - 256) : 0;
    const long rows = (long)(156785 * scale);
    float *pa, *pb, *m, *v, *ba, *bb, *bm, *bv, *g;
    hipMalloc(&pa, rows * 192 * 4); hipMalloc(&pb, rows * 64 * 4); hipMalloc(&m, rows * 192 * 4);
    hipMalloc(&v, rows * 64 * 4);
    hipMalloc(&ba, rows * 4); hipMalloc(&bb, rows * 4); hipMalloc(&bm, rows * 4); hipMalloc(&bv, rows * 4);
    hipMalloc(&g, rows * 4);
    hipMemset(pa, 0, rows * 192 * 4); hipMemset(pb, 0, rows * 64 * 4); hipMemset(m, 0, rows * 192 * 4);
    hipMemset(v, 0, rows * 64 * 4); hipMemset(ba, 0, rows * 4); hipMemset(bb, 0, rows * 4);
    hipMemset(bm, 0, rows * 4); hipMemset(bv, 0, rows * 4); hipMemset(g, 0, rows * 4);
    // argv[5] = 1: every other pass streams the rows in reverse order
    const int alt = argc > 5 ? atoi(argv[5]) : 0;
    // argv[4] = 1: random positive values instead of zeros
    if (argc > 4 && atoi(argv[4]) == 1) {
        fill<<<4096, 256>>>(pa, rows * 192, 1); fill<<<4096, 256>>>(pb, rows * 64, 2);
        fill<<<4096, 256>>>(m, rows * 192, 3); fill<<<4096, 256>>>(v, rows * 64, 4);
        fill<<<4096, 256>>>(ba, rows, 5); fill<<<4096, 256>>>(bb, rows, 6); fill<<<4096, 256>>>(bm, rows, 7);
        fill<<<4096, 256>>>(bv, rows, 8); fill<<<4096, 256>>>(g, rows, 9);
        hipDeviceSynchronize();
    }
    Opt o{0.999f, 1e-8f, 1e-5f, 0.1f, 0.001f, 1e-3f, 0.03f};
    const int blocks = (int)((rows * 8 + 255) / 256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const double bytes = (double)rows * (6 * 64 * 4 + 6 * 4 + 4);
    void *flush;
    const size_t fbytes = (size_t)1 << 30;
    hipMalloc(&flush, fbytes);
    for (int mm = 0; mm < 8; ++mm) {
        const int mode = mm & 3;
        if (only >= 0 && mm != only && mm != only + 4) continue;
        std::vector<float> t;
        for (int it = 0; it < 50; ++it) {
            const float *pin = (it & 1) ? pb : pa;
            float *pout = (it & 1) ? pa : pb;
            if (mm >= 4) hipMemsetAsync(flush, it & 0xff, fbytes);
            hipEventRecord(e0);
            if (mode == 0) dense<0><<<blocks, 256, lds>>>(pin, pout, m, v, ba, bb, bm, bv, g, rows, o, alt ? (it & 1) : 0);
            if (mode == 1) dense<1><<<blocks, 256, lds>>>(pin, pout, m, v, ba, bb, bm, bv, g, rows, o, alt ? (it & 1) : 0);
            if (mode == 2) dense<2><<<blocks, 256, lds>>>(pin, pout, m, v, ba, bb, bm, bv, g, rows, o, alt ? (it & 1) : 0);
            if (mode == 3) dense<3><<<blocks, 256, lds>>>(pin, pout, m, v, ba, bb, bm, bv, g, rows, o, alt ? (it & 1) : 0);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (it >= 10) t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        printf("occ %d scale %.2f (%.0f MB) mode %d: %.2f us (min %.2f) = %.2f TB/s\n", occ, scale, rows * (mode == 0 ? 1056.0 : 800.0) / 1e6, mm, t[t.size() / 2], t[0], bytes / (t[t.size() / 2] * 1e-6) / 1e12);
    }
    return 0;
}
