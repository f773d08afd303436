// Microbenchmark (scripts only): what the MF dense pass's per-row small arrays cost on
// top of the p, m, v stream.  rows x 64 floats, 16 lanes per row (float4 each), 4 rows
// per wave, one row group per wave (the product kernel's shape), ping-pong p.
//   mode 0: p, m, v only;  1: + the six bias arrays (4 B per row);  2: + count and the
//   64-B list per row;  3: 2 with biases interleaved into 68-float rows (p | pb pad);
//   4: 2 with the product's exact Adam update (rg_common.h opt_update: two IEEE divides);
//   5: 4 + the whole 64-B list (4 int4 per lane) and a 2-int slot range per row;
//   6: 5 + rows split over two tables (items then users, pointers picked per lane);
//   7: 6 + the pull: rows with count > 0 (36 %) gather 1-2 partner rows of the other table.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

struct Opt { int kind; float lr, beta1, beta2, eps, wd, alpha, omb1, omb2, oma, step_size, bc2s; };
__device__ __forceinline__ float opt_update(const Opt &o, float p, float gdata, float &m, float &v) {
    const float g = fmaf(o.wd, p, gdata);
    if (o.kind == 0) {
        const float w = o.omb1;
        m = (fabsf(w) < 0.5f) ? fmaf(w, g - m, m) : fmaf(w - 1.0f, g - m, g);
        v = fmaf(o.omb2 * g, g, v * o.beta2);
        const float denom = sqrtf(v) / o.bc2s + o.eps;
        return p + ((-o.step_size) * m) / denom;
    }
    if (o.kind == 1) return fmaf(-o.lr, g, p);
    v = fmaf(o.oma * g, g, v * o.alpha);
    return p + ((-o.lr) * g) / (sqrtf(v) + o.eps);
}

template <int MODE>
__global__ __launch_bounds__(256) void pass(const float *__restrict__ pin, float *__restrict__ pout,
                                            float *__restrict__ m, float *__restrict__ v,
                                            const float *__restrict__ bin, float *__restrict__ bout,
                                            float *__restrict__ bm, float *__restrict__ bv,
                                            int *__restrict__ cnt, const int4 *__restrict__ lst, long rows, Opt o) {
    const long t = (long)blockIdx.x * 256 + threadIdx.x;
    const long r = t >> 4;
    const int sub = threadIdx.x & 15;
    if (r >= rows) return;
    const int RS = MODE == 3 ? 68 : 64;
    float4 p = *reinterpret_cast<const float4 *>(pin + r * RS + sub * 4);
    float4 a = *reinterpret_cast<const float4 *>(m + r * RS + sub * 4);
    float4 b = *reinterpret_cast<const float4 *>(v + r * RS + sub * 4);
    float pb = 0, mb = 0, vb = 0;
    int c = 0;
    int4 l0 = make_int4(0, 0, 0, 0);
    if (MODE == 1 || MODE == 2 || MODE >= 4) { pb = bin[r]; mb = bm[r]; vb = bv[r]; }
    if (MODE == 3) { pb = pin[r * RS + 64]; mb = m[r * RS + 64]; vb = v[r * RS + 64]; }
    if (MODE >= 2) { c = cnt[r]; l0 = lst[r * 4]; }
    float g = 1e-5f * (c + l0.x);
    if (MODE >= 5) {
        const int4 l1 = lst[r * 4 + 1], l2 = lst[r * 4 + 2], l3 = lst[r * 4 + 3];
        const int s0 = cnt[(r + 1) % rows], s1 = cnt[(r + 2) % rows];
        g += 1e-6f * (l1.x + l2.y + l3.z + s0 + s1);
    }
    if (MODE >= 7 && c > 0) {
        const int ne = c < 8 ? c : 8;
        for (int e = 0; e < ne; ++e) {
            const float4 q = *reinterpret_cast<const float4 *>(pin + (long)((l0.x + e * 7919) % rows) * RS + sub * 4);
            g += 1e-7f * q.x;
        }
    }
    if (MODE >= 4) {
        p.x = opt_update(o, p.x, g, a.x, b.x); p.y = opt_update(o, p.y, g, a.y, b.y);
        p.z = opt_update(o, p.z, g, a.z, b.z); p.w = opt_update(o, p.w, g, a.w, b.w);
        pb = opt_update(o, pb, g, mb, vb);
    } else {
    a.x = 0.5f * a.x + 0.5f * (p.x * 1e-5f + g); a.y = 0.5f * a.y + 0.5f * p.y * 1e-5f;
    a.z = 0.5f * a.z + 0.5f * p.z * 1e-5f; a.w = 0.5f * a.w + 0.5f * p.w * 1e-5f;
    b.x = 0.999f * b.x + 1e-3f * a.x * a.x; b.y = 0.999f * b.y + 1e-3f * a.y * a.y;
    b.z = 0.999f * b.z + 1e-3f * a.z * a.z; b.w = 0.999f * b.w + 1e-3f * a.w * a.w;
    p.x -= 1e-3f * a.x / (sqrtf(b.x) + 1e-8f); p.y -= 1e-3f * a.y / (sqrtf(b.y) + 1e-8f);
    p.z -= 1e-3f * a.z / (sqrtf(b.z) + 1e-8f); p.w -= 1e-3f * a.w / (sqrtf(b.w) + 1e-8f);
    }
    *reinterpret_cast<float4 *>(pout + r * RS + sub * 4) = p;
    *reinterpret_cast<float4 *>(m + r * RS + sub * 4) = a;
    *reinterpret_cast<float4 *>(v + r * RS + sub * 4) = b;
    if (sub == 0) {
        if (MODE == 1 || MODE == 2) { bout[r] = pb * 0.999f; bm[r] = mb * 0.5f; bv[r] = vb * 0.9f; }
        if (MODE >= 4) { bout[r] = pb; bm[r] = mb; bv[r] = vb; }
        if (MODE == 3) { pout[r * RS + 64] = pb * 0.999f; m[r * RS + 64] = mb * 0.5f; v[r * RS + 64] = vb * 0.9f; }
        if (MODE >= 2 && MODE < 5 && c) cnt[r] = 0;
    }
}

template <int MODE>
void run(long rows, float **P, float *m, float *v, float **B, float *bm, float *bv, int *cnt, int4 *lst) {
    Opt o{0, 1e-3f, 0.5f, 0.999f, 1e-8f, 1e-5f, 0.99f, 0.5f, 0.001f, 0.01f, 2e-3f, 0.03f};
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int grid = (int)((rows * 16 + 255) / 256);
    for (int w = 0; w < 10; ++w)
        hipLaunchKernelGGL(pass<MODE>, dim3(grid), dim3(256), 0, 0, P[0], P[1], m, v, B[0], B[1], bm, bv, cnt, lst, rows, o);
    hipEventRecord(a, 0);
    const int it = 50;
    for (int k = 0; k < it; ++k) {
        const int s = k & 1;
        hipLaunchKernelGGL(pass<MODE>, dim3(grid), dim3(256), 0, 0, P[s], P[1 - s], m, v, B[s], B[1 - s], bm, bv, cnt,
                           lst, rows, o);
    }
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("mode %d rows %ld: %.2f us/pass\n", MODE, rows, ms * 1e3 / it);
}

int main(int argc, char **argv) {
    const long rows = argc > 1 ? atol(argv[1]) : 156785;
    float *P[2], *m, *v, *B[2], *bm, *bv;
    int *cnt;
    int4 *lst;
    const size_t tb = rows * 68 * 4;
    hipMalloc(&P[0], tb); hipMalloc(&P[1], tb); hipMalloc(&m, tb); hipMalloc(&v, tb);
    hipMalloc(&B[0], rows * 4); hipMalloc(&B[1], rows * 4); hipMalloc(&bm, rows * 4); hipMalloc(&bv, rows * 4);
    hipMalloc(&cnt, rows * 4); hipMalloc(&lst, rows * 64);
    hipMemset(P[0], 0, tb); hipMemset(P[1], 0, tb); hipMemset(m, 0, tb); hipMemset(v, 0, tb);
    hipMemset(B[0], 0, rows * 4); hipMemset(B[1], 0, rows * 4); hipMemset(bm, 0, rows * 4); hipMemset(bv, 0, rows * 4);
    hipMemset(cnt, 0, rows * 4); hipMemset(lst, 0, rows * 64);
    {
        int *hc = (int *)malloc(rows * 4);
        int4 *hl = (int4 *)malloc(rows * 64);
        srand(1);
        for (long r = 0; r < rows; ++r) {
            hc[r] = (rand() % 100) < 36 ? 1 + rand() % 2 : 0;
            for (int k = 0; k < 4; ++k) hl[r * 4 + k] = make_int4(rand() % (int)rows, 0, rand() % (int)rows, 0);
        }
        hipMemcpy(cnt, hc, rows * 4, hipMemcpyHostToDevice);
        hipMemcpy(lst, hl, rows * 64, hipMemcpyHostToDevice);
    }
    for (int rep = 0; rep < 2; ++rep) {
        run<0>(rows, P, m, v, B, bm, bv, cnt, lst);
        run<1>(rows, P, m, v, B, bm, bv, cnt, lst);
        run<2>(rows, P, m, v, B, bm, bv, cnt, lst);
        run<3>(rows, P, m, v, B, bm, bv, cnt, lst);
        run<4>(rows, P, m, v, B, bm, bv, cnt, lst);
        run<5>(rows, P, m, v, B, bm, bv, cnt, lst);
        run<7>(rows, P, m, v, B, bm, bv, cnt, lst);
    }
    return 0;
}
