// Microbenchmark (scripts only): the PRODUCT dense pass (librg_hip.so rg_mf_apply_prepare,
// rg_mf_apply) on micro-style allocations, beside the micro's own streaming kernel on the same
// buffers, in one process: is the product kernel slower than a plain stream of the same bytes,
// or is it the bench's environment?  Tables ML-20M-shaped (U = 136,677, I = 20,108, d = 64),
// random values, empty contribution lists (every row's data gradient zero: a pure stream).
// Build: hipcc -O3 --offload-arch=gfx950 -I include scripts/micro/product_dense.cpp \
//        -L recommendation_gans_amd -lrg_hip -Wl,-rpath,$PWD/recommendation_gans_amd
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rg_hip.h"

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
// the micro's stream over one table (rows x 64 + biases)
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
    *reinterpret_cast<v4f *>(pout + r * 64 + sub * 4) = p;
    *reinterpret_cast<v4f *>(m + r * 64 + sub * 4) = a;
    *reinterpret_cast<v4f *>(v + r * 64 + sub * 4) = b;
    if (sub == 0) { pb = adam(o, pb, 0.0f, mb, vb); bout[r] = pb; bm[r] = mb; bv[r] = vb; }
}

static float *dalloc(size_t n, float scale, unsigned seed) {
    float *p;
    if (hipMalloc(&p, n * 4) != hipSuccess) { fprintf(stderr, "alloc\n"); exit(1); }
    std::vector<float> h(n);
    srand(seed);
    for (auto &x : h) x = ((rand() & 0xffff) - 32768) * (scale / 32768);
    hipMemcpy(p, h.data(), n * 4, hipMemcpyHostToDevice);
    return p;
}

int main() {
    const long U = 136677, I = 20108, R = U + I, D = 64;
    rg_mf_tables_t t[2];
    std::memset(t, 0, sizeof t);
    float *uw[2] = {dalloc(U * D, 1.0f / 64, 1), dalloc(U * D, 1.0f / 64, 1)};
    float *iw[2] = {dalloc(I * D, 1.0f / 64, 2), dalloc(I * D, 1.0f / 64, 2)};
    float *ub[2] = {dalloc(U, 1e-3f, 3), dalloc(U, 1e-3f, 3)};
    float *ib[2] = {dalloc(I, 1e-3f, 4), dalloc(I, 1e-3f, 4)};
    float *um = dalloc(U * D, 1e-6f, 5), *uv = dalloc(U * D, 1e-12f, 6), *im = dalloc(I * D, 1e-6f, 7),
          *iv = dalloc(I * D, 1e-12f, 8);
    float *ubm = dalloc(U, 1e-6f, 9), *ubv = dalloc(U, 1e-12f, 10), *ibm = dalloc(I, 1e-6f, 11),
          *ibv = dalloc(I, 1e-12f, 12);
    hipMemset(uv, 0, U * D * 4); hipMemset(iv, 0, I * D * 4);   // v >= 0
    for (int s = 0; s < 2; ++s) {
        t[s].user_w = uw[s]; t[s].item_w = iw[s]; t[s].user_b = ub[s]; t[s].item_b = ib[s];
        t[s].user_w_out = uw[1 - s]; t[s].item_w_out = iw[1 - s]; t[s].user_b_out = ub[1 - s]; t[s].item_b_out = ib[1 - s];
        t[s].user_w_m = um; t[s].user_w_v = uv; t[s].item_w_m = im; t[s].item_w_v = iv;
        t[s].user_b_m = ubm; t[s].user_b_v = ubv; t[s].item_b_m = ibm; t[s].item_b_v = ibv;
        t[s].num_users = U; t[s].num_items = I; t[s].dim = D;
    }
    rg_mf_work_t w;
    std::memset(&w, 0, sizeof w);
    hipMalloc(&w.row_count, R * 4); hipMemset(w.row_count, 0, R * 4);
    hipMalloc(&w.row_list, R * 8 * 8); hipMemset(w.row_list, 0, R * 64);
    hipMalloc(&w.hot_grad, R * D * 8); hipMemset(w.hot_grad, 0, R * D * 8);
    hipMalloc(&w.hot_bias_grad, R * 8); hipMemset(w.hot_bias_grad, 0, R * 8);
    hipMalloc(&w.loss_partials, 4096 * 4); hipMemset(w.loss_partials, 0, 4096 * 4);
    rg_opt_t o;
    std::memset(&o, 0, sizeof o);
    o.kind = RG_OPT_ADAM; o.lr = 1e-3f; o.beta1 = 0.5f; o.beta2 = 0.999f; o.eps = 1e-8f; o.weight_decay = 1e-5f;
    o.one_minus_beta1 = 0.5f; o.one_minus_beta2 = 0.001f; o.step_size = 2e-3f; o.bias_correction2_sqrt = 0.03f;
    Opt mo{1e-3f, 0.5f, 0.999f, 1e-8f, 1e-5f, 0.5f, 0.001f, 2e-3f, 0.03f};
    hipStream_t st;
    hipStreamCreate(&st);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    auto timeit = [&](const char *what, auto &&fn) {
        for (int k = 0; k < 20; ++k) fn(k);
        hipEventRecord(e0, st);
        const int it = 200;
        for (int k = 0; k < it; ++k) fn(k);
        hipEventRecord(e1, st);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / it;
        printf("%-44s %7.2f us/pass  %.2f TB/s algorithmic\n", what, us, 6.0 * R * 65 * 4 / us / 1e6);
    };
    int rc = 0;
    for (int rep = 0; rep < 2; ++rep) {
        timeit("micro stream (users, then items)", [&](int k) {
            const int s = k & 1;
            hipLaunchKernelGGL(stream, dim3((U * 16 + 255) / 256), dim3(256), 0, st, t[s].user_w, t[s].user_w_out, um, uv,
                               t[s].user_b, t[s].user_b_out, ubm, ubv, U, mo);
            hipLaunchKernelGGL(stream, dim3((I * 16 + 255) / 256), dim3(256), 0, st, t[s].item_w, t[s].item_w_out, im, iv,
                               t[s].item_b, t[s].item_b_out, ibm, ibv, I, mo);
        });
        timeit("product rg_mf_apply (mf_apply_kernel)", [&](int k) {
            rc |= rg_mf_apply(st, &t[k & 1], &w, &o, 0, R, nullptr);
        });
        timeit("product rg_mf_apply_prepare (mf_back_kernel)", [&](int k) {
            rc |= rg_mf_apply_prepare(st, &t[k & 1], &w, &o, 0, R, nullptr, nullptr, nullptr);
        });
    }
    hipError_t err = hipDeviceSynchronize();
    printf("status %s rc %d %s\n", hipGetErrorString(err), rc, rc ? rg_last_error() : "");
    return err == hipSuccess && rc == 0 ? 0 : 1;
}
