// Microbenchmark (scripts only): does an in-place Adam-like pass over p, m, v stay
// resident in the 256 MiB Infinity Cache, vs the ping-pong pass (p read from set A,
// written to set B) the MF dense pass uses?  rows x 65 floats per table, like d = 64.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void pass(const float4 *__restrict__ pin, float4 *__restrict__ pout,
                                            float4 *__restrict__ m, float4 *__restrict__ v, long n4, float lr) {
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    for (; i < n4; i += (long)gridDim.x * 256) {
        float4 p = pin[i], a = m[i], b = v[i];
        a.x = 0.5f * a.x + 0.5f * p.x * 1e-5f; a.y = 0.5f * a.y + 0.5f * p.y * 1e-5f;
        a.z = 0.5f * a.z + 0.5f * p.z * 1e-5f; a.w = 0.5f * a.w + 0.5f * p.w * 1e-5f;
        b.x = 0.999f * b.x + 1e-3f * a.x * a.x; b.y = 0.999f * b.y + 1e-3f * a.y * a.y;
        b.z = 0.999f * b.z + 1e-3f * a.z * a.z; b.w = 0.999f * b.w + 1e-3f * a.w * a.w;
        p.x -= lr * a.x / (sqrtf(b.x) + 1e-8f); p.y -= lr * a.y / (sqrtf(b.y) + 1e-8f);
        p.z -= lr * a.z / (sqrtf(b.z) + 1e-8f); p.w -= lr * a.w / (sqrtf(b.w) + 1e-8f);
        pout[i] = p; m[i] = a; v[i] = b;
    }
}

int main(int argc, char **argv) {
    const long rows = argc > 1 ? atol(argv[1]) : 156785;
    const long n4 = rows * 64 / 4;
    float4 *p[2], *m, *v;
    hipMalloc(&p[0], n4 * 16); hipMalloc(&p[1], n4 * 16); hipMalloc(&m, n4 * 16); hipMalloc(&v, n4 * 16);
    hipMemset(p[0], 0, n4 * 16); hipMemset(p[1], 0, n4 * 16); hipMemset(m, 0, n4 * 16); hipMemset(v, 0, n4 * 16);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int grids[3] = {2048, 4096, (int)((n4 + 255) / 256)};
    for (int gi = 0; gi < 3; ++gi) {
        for (int mode = 0; mode < 2; ++mode) {        // 0 in place, 1 ping-pong
            for (int w = 0; w < 10; ++w) hipLaunchKernelGGL(pass, dim3(grids[gi]), dim3(256), 0, 0, p[0], mode ? p[1] : p[0], m, v, n4, 1e-3f);
            hipEventRecord(a, 0);
            const int it = 50;
            for (int k = 0; k < it; ++k) {
                const int s = mode ? (k & 1) : 0;
                hipLaunchKernelGGL(pass, dim3(grids[gi]), dim3(256), 0, 0, p[s], mode ? p[1 - s] : p[s], m, v, n4, 1e-3f);
            }
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double us = ms * 1e3 / it, bytes = 6.0 * n4 * 16;
            printf("rows %ld grid %d %s: %.2f us/pass, %.2f TB/s (6 x %.1f MB)\n", rows, grids[gi],
                   mode ? "ping-pong" : "in-place", us, bytes / us / 1e6, n4 * 16 / 1e6);
        }
    }
    return 0;
}
