// cGAN training iterations on gfx950 (C4: slate_generation.py, CGANs.py).
//
// One call enqueues a whole discriminator or generator iteration on `stream`:
// the large contractions (D layer 1 over the S*N one-hot / tanh slate columns,
// its input gradient, the S generator heads and their weight gradient) run on
// the fp32 MFMA GEMM of rg_gemm.hip with fused epilogues (tanh, tanh backward +
// bias column sums, LeakyReLU backward, in-place RMSprop/Adam/SGD with the clamp
// and the real slates' sparse gradient rows); the small layers, BatchNorm,
// dropout, the history-embedding sums and their backward are short kernels here.
//
// Reference semantics (file:line in /root/reference):
//   generator.forward      spotlight/dnn_models/cGAN_models.py:41-68
//   discriminator.forward  spotlight/dnn_models/cGAN_models.py:102-109
//   D iteration            CGANs.py:410-457 (clamp +-0.01, D(real one-hot), G(z),
//                          D(fake.detach()), d_loss = mean fake - mean real)
//   G iteration            CGANs.py:370-408 (g_loss = -mean D(G(z)); eval inference
//                          on the same z after the step)
//   one-hot real slates    CGANs.py:181-198 (never materialised: D layer 1 gathers
//                          the S columns of W1 per row, and its weight gradient gets
//                          the real rows as sparse column hits)
#include "rg_gemm.h"

namespace rg {
namespace {

constexpr float kSlope = 0.2f;       // LeakyReLU(0.2) everywhere in cGAN_models.py
constexpr float kClamp = 0.01f;      // CGANs.py:122 weight_cliping_limit
constexpr float kBnEps = 1e-5f;      // BatchNorm1d defaults
constexpr float kBnMomentum = 0.1f;
constexpr float kDropG = 0.1f;       // cGAN_models.py:30
constexpr float kDropD = 0.3f;       // cGAN_models.py:94

int64_t r4(int64_t x) { return (x + 3) / 4 * 4; }
int64_t r64(int64_t x) { return (x + 63) / 64 * 64; }

struct Dims {
    int64_t N, S, H, E, Z, B;
    int64_t H1, H2;    // H/2 (G first hidden, D last hidden), 2H (D first hidden)
    int64_t kz, ks, SN;
    explicit Dims(const rg_gan_dims_t &d)
        : N(d.num_items), S(d.slate_size), H(d.hidden), E(d.emb_dim), Z(d.z_dim), B(d.batch_max) {
        H1 = H / 2;
        H2 = 2 * H;
        SN = S * N;
        kz = r4(Z + E);
        ks = r4(SN);
    }
};

void layout(const Dims &m, int64_t *g, int64_t *d) {
    int64_t o = 0;
    auto put = [&](int64_t *arr, int k, int64_t n) { arr[k] = o; o += r64(n); };
    put(g, RG_GAN_G_WH, m.ks * m.H);      // rows [SN, ks) stay zero
    put(g, RG_GAN_G_BH, m.ks);
    put(g, RG_GAN_G_EMB, (m.N + 1) * m.E);
    put(g, RG_GAN_G_W1, m.H1 * m.kz);
    put(g, RG_GAN_G_B1, m.H1);
    put(g, RG_GAN_G_GAMMA1, m.H1);
    put(g, RG_GAN_G_BETA1, m.H1);
    put(g, RG_GAN_G_W2, m.H * m.H1);
    put(g, RG_GAN_G_B2, m.H);
    put(g, RG_GAN_G_GAMMA2, m.H);
    put(g, RG_GAN_G_BETA2, m.H);
    put(g, RG_GAN_G_RM1, m.H1);
    put(g, RG_GAN_G_RV1, m.H1);
    put(g, RG_GAN_G_RM2, m.H);
    put(g, RG_GAN_G_RV2, m.H);
    g[RG_GAN_G_END] = o;
    o = 0;
    put(d, RG_GAN_D_W1S, m.H2 * m.ks);
    put(d, RG_GAN_D_EMB, (m.N + 1) * m.E);
    put(d, RG_GAN_D_W1E, m.H2 * m.E);
    put(d, RG_GAN_D_B1, m.H2);
    put(d, RG_GAN_D_W2, m.H * m.H2);
    put(d, RG_GAN_D_B2, m.H);
    put(d, RG_GAN_D_W3, m.H1 * m.H);
    put(d, RG_GAN_D_B3, m.H1);
    put(d, RG_GAN_D_W4, m.H1);
    put(d, RG_GAN_D_B4, 1);
    d[RG_GAN_D_END] = o;
}

constexpr int64_t kPartTileSplits = 1024;   // split-K: tiles * splits <= this (partials buffer)

// tiles * splits aimed for: one whole wave of resident workgroups (3 per CU, rg_gemm.hip)
int64_t part_target() { return std::max<int64_t>(64, std::min<int64_t>(kPartTileSplits, 3 * num_cus())); }

// workspace carve-up (floats), sized for batch_max rows (2 * batch_max stacked in D)
struct Ws {
    int64_t cg, cd, a0, y1, yh1, d1, q1g, a1, rs1, y2, yh2, d2, q2g, a2, rs2, fake;
    int64_t h1, u1, q1, h2, u2, q2, h3, u3, q3, dout, dval, part;
    int64_t dl1, dl2, dl3, dc, dlogit, colsum, do2, dy2, do1, dy1, dx0, ggrad, dgrad, amax, scal, total;
    Ws(const Dims &m, const int64_t *g, const int64_t *d) {
        int64_t o = 0;
        auto put = [&](int64_t n) { const int64_t r = o; o += r64(n); return r; };
        const int64_t B = m.B, B2 = 2 * m.B;
        cg = put(B * m.E); cd = put(B * m.E); a0 = put(B * m.kz);
        y1 = put(B * m.H1); yh1 = put(B * m.H1); d1 = put(B * m.H1); q1g = put(B * m.H1); a1 = put(B * m.H1);
        rs1 = put(m.H1);
        y2 = put(B * m.H); yh2 = put(B * m.H); d2 = put(B * m.H); q2g = put(B * m.H); a2 = put(B * m.H);
        rs2 = put(m.H);
        fake = put(B * m.ks);
        h1 = put(B2 * m.H2); u1 = put(B2 * m.H2); q1 = put(B2 * m.H2);
        h2 = put(B2 * m.H); u2 = put(B2 * m.H); q2 = put(B2 * m.H);
        h3 = put(B2 * m.H1); u3 = put(B2 * m.H1); q3 = put(B2 * m.H1);
        dout = put(B2); dval = put(B2);
        part = put(kPartTileSplits * kGemmBM * kGemmBN);
        dl1 = put(B2 * m.H2); dl2 = put(B2 * m.H); dl3 = put(B2 * m.H1); dc = put(B * m.E);
        dlogit = put(B * m.ks); colsum = put(gemm_tiles_m(B) * m.ks);
        do2 = put(B * m.H); dy2 = put(B * m.H); do1 = put(B * m.H1); dy1 = put(B * m.H1); dx0 = put(B * m.kz);
        ggrad = put(g[RG_GAN_G_RM1] - g[RG_GAN_G_BH]);
        dgrad = put(d[RG_GAN_D_END] - d[RG_GAN_D_EMB]);
        amax = put(B * gemm_tiles_n(m.SN) * 4);
        scal = put(16);
        total = o;
    }
};

// ------------------------------------------------------------------ dropout
struct Drop {
    const uint8_t *mask;   // [rows][width] or null
    int64_t width;
    uint64_t seed;
    uint32_t salt, thr;    // hash keeps when >= thr (= p * 2^32)
    float scale;           // 1 / (1 - p), the value torch's noise.div_(1 - p) holds
    int train;
};

__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

__device__ __forceinline__ float drop_mult(const Drop &q, int64_t row, int64_t unit) {
    if (!q.train) return 1.0f;
    if (q.mask) return q.mask[row * q.width + unit] ? q.scale : 0.0f;
    const uint64_t k = splitmix(q.seed ^ ((uint64_t)q.salt << 56) ^ ((uint64_t)row << 24) ^ (uint64_t)unit);
    return (uint32_t)(k >> 32) >= q.thr ? q.scale : 0.0f;
}

__device__ __forceinline__ float lrelu(float x) { return x > 0.0f ? x : x * kSlope; }

// ------------------------------------------------------------------ kernels
constexpr int kEChunk = 8;   // embedding columns accumulated per pass

// fixed-order tree over a block's 256 partials in LDS (all threads call it)
__device__ __forceinline__ float block_sum256(float v, float *red) {
    const int t = threadIdx.x;
    red[t] = v;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w) red[t] += red[t + w];
        __syncthreads();
    }
    const float r = red[0];
    __syncthreads();
    return r;
}

// emb(hist).sum(1): one block per row, threads over history slots, fixed-order tree
__global__ __launch_bounds__(256) void hist_sum_kernel(const float *__restrict__ emb, const int32_t *__restrict__ hist,
                                                       int L, int rows, int E, int pad, float *__restrict__ out) {
    __shared__ float red[256];
    const int row = blockIdx.x, t = threadIdx.x;
    for (int e0 = 0; e0 < E; e0 += kEChunk) {
        float acc[kEChunk];
#pragma unroll
        for (int e = 0; e < kEChunk; ++e) acc[e] = 0.0f;
        // the thread's positions t, t + 256, ... in order; ids and rows of kB positions in flight
        constexpr int kB = 4;
        for (int l0 = t; l0 < L; l0 += 256 * kB) {
            int it[kB];
#pragma unroll
            for (int u = 0; u < kB; ++u) it[u] = l0 + 256 * u < L ? hist[(int64_t)row * L + l0 + 256 * u] : pad;
            float x[kB][kEChunk];
#pragma unroll
            for (int u = 0; u < kB; ++u)
#pragma unroll
                for (int e = 0; e < kEChunk; ++e)
                    x[u][e] = (it[u] != pad && e0 + e < E) ? emb[(int64_t)it[u] * E + e0 + e] : 0.0f;
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                if (it[u] == pad) continue;
#pragma unroll
                for (int e = 0; e < kEChunk; ++e)
                    if (e0 + e < E) acc[e] += x[u][e];
            }
        }
#pragma unroll
        for (int e = 0; e < kEChunk; ++e) {
            if (e0 + e >= E) break;
            const float v = block_sum256(acc[e], red);
            if (t == 0) out[(int64_t)row * E + e0 + e] = v;
        }
    }
}

// a0 = LeakyReLU(cat([z, e])) (cGAN_models.py:44-47), zero pad to kz
__global__ __launch_bounds__(256) void g_input_kernel(const float *__restrict__ z, int Z, const float *__restrict__ c,
                                                      int E, int rows, int kz, float *__restrict__ a0) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= (int64_t)rows * kz) return;
    const int64_t b = e / kz;
    const int k = (int)(e % kz);
    const float x = k < Z ? z[b * Z + k] : (k < Z + E ? c[b * E + (k - Z)] : 0.0f);
    a0[e] = lrelu(x);
}

// BatchNorm1d (batch stats in train mode, running stats in eval) -> Dropout -> LeakyReLU,
// one block per channel (cGAN_models.py:28-31)
__global__ __launch_bounds__(256) void bn_fwd_kernel(const float *__restrict__ y, int rows, int C,
                                                     const float *__restrict__ gamma, const float *__restrict__ beta,
                                                     float *__restrict__ rm, float *__restrict__ rv, Drop q,
                                                     float *__restrict__ yhat, float *__restrict__ dmul,
                                                     float *__restrict__ qout, float *__restrict__ a,
                                                     float *__restrict__ rstd_out) {
    __shared__ float red[256];
    const int c = blockIdx.x, t = threadIdx.x;
    float mean, rstd;
    if (q.train) {
        float s = 0.0f;
        for (int r = t; r < rows; r += 256) s += y[(int64_t)r * C + c];
        red[t] = s;
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if (t < w) red[t] += red[t + w];
            __syncthreads();
        }
        mean = red[0] / (float)rows;
        __syncthreads();
        float v = 0.0f;
        for (int r = t; r < rows; r += 256) {
            const float dd = y[(int64_t)r * C + c] - mean;
            v = fmaf(dd, dd, v);
        }
        red[t] = v;
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if (t < w) red[t] += red[t + w];
            __syncthreads();
        }
        const float var_sum = red[0];
        rstd = 1.0f / sqrtf(var_sum / (float)rows + kBnEps);
        if (t == 0) {
            rm[c] = (1.0f - kBnMomentum) * rm[c] + kBnMomentum * mean;
            rv[c] = (1.0f - kBnMomentum) * rv[c] + kBnMomentum * (var_sum / (float)(rows - 1));
            rstd_out[c] = rstd;
        }
    } else {
        mean = rm[c];
        rstd = 1.0f / sqrtf(rv[c] + kBnEps);
    }
    const float g = gamma[c], bb = beta[c];
    for (int r = t; r < rows; r += 256) {
        const int64_t e = (int64_t)r * C + c;
        const float yh = (y[e] - mean) * rstd;
        const float mult = drop_mult(q, r, c);
        const float dv = fmaf(yh, g, bb) * mult;
        if (yhat) yhat[e] = yh;
        if (dmul) dmul[e] = dv;
        if (qout) qout[e] = mult;
        a[e] = lrelu(dv);
    }
}

// D layer 1 on the real slates: the one-hot row selects S columns of W1
// (clamped, as CGANs.py:438-439 leaves them for this pass) -> Dropout -> LeakyReLU
__global__ __launch_bounds__(256) void d_real_l1_kernel(const float *__restrict__ w1s, int64_t ks,
                                                        const float *__restrict__ w1e, const float *__restrict__ b1,
                                                        const float *__restrict__ c, int E,
                                                        const int32_t *__restrict__ slates, int S, int64_t N,
                                                        int rows, int H2, Drop q, float *__restrict__ u,
                                                        float *__restrict__ h, float *__restrict__ qo) {
    const int b = blockIdx.x;
    if (b >= rows) return;
    for (int un = threadIdx.x; un < H2; un += 256) {
        float v = 0.0f;
        for (int e = 0; e < E; ++e) v = fmaf(w1e[(int64_t)un * E + e], c[(int64_t)b * E + e], v);
        for (int s = 0; s < S; ++s) {
            const float w = w1s[(int64_t)un * ks + s * N + slates[(int64_t)b * S + s]];
            v += fminf(fmaxf(w, -kClamp), kClamp);
        }
        v += b1[un];
        const float mult = drop_mult(q, b, un);
        const float uu = v * mult;
        const int64_t o = (int64_t)b * H2 + un;
        u[o] = uu;
        h[o] = lrelu(uu);
        qo[o] = mult;
    }
}

// split-K reduction + bias (+ history-embedding columns of W1) -> Dropout -> LeakyReLU
// sum over split-K partials in split order (part[z * stride + e], z = 0..splits-1), the
// loads issued kSplitBatch at a time ahead of the in-order adds: the same sums as the
// plain loop, with kSplitBatch loads in flight per thread instead of the compiler's few
constexpr int kSplitBatch = 16;
__device__ __forceinline__ float sum_splits(const float *__restrict__ part, int splits, int64_t stride, int64_t e) {
    float v = 0.0f;
    int z = 0;
    for (; z + kSplitBatch <= splits; z += kSplitBatch) {
        float x[kSplitBatch];
#pragma unroll
        for (int u = 0; u < kSplitBatch; ++u) x[u] = part[(int64_t)(z + u) * stride + e];
#pragma unroll
        for (int u = 0; u < kSplitBatch; ++u) v += x[u];
    }
    for (; z < splits; ++z) v += part[(int64_t)z * stride + e];
    return v;
}

__global__ __launch_bounds__(256) void reduce_act_kernel(const float *__restrict__ part, int splits, int64_t zstride,
                                                         int rows, int C,
                                                         const float *__restrict__ bias,
                                                         const float *__restrict__ c, const float *__restrict__ we,
                                                         int E, Drop q, float *__restrict__ u,
                                                         float *__restrict__ h, float *__restrict__ qo) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t total = (int64_t)rows * C;
    if (e >= total) return;
    const int64_t r = e / C;
    const int un = (int)(e % C);
    float v = sum_splits(part, splits, zstride, e);
    if (we)
        for (int k = 0; k < E; ++k) v = fmaf(we[(int64_t)un * E + k], c[r * E + k], v);
    v += bias[un];
    const float mult = drop_mult(q, r, un);
    const float uu = v * mult;
    u[e] = uu;
    h[e] = lrelu(uu);
    qo[e] = mult;
}

// split-K reduction, then * LeakyReLU'(U) * Mult (backward through Dropout + LeakyReLU)
__global__ __launch_bounds__(256) void reduce_lrelu_grad_kernel(const float *__restrict__ part, int splits,
                                                                int64_t total, const float *__restrict__ U,
                                                                const float *__restrict__ Mult,
                                                                float *__restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= total) return;
    float v = sum_splits(part, splits, total, e);
    v = v * (U[e] > 0.0f ? 1.0f : kSlope);
    if (Mult) v = v * Mult[e];
    out[e] = v;
}

// last D layer Linear(H/2 -> 1): one wave per row
__global__ __launch_bounds__(256) void d_out_kernel(const float *__restrict__ h3, int rows, int K,
                                                    const float *__restrict__ w4, const float *__restrict__ b4,
                                                    float *__restrict__ out) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= rows) return;
    float s = 0.0f;
    for (int k = lane; k < K; k += 64) s = fmaf(h3[(int64_t)row * K + k], w4[k], s);
    s = group_sum<64>(s);
    if (lane == 0) out[row] = s + b4[0];
}

// losses and dL/dout.  D step (rows = 2B stacked): d_loss = mean(fake) - mean(real),
// dout = -1/B on real rows, +1/B on fake rows.  G step: g_loss = -mean, dout = -1/B.
__global__ __launch_bounds__(256) void d_loss_kernel(const float *__restrict__ dval, int B, int d_step,
                                                     float *__restrict__ dout, float *__restrict__ out) {
    __shared__ double red[2][256];
    const int t = threadIdx.x;
    double sr = 0.0, sf = 0.0;
    for (int r = t; r < B; r += 256) {
        if (d_step) {
            sr += dval[r];
            sf += dval[B + r];
        } else {
            sf += dval[r];
        }
    }
    red[0][t] = sr;
    red[1][t] = sf;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w) {
            red[0][t] += red[0][t + w];
            red[1][t] += red[1][t + w];
        }
        __syncthreads();
    }
    const float inv = 1.0f / (float)B;
    for (int r = t; r < (d_step ? 2 * B : B); r += 256) dout[r] = d_step ? (r < B ? -inv : inv) : -inv;
    if (t == 0) {
        const float mr = (float)(red[0][0] / B), mf = (float)(red[1][0] / B);
        if (d_step) {
            out[0] = mf - mr;
            out[1] = mr;
            out[2] = mf;
        } else {
            out[0] = -mf;
        }
    }
}

// backward of the last D layer, elementwise: dl3 = dout * w4 * LeakyReLU'(u3) * mult3
// (dW4 / db4 are weighted column sums: colsum_kernel)
__global__ __launch_bounds__(256) void d_out_bwd_kernel(const float *__restrict__ u3, const float *__restrict__ q3,
                                                        const float *__restrict__ dout, int rows, int K,
                                                        const float *__restrict__ w4, float *__restrict__ dl3) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= (int64_t)rows * K) return;
    const int k = (int)(e % K);
    const float v = dout[e / K] * w4[k];
    dl3[e] = v * (u3[e] > 0.0f ? 1.0f : kSlope) * q3[e];
}

// split-K reduction + bias + post op (small GEMMs split for parallelism)
__global__ __launch_bounds__(256) void reduce_post_kernel(const float *__restrict__ part, int splits, int64_t M,
                                                          int64_t N, float *__restrict__ C, int64_t ldc,
                                                          const float *__restrict__ bias, int post,
                                                          const float *__restrict__ T, int64_t ldt,
                                                          const float *__restrict__ Mult) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= M * N) return;
    const int64_t m = e / N, n = e % N;
    float v = sum_splits(part, splits, M * N, e);
    if (bias) v += bias[n];
    if (post == kPostTanh) {
        v = tanhf(v);
    } else if (post == kPostLreluGrad) {
        v = v * (T[m * ldt + n] > 0.0f ? 1.0f : kSlope);
        if (Mult) v = v * Mult[m * ldt + n];
    }
    C[m * ldc + n] = v;
}

// out[c] = sum_r w[r] X[r][c] (w null: 1; X null: a column of ones), 64 columns per
// block, 16 waves over interleaved rows, combined in wave order (deterministic)
__global__ __launch_bounds__(1024) void colsum_kernel(const float *__restrict__ X, int64_t rows, int64_t C,
                                                      int64_t ld, const float *__restrict__ w,
                                                      float *__restrict__ out) {
    __shared__ float red[16][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t c = (int64_t)blockIdx.x * 64 + lane;
    float s = 0.0f;
    if (c < C) {
        // the wave's rows wave, wave + 16, ... in order; their loads issued kB at a time
        constexpr int kB = 8;
        for (int64_t r0 = wave; r0 < rows; r0 += 16 * kB) {
            float x[kB], wr[kB];
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int64_t r = r0 + 16 * u;
                x[u] = (X && r < rows) ? X[r * ld + c] : 1.0f;
                wr[u] = (w && r < rows) ? w[r] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < kB; ++u)
                if (r0 + 16 * u < rows) s = w ? fmaf(wr[u], x[u], s) : s + x[u];
        }
    }
    red[wave][lane] = s;
    __syncthreads();
    if (wave == 0 && c < C) {
        float v = red[0][lane];
        for (int k = 1; k < 16; ++k) v += red[k][lane];
        out[c] = v;
    }
}

// D layer 1, history columns: dW1e[u][e] = sum_r dl1[r][u] c[r mod B][e] over the 2B
// stacked rows (real, then fake); 64 units per block, 16 waves over rows
__global__ __launch_bounds__(1024) void d_l1_w1e_grad_kernel(const float *__restrict__ dl1, int B, int H2,
                                                             const float *__restrict__ c, int E,
                                                             float *__restrict__ gw1e) {
    __shared__ float red[16][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int un = blockIdx.x * 64 + lane;
    for (int e0 = 0; e0 < E; e0 += kEChunk) {
        float acc[kEChunk];
#pragma unroll
        for (int e = 0; e < kEChunk; ++e) acc[e] = 0.0f;
        if (un < H2) {
            constexpr int kB = 4;   // rows whose loads are issued together (same fma order)
            for (int r0 = wave; r0 < 2 * B; r0 += 16 * kB) {
                float g[kB], cv[kB][kEChunk];
#pragma unroll
                for (int u = 0; u < kB; ++u) {
                    const int r = r0 + 16 * u;
                    const bool ok = r < 2 * B;
                    g[u] = ok ? dl1[(int64_t)r * H2 + un] : 0.0f;
                    const float *cr = c + (int64_t)((ok ? r : 0) % B) * E + e0;
#pragma unroll
                    for (int e = 0; e < kEChunk; ++e) cv[u][e] = (e0 + e < E) ? cr[e] : 0.0f;
                }
#pragma unroll
                for (int u = 0; u < kB; ++u) {
                    if (r0 + 16 * u >= 2 * B) continue;
#pragma unroll
                    for (int e = 0; e < kEChunk; ++e)
                        if (e0 + e < E) acc[e] = fmaf(g[u], cv[u][e], acc[e]);
                }
            }
        }
#pragma unroll
        for (int e = 0; e < kEChunk; ++e) {
            if (e0 + e >= E) break;
            red[wave][lane] = acc[e];
            __syncthreads();
            if (wave == 0 && un < H2) {
                float v = red[0][lane];
                for (int k = 1; k < 16; ++k) v += red[k][lane];
                gw1e[(int64_t)un * E + e0 + e] = v;
            }
            __syncthreads();
        }
    }
}

// dc[b][e] = dl1_real[b] . W1e[:, e] + dl1_fake[b] . W1e[:, e] (each pass its own sum, as
// autograd accumulates the two embedding lookups); one block per row
__global__ __launch_bounds__(256) void d_l1_dc_kernel(const float *__restrict__ dl1, int B, int H2, int E,
                                                      const float *__restrict__ w1e, float *__restrict__ dc) {
    __shared__ float red[256];
    const int b = blockIdx.x, t = threadIdx.x;
    for (int e0 = 0; e0 < E; e0 += kEChunk) {
        float ar[kEChunk], af[kEChunk];
#pragma unroll
        for (int e = 0; e < kEChunk; ++e) ar[e] = af[e] = 0.0f;
        for (int un = t; un < H2; un += 256) {
            const float gr = dl1[(int64_t)b * H2 + un], gf = dl1[(int64_t)(B + b) * H2 + un];
#pragma unroll
            for (int e = 0; e < kEChunk; ++e)
                if (e0 + e < E) {
                    const float w = w1e[(int64_t)un * E + e0 + e];
                    ar[e] = fmaf(gr, w, ar[e]);
                    af[e] = fmaf(gf, w, af[e]);
                }
        }
#pragma unroll
        for (int e = 0; e < kEChunk; ++e) {
            if (e0 + e >= E) break;
            const float sr = block_sum256(ar[e], red);
            const float sf = block_sum256(af[e], red);
            if (t == 0) dc[(int64_t)b * E + e0 + e] = sr + sf;
        }
    }
}

// embedding backward with padding_idx: grad[item] = sum over the batch rows whose
// history holds it (grouped host-side) of src[row]; one wave per item, lanes over its
// rows, fixed-order DPP tree
__global__ __launch_bounds__(256) void emb_grad_kernel(const int32_t *__restrict__ items,
                                                       const int32_t *__restrict__ off,
                                                       const int32_t *__restrict__ brow, int n_items,
                                                       const float *__restrict__ src, int64_t src_ld, int E,
                                                       float *__restrict__ grad) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (i >= n_items) return;
    const int j0 = off[i], j1 = off[i + 1];
    for (int e0 = 0; e0 < E; e0 += kEChunk) {
        float acc[kEChunk];
#pragma unroll
        for (int e = 0; e < kEChunk; ++e) acc[e] = 0.0f;
        for (int j = j0 + lane; j < j1; j += 64) {
            const float *sr = src + (int64_t)brow[j] * src_ld + e0;
#pragma unroll
            for (int e = 0; e < kEChunk; ++e)
                if (e0 + e < E) acc[e] += sr[e];
        }
#pragma unroll
        for (int e = 0; e < kEChunk; ++e) {
            if (e0 + e >= E) break;
            const float v = group_sum<64>(acc[e]);
            if (lane == 0) grad[(int64_t)items[i] * E + e0 + e] = v;
        }
    }
}

// BatchNorm backward per channel (train mode): do = dL/d(gamma*yhat+beta) after the
// dropout multiplier; dgamma, dbeta, dy = rstd (do*g - mean(do*g) - yhat mean(do*g*yhat))
__global__ __launch_bounds__(256) void bn_bwd_kernel(const float *__restrict__ dO, const float *__restrict__ yhat,
                                                     const float *__restrict__ rstd, const float *__restrict__ gamma,
                                                     int rows, int C, float *__restrict__ gg, float *__restrict__ gb,
                                                     float *__restrict__ dy) {
    __shared__ float red[3][256];
    const int c = blockIdx.x, t = threadIdx.x;
    float s0 = 0.0f, s1 = 0.0f;
    for (int r = t; r < rows; r += 256) {
        const int64_t e = (int64_t)r * C + c;
        s0 += dO[e];
        s1 = fmaf(dO[e], yhat[e], s1);
    }
    red[0][t] = s0;
    red[1][t] = s1;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w) {
            red[0][t] += red[0][t + w];
            red[1][t] += red[1][t + w];
        }
        __syncthreads();
    }
    const float sum_do = red[0][0], sum_doy = red[1][0];
    const float g = gamma[c], rs = rstd[c];
    if (t == 0) {
        gg[c] = sum_doy;
        gb[c] = sum_do;
    }
    const float inv = 1.0f / (float)rows;
    const float mean_dyh = sum_do * g * inv, mean_dyhy = sum_doy * g * inv;
    for (int r = t; r < rows; r += 256) {
        const int64_t e = (int64_t)r * C + c;
        dy[e] = rs * (dO[e] * g - mean_dyh - yhat[e] * mean_dyhy);
    }
}

// out[n] = sum_t rows[t][n] (tile partials in order)
__global__ __launch_bounds__(256) void sum_rows_kernel(const float *__restrict__ x, int nrows, int64_t N,
                                                       int64_t ld, float *__restrict__ out) {
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (n >= N) return;
    float s = 0.0f;
    for (int r = 0; r < nrows; ++r) s += x[(int64_t)r * ld + n];
    out[n] = s;
}

__global__ __launch_bounds__(256) void copy_cols_kernel(const float *__restrict__ x, int64_t ld, int64_t off,
                                                        int rows, int E, float *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)rows * E) return;
    out[t] = x[(t / E) * ld + off + t % E];
}

__global__ __launch_bounds__(256) void clamp_kernel(float *__restrict__ p, int64_t n, float c) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e < n) p[e] = fminf(fmaxf(p[e], -c), c);
}

__global__ __launch_bounds__(256) void opt_flat_kernel(float *__restrict__ p, const float *__restrict__ g,
                                                       float *__restrict__ m, float *__restrict__ v, int64_t n,
                                                       rg_opt_t opt) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n) return;
    float mm = m ? m[e] : 0.0f, vv = v ? v[e] : 0.0f;
    p[e] = opt_update(opt, p[e], g[e], mm, vv);
    if (m) m[e] = mm;
    if (v) v[e] = vv;
}

// per (row, head): best (value, index) over the column tiles overlapping the head
// (first maximum, as torch.max): one wave per (row, head), lanes over tiles
__global__ __launch_bounds__(256) void argmax_final_kernel(const float2 *__restrict__ amax, int rows, int64_t ntile,
                                                           int S, int64_t N, float *__restrict__ slates) {
    const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= (int64_t)rows * S) return;
    const int64_t m = t / S;
    const int s = (int)(t % S);
    const int64_t c0 = (int64_t)s * N, c1 = c0 + N;
    const int64_t t0 = c0 / kGemmBN, t1 = std::min<int64_t>((c1 + kGemmBN - 1) / kGemmBN, ntile);
    float bv = -INFINITY, bi = INFINITY;
    for (int64_t tile = t0 + lane; tile < t1; tile += 64) {
        const int seg = (int)(s - tile * kGemmBN / N);
        if (seg < 0 || seg > 1) continue;
        const float2 o = amax[(m * ntile + tile) * 2 + seg];
        if (o.x > bv || (o.x == bv && o.y < bi)) { bv = o.x; bi = o.y; }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const float ov = __shfl_xor(bv, off), oi = __shfl_xor(bi, off);
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) slates[t] = bi;
}

// per (row, head): first maximum of the tanh outputs T[row][s*N .. (s+1)*N) (heads
// narrower than a GEMM column tile)
__global__ __launch_bounds__(256) void argmax_rows_kernel(const float *__restrict__ T, int64_t ld, int rows, int S,
                                                          int64_t N, float *__restrict__ slates) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)rows * S) return;
    const int64_t m = t / S;
    const int s = (int)(t % S);
    const float *row = T + m * ld + (int64_t)s * N;
    float bv = row[0];
    int64_t bi = 0;
    for (int64_t n = 1; n < N; ++n)
        if (row[n] > bv) { bv = row[n]; bi = n; }
    slates[t] = (float)bi;
}

unsigned blocks(int64_t n) { return (unsigned)((n + 255) / 256); }

void colsum(hipStream_t st, const float *X, int64_t rows, int64_t C, int64_t ld, const float *w, float *out) {
    hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)((C + 63) / 64)), dim3(1024), 0, st, X, rows, C, ld, w, out);
}

void hist_sum(hipStream_t st, const float *emb, const rg_gan_batch_t *bt, int rows, int E, int pad, float *out) {
    hipLaunchKernelGGL(hist_sum_kernel, dim3(rows), dim3(256), 0, st, emb, bt->hist, bt->hist_len, rows, E, pad, out);
}

void emb_grad(hipStream_t st, const rg_gan_batch_t *bt, const float *src, int64_t ld, int E, float *grad) {
    if (bt->n_hist_items <= 0) return;
    hipLaunchKernelGGL(emb_grad_kernel, dim3((unsigned)((bt->n_hist_items + 3) / 4)), dim3(256), 0, st,
                       bt->hist_items, bt->hist_off, bt->hist_rows, bt->n_hist_items, src, ld, E, grad);
}

// a GEMM with few output tiles (the small layers): split K over more workgroups and
// reduce in split order with the same bias / post op
int gemm_small(hipStream_t st, GemmDesc d, float *part) {
    const int64_t tiles = gemm_tiles_m(d.M) * gemm_tiles_n(d.N);
    int splits = (int)std::min<int64_t>(std::max<int64_t>(1, 64 / tiles), std::max<int64_t>(1, d.K / 64));
    if (d.epi != kEpiStore || d.post == kPostTanhGrad || splits <= 1) return gemm(st, d);
    GemmDesc p = d;
    p.epi = kEpiPartial;
    p.splits = splits;
    p.C = part;
    p.bias = nullptr;
    p.post = kPostNone;
    const int rc = gemm(st, p);
    if (rc) return rc;
    hipLaunchKernelGGL(reduce_post_kernel, dim3(blocks(d.M * d.N)), dim3(256), 0, st, part, splits, d.M, d.N, d.C,
                       d.ldc, d.bias, d.post, d.T, d.ldt, d.Mult);
    return check_launch("reduce_post_kernel");
}

int pick_splits(int64_t M, int64_t N, int64_t K) {
    const int64_t tiles = gemm_tiles_m(M) * gemm_tiles_n(N);
    int64_t s = part_target() / tiles;
    s = std::min<int64_t>(s, std::max<int64_t>(1, K / 256));
    return (int)std::max<int64_t>(1, s);
}

Drop make_drop(const rg_gan_noise_t *nz, int slot, int64_t width, float p, uint64_t salt_base) {
    Drop q{};
    q.mask = nz ? nz->masks[slot] : nullptr;
    q.width = width;
    q.seed = nz ? nz->seed : 0;
    q.salt = (uint32_t)(salt_base + slot);
    q.thr = (uint32_t)((double)p * 4294967296.0);
    q.scale = (float)(1.0 / (1.0 - (double)p));
    q.train = 1;
    return q;
}

struct Ctx {
    hipStream_t st;
    Dims m;
    const int64_t *go, *dof;
    const Ws &w;
    char *base;
    float *f(int64_t off) const { return reinterpret_cast<float *>(base) + off; }
};

#define RG_TRY(x)                  \
    do {                           \
        const int rc_ = (x);       \
        if (rc_) return rc_;       \
    } while (0)

// generator forward (train: batch-stat BN, dropout slots slot0 / slot0 + 1; eval:
// running stats, no dropout) -> a2 [rows][H]
int g_forward(const Ctx &x, const rg_gan_model_t *mdl, const rg_gan_batch_t *bt, const float *z,
              const rg_gan_noise_t *nz, int slot0, bool train, bool update_stats) {
    const Dims &m = x.m;
    const int rows = bt->rows;
    float *G = mdl->g;
    hist_sum(x.st, G + x.go[RG_GAN_G_EMB], bt, rows, (int)m.E, (int)m.N, x.f(x.w.cg));
    hipLaunchKernelGGL(g_input_kernel, dim3(blocks((int64_t)rows * m.kz)), dim3(256), 0, x.st, z, (int)m.Z,
                       x.f(x.w.cg), (int)m.E, rows, (int)m.kz, x.f(x.w.a0));
    // layer 1
    GemmDesc d;
    d.A = x.f(x.w.a0); d.lda = m.kz;
    d.B = G + x.go[RG_GAN_G_W1]; d.ldb = m.kz;
    d.M = rows; d.N = m.H1; d.K = m.kz;
    d.C = x.f(x.w.y1); d.ldc = m.H1; d.bias = G + x.go[RG_GAN_G_B1];
    RG_TRY(gemm_small(x.st, d, x.f(x.w.part)));
    Drop q1 = make_drop(nz, slot0, m.H1, kDropG, 0);
    q1.train = train ? 1 : 0;
    // running stats: eval reads them; train updates them (the reference's every train-mode forward)
    float *rm1 = G + x.go[RG_GAN_G_RM1], *rv1 = G + x.go[RG_GAN_G_RV1];
    (void)update_stats;
    hipLaunchKernelGGL(bn_fwd_kernel, dim3((unsigned)m.H1), dim3(256), 0, x.st, x.f(x.w.y1), rows, (int)m.H1,
                       G + x.go[RG_GAN_G_GAMMA1], G + x.go[RG_GAN_G_BETA1], rm1, rv1, q1, x.f(x.w.yh1),
                       x.f(x.w.d1), x.f(x.w.q1g), x.f(x.w.a1), x.f(x.w.rs1));
    // layer 2
    d = GemmDesc();
    d.A = x.f(x.w.a1); d.lda = m.H1;
    d.B = G + x.go[RG_GAN_G_W2]; d.ldb = m.H1;
    d.M = rows; d.N = m.H; d.K = m.H1;
    d.C = x.f(x.w.y2); d.ldc = m.H; d.bias = G + x.go[RG_GAN_G_B2];
    RG_TRY(gemm_small(x.st, d, x.f(x.w.part)));
    Drop q2 = make_drop(nz, slot0 + 1, m.H, kDropG, 0);
    q2.train = train ? 1 : 0;
    hipLaunchKernelGGL(bn_fwd_kernel, dim3((unsigned)m.H), dim3(256), 0, x.st, x.f(x.w.y2), rows, (int)m.H,
                       G + x.go[RG_GAN_G_GAMMA2], G + x.go[RG_GAN_G_BETA2], G + x.go[RG_GAN_G_RM2],
                       G + x.go[RG_GAN_G_RV2], q2, x.f(x.w.yh2), x.f(x.w.d2), x.f(x.w.q2g), x.f(x.w.a2),
                       x.f(x.w.rs2));
    return check_launch("g_forward");
}

// heads: fake = tanh(a2 WH^T + bh) [rows][ks]
int g_heads(const Ctx &x, const rg_gan_model_t *mdl, int rows) {
    const Dims &m = x.m;
    GemmDesc d;
    d.A = x.f(x.w.a2); d.lda = m.H;
    d.B = mdl->g + x.go[RG_GAN_G_WH]; d.ldb = m.H;
    d.M = rows; d.N = m.SN; d.K = m.H;
    d.C = x.f(x.w.fake); d.ldc = m.ks; d.bias = mdl->g + x.go[RG_GAN_G_BH]; d.post = kPostTanh;
    return gemm(x.st, d);
}

// D layers 2..4 on `rows` stacked rows (h1 given) -> dval; dropout slots slot0 + 1, + 2
// for the row ranges [0, B) / [B, 2B) given by drop0 / drop1 salts
int d_upper_forward(const Ctx &x, const rg_gan_model_t *mdl, int rows, const Drop *qs2, const Drop *qs3,
                    int n_pass, int B) {
    const Dims &m = x.m;
    float *D = mdl->d;
    const int64_t in[2] = {m.H2, m.H}, out[2] = {m.H, m.H1};
    const int64_t wblk[2] = {RG_GAN_D_W2, RG_GAN_D_W3}, bblk[2] = {RG_GAN_D_B2, RG_GAN_D_B3};
    const int64_t hin[2] = {x.w.h1, x.w.h2}, hout[2] = {x.w.h2, x.w.h3}, uout[2] = {x.w.u2, x.w.u3},
                  qout[2] = {x.w.q2, x.w.q3};
    for (int k = 0; k < 2; ++k) {
        GemmDesc d;
        d.A = x.f(hin[k]); d.lda = in[k];
        d.B = D + x.dof[wblk[k]]; d.ldb = in[k];
        d.M = rows; d.N = out[k]; d.K = in[k];
        const int64_t tiles = gemm_tiles_m(rows) * gemm_tiles_n(out[k]);
        d.epi = kEpiPartial; d.C = x.f(x.w.part);
        d.splits = (int)std::min<int64_t>(std::max<int64_t>(1, 64 / tiles), std::max<int64_t>(1, in[k] / 64));
        RG_TRY(gemm_small(x.st, d, x.f(x.w.part)));
        // per pass (real / fake rows have their own dropout draws)
        for (int p = 0; p < n_pass; ++p) {
            const Drop &q = k == 0 ? qs2[p] : qs3[p];
            const int64_t r0 = (int64_t)p * B;
            hipLaunchKernelGGL(reduce_act_kernel, dim3(blocks((int64_t)B * out[k])), dim3(256), 0, x.st,
                               x.f(x.w.part) + r0 * out[k], d.splits, (int64_t)rows * out[k], B, (int)out[k],
                               D + x.dof[bblk[k]], nullptr, nullptr, 0, q, x.f(uout[k]) + r0 * out[k],
                               x.f(hout[k]) + r0 * out[k], x.f(qout[k]) + r0 * out[k]);
        }
    }
    hipLaunchKernelGGL(d_out_kernel, dim3((rows + 3) / 4), dim3(256), 0, x.st, x.f(x.w.h3), rows, (int)m.H1,
                       D + x.dof[RG_GAN_D_W4], D + x.dof[RG_GAN_D_B4], x.f(x.w.dval));
    return check_launch("d_upper_forward");
}

// backward through D layers 4..2 -> dl1 [rows][2H]; param grads into dgrad when given
int d_upper_backward(const Ctx &x, const rg_gan_model_t *mdl, int rows, float *dgrad) {
    const Dims &m = x.m;
    float *D = mdl->d;
    auto gslot = [&](int blk) { return dgrad ? dgrad + (x.dof[blk] - x.dof[RG_GAN_D_EMB]) : nullptr; };
    hipLaunchKernelGGL(d_out_bwd_kernel, dim3(blocks((int64_t)rows * m.H1)), dim3(256), 0, x.st, x.f(x.w.u3),
                       x.f(x.w.q3), x.f(x.w.dout), rows, (int)m.H1, D + x.dof[RG_GAN_D_W4], x.f(x.w.dl3));
    if (dgrad) {
        colsum(x.st, x.f(x.w.h3), rows, m.H1, m.H1, x.f(x.w.dout), gslot(RG_GAN_D_W4));
        colsum(x.st, nullptr, rows, 1, 1, x.f(x.w.dout), gslot(RG_GAN_D_B4));
    }
    const int64_t in[2] = {m.H, m.H2}, out[2] = {m.H1, m.H};      // layer 3 then layer 2
    const int64_t wblk[2] = {RG_GAN_D_W3, RG_GAN_D_W2}, bblk[2] = {RG_GAN_D_B3, RG_GAN_D_B2};
    const int64_t dl[2] = {x.w.dl3, x.w.dl2}, dlin[2] = {x.w.dl2, x.w.dl1}, hin[2] = {x.w.h2, x.w.h1},
                  uin[2] = {x.w.u2, x.w.u1}, qin[2] = {x.w.q2, x.w.q1};
    for (int k = 0; k < 2; ++k) {
        if (dgrad) {
            // dW = dl^T h_in: [out][in], reduction over rows
            GemmDesc d;
            d.A = x.f(dl[k]); d.lda = out[k]; d.a_kmajor = false;
            d.B = x.f(hin[k]); d.ldb = in[k]; d.b_kmajor = false;
            d.M = out[k]; d.N = in[k]; d.K = rows;
            d.C = gslot(wblk[k]); d.ldc = in[k];
            RG_TRY(gemm_small(x.st, d, x.f(x.w.part)));
            colsum(x.st, x.f(dl[k]), rows, out[k], out[k], nullptr, gslot(bblk[k]));
        }
        // dh_in = dl W, then * LeakyReLU'(u_in) * mult_in
        GemmDesc d;
        d.A = x.f(dl[k]); d.lda = out[k];
        d.B = D + x.dof[wblk[k]]; d.ldb = in[k]; d.b_kmajor = false;
        d.M = rows; d.N = in[k]; d.K = out[k];
        d.C = x.f(dlin[k]); d.ldc = in[k];
        d.post = kPostLreluGrad; d.T = x.f(uin[k]); d.ldt = in[k]; d.Mult = x.f(qin[k]);
        RG_TRY(gemm_small(x.st, d, x.f(x.w.part)));
    }
    return check_launch("d_upper_backward");
}

Ws make_ws(const Dims &m, int64_t *go, int64_t *dof) {
    layout(m, go, dof);
    return Ws(m, go, dof);
}

int check_common(const rg_gan_model_t *mdl, void *ws, const rg_gan_batch_t *bt) {
    if (!mdl || !ws || !bt || !mdl->g || !mdl->d) return fail_arg("rg_gan: null model / workspace / batch");
    const rg_gan_dims_t &dm = mdl->dims;
    if (dm.num_items <= 0 || dm.slate_size <= 0 || dm.hidden < 2 || dm.hidden % 8 || dm.emb_dim <= 0 ||
        dm.z_dim <= 0 || dm.batch_max <= 0)
        return fail_arg("rg_gan: bad dims (hidden must be a positive multiple of 8)");
    if (bt->rows < 1 || bt->rows > dm.batch_max) return fail_arg("rg_gan: rows must be in [1, batch_max]");
    if (bt->hist_len <= 0 || !bt->hist) return fail_arg("rg_gan: empty history");
    return 0;
}

}  // namespace
}  // namespace rg

using namespace rg;

extern "C" int rg_gan_layout(const rg_gan_dims_t *dims, int64_t *g_off, int64_t *d_off, int64_t *strides) {
    if (!dims || !g_off || !d_off) return fail_arg("rg_gan_layout: null argument");
    const Dims m(*dims);
    layout(m, g_off, d_off);
    if (strides) {
        strides[0] = m.kz;
        strides[1] = m.ks;
    }
    return 0;
}

extern "C" int64_t rg_gan_workspace_bytes(const rg_gan_dims_t *dims) {
    const Dims m(*dims);
    int64_t go[RG_GAN_G_END + 1], dof[RG_GAN_D_END + 1];
    return make_ws(m, go, dof).total * 4;
}

extern "C" int64_t rg_gan_workspace_offset(const rg_gan_dims_t *dims, int32_t view) {
    const Dims m(*dims);
    int64_t go[RG_GAN_G_END + 1], dof[RG_GAN_D_END + 1];
    const Ws w = make_ws(m, go, dof);
    if (view == RG_GAN_WS_FAKE) return w.fake * 4;
    if (view == RG_GAN_WS_DOUT) return w.dval * 4;
    return -1;
}

extern "C" int rg_gan_d_step(void *stream, const rg_gan_model_t *mdl, void *workspace, const rg_gan_batch_t *bt,
                             const rg_gan_noise_t *nz, const rg_opt_t *opt, float *out) {
    RG_TRY(check_common(mdl, workspace, bt));
    if (bt->rows < 2) return fail_arg("rg_gan_d_step: training needs >= 2 rows (BatchNorm batch statistics)");
    if (!bt->slates || !bt->hit_col || !bt->hit_row || !bt->hit_tile_off || !nz || !nz->z || !opt || !out)
        return fail_arg("rg_gan_d_step: slates, hits, noise, opt and out are required");
    const Dims m(mdl->dims);
    if (bt->n_hits != bt->rows * m.S) return fail_arg("rg_gan_d_step: n_hits != rows * S");
    int64_t go[RG_GAN_G_END + 1], dof[RG_GAN_D_END + 1];
    const Ws w = make_ws(m, go, dof);
    const Ctx x{(hipStream_t)stream, m, go, dof, w, (char *)workspace};
    const int B = bt->rows;
    float *D = mdl->d;
    float *dgrad = x.f(w.dgrad);
    const int64_t small0 = dof[RG_GAN_D_EMB], small_n = dof[RG_GAN_D_END] - small0;

    // 1. clamp every D parameter (CGANs.py:438-439): the small ones in place; W1S is
    //    clamped where it is read (GEMM B-operand loads, the real-slate gather, and the
    //    optimizer epilogue before its update), so it is never rewritten just for this
    hipLaunchKernelGGL(clamp_kernel, dim3(blocks(small_n)), dim3(256), 0, x.st, D + small0, small_n, kClamp);
    // 2. D(real): history sums, sparse layer 1 (rows [0, B))
    hist_sum(x.st, D + dof[RG_GAN_D_EMB], bt, B, (int)m.E, (int)m.N, x.f(w.cd));
    const Drop qr1 = make_drop(nz, 0, m.H2, kDropD, 0);
    hipLaunchKernelGGL(d_real_l1_kernel, dim3(B), dim3(256), 0, x.st, D + dof[RG_GAN_D_W1S], m.ks,
                       D + dof[RG_GAN_D_W1E], D + dof[RG_GAN_D_B1], x.f(w.cd), (int)m.E, bt->slates, (int)m.S, m.N,
                       B, (int)m.H2, qr1, x.f(w.u1), x.f(w.h1), x.f(w.q1));
    // 3. G(z) in train mode (running stats move; its dropout draws sit between D's)
    RG_TRY(g_forward(x, mdl, bt, nz->z, nz, 3, true, true));
    RG_TRY(g_heads(x, mdl, B));
    // 4. D(fake.detach()) layer 1: dense split-K GEMM over the S*N slate columns (rows [B, 2B))
    {
        GemmDesc d;
        d.A = x.f(w.fake); d.lda = m.ks;
        d.B = D + dof[RG_GAN_D_W1S]; d.ldb = m.ks; d.clamp_b = kClamp;
        d.M = B; d.N = m.H2; d.K = m.ks;    // pad columns of fake and W1S are zero
        d.epi = kEpiPartial; d.splits = pick_splits(B, m.H2, m.ks); d.C = x.f(w.part);
        RG_TRY(gemm_small(x.st, d, x.f(x.w.part)));
        const Drop qf1 = make_drop(nz, 5, m.H2, kDropD, 0);
        hipLaunchKernelGGL(reduce_act_kernel, dim3(blocks((int64_t)B * m.H2)), dim3(256), 0, x.st, x.f(w.part),
                           d.splits, (int64_t)B * m.H2, B, (int)m.H2, D + dof[RG_GAN_D_B1], x.f(w.cd),
                           D + dof[RG_GAN_D_W1E], (int)m.E, qf1, x.f(w.u1) + (int64_t)B * m.H2, x.f(w.h1) + (int64_t)B * m.H2,
                           x.f(w.q1) + (int64_t)B * m.H2);
    }
    // 5. layers 2..4 on the stacked [real; fake] rows, losses
    const Drop q2[2] = {make_drop(nz, 1, m.H, kDropD, 0), make_drop(nz, 6, m.H, kDropD, 0)};
    const Drop q3[2] = {make_drop(nz, 2, m.H1, kDropD, 0), make_drop(nz, 7, m.H1, kDropD, 0)};
    RG_TRY(d_upper_forward(x, mdl, 2 * B, q2, q3, 2, B));
    hipLaunchKernelGGL(d_loss_kernel, dim3(1), dim3(256), 0, x.st, x.f(w.dval), B, 1, x.f(w.dout), out);
    // 6. backward: small-parameter gradients, dl1 for both passes
    hipMemsetAsync(dgrad, 0, (size_t)small_n * 4, x.st);
    RG_TRY(d_upper_backward(x, mdl, 2 * B, dgrad));
    colsum(x.st, x.f(w.dl1), 2 * B, m.H2, m.H2, nullptr, dgrad + (dof[RG_GAN_D_B1] - small0));
    hipLaunchKernelGGL(d_l1_w1e_grad_kernel, dim3((unsigned)((m.H2 + 63) / 64)), dim3(1024), 0, x.st, x.f(w.dl1), B,
                       (int)m.H2, x.f(w.cd), (int)m.E, dgrad + (dof[RG_GAN_D_W1E] - small0));
    hipLaunchKernelGGL(d_l1_dc_kernel, dim3(B), dim3(256), 0, x.st, x.f(w.dl1), B, (int)m.H2, (int)m.E,
                       D + dof[RG_GAN_D_W1E], x.f(w.dc));
    emb_grad(x.st, bt, x.f(w.dc), m.E, (int)m.E, dgrad);
    // 7. W1S: gradient GEMM over the fake rows + the real rows' sparse column hits,
    //    fused with clamp + optimizer update in place
    {
        GemmDesc d;
        d.A = x.f(w.dl1) + (int64_t)B * m.H2; d.lda = m.H2; d.a_kmajor = false;
        d.B = x.f(w.fake); d.ldb = m.ks; d.b_kmajor = false;
        d.M = m.H2; d.N = m.SN; d.K = B;
        d.epi = kEpiOpt;
        d.P = D + dof[RG_GAN_D_W1S]; d.ldp = m.ks;
        d.Ms = mdl->d_m ? mdl->d_m + dof[RG_GAN_D_W1S] : nullptr;
        d.Vs = mdl->d_v ? mdl->d_v + dof[RG_GAN_D_W1S] : nullptr;
        d.opt = *opt; d.clamp_p = kClamp;
        d.hit_col = bt->hit_col; d.hit_row = bt->hit_row; d.n_hits = bt->n_hits; d.hit_tile_off = bt->hit_tile_off;
        d.hit_src = x.f(w.dl1); d.hit_ld = m.H2;
        RG_TRY(gemm_small(x.st, d, x.f(x.w.part)));
    }
    // 8. the small D parameters (clamped above)
    hipLaunchKernelGGL(opt_flat_kernel, dim3(blocks(small_n)), dim3(256), 0, x.st, D + small0, dgrad,
                       mdl->d_m ? mdl->d_m + small0 : nullptr, mdl->d_v ? mdl->d_v + small0 : nullptr, small_n,
                       *opt);
    return check_launch("rg_gan_d_step");
}

extern "C" int rg_gan_g_step(void *stream, const rg_gan_model_t *mdl, void *workspace, const rg_gan_batch_t *bt,
                             const rg_gan_noise_t *nz, const rg_opt_t *opt, float *out, float *slates) {
    RG_TRY(check_common(mdl, workspace, bt));
    if (bt->rows < 2) return fail_arg("rg_gan_g_step: training needs >= 2 rows (BatchNorm batch statistics)");
    if (!nz || !nz->z || !opt || !out) return fail_arg("rg_gan_g_step: noise, opt and out are required");
    const Dims m(mdl->dims);
    int64_t go[RG_GAN_G_END + 1], dof[RG_GAN_D_END + 1];
    const Ws w = make_ws(m, go, dof);
    const Ctx x{(hipStream_t)stream, m, go, dof, w, (char *)workspace};
    const int B = bt->rows;
    float *G = mdl->g, *D = mdl->d;
    float *ggrad = x.f(w.ggrad);
    const int64_t small0 = go[RG_GAN_G_BH], small_n = go[RG_GAN_G_RM1] - small0;
    auto gslot = [&](int blk) { return ggrad + (go[blk] - small0); };

    // 1. fake = G(z) (train), D(fake) with D frozen and in train mode (dropout slots 2..4)
    RG_TRY(g_forward(x, mdl, bt, nz->z, nz, 0, true, true));
    RG_TRY(g_heads(x, mdl, B));
    hist_sum(x.st, D + dof[RG_GAN_D_EMB], bt, B, (int)m.E, (int)m.N, x.f(w.cd));
    {
        GemmDesc d;
        d.A = x.f(w.fake); d.lda = m.ks;
        d.B = D + dof[RG_GAN_D_W1S]; d.ldb = m.ks;
        d.M = B; d.N = m.H2; d.K = m.ks;
        d.epi = kEpiPartial; d.splits = pick_splits(B, m.H2, m.ks); d.C = x.f(w.part);
        RG_TRY(gemm_small(x.st, d, x.f(x.w.part)));
        const Drop q1 = make_drop(nz, 2, m.H2, kDropD, 8);
        hipLaunchKernelGGL(reduce_act_kernel, dim3(blocks((int64_t)B * m.H2)), dim3(256), 0, x.st, x.f(w.part),
                           d.splits, (int64_t)B * m.H2, B, (int)m.H2, D + dof[RG_GAN_D_B1], x.f(w.cd),
                           D + dof[RG_GAN_D_W1E], (int)m.E, q1, x.f(w.u1), x.f(w.h1), x.f(w.q1));
    }
    const Drop q2 = make_drop(nz, 3, m.H, kDropD, 8), q3 = make_drop(nz, 4, m.H1, kDropD, 8);
    RG_TRY(d_upper_forward(x, mdl, B, &q2, &q3, 1, B));
    hipLaunchKernelGGL(d_loss_kernel, dim3(1), dim3(256), 0, x.st, x.f(w.dval), B, 0, x.f(w.dout), out);
    // 2. backward through D (no D gradients) to its slate input, through tanh: dlogit
    RG_TRY(d_upper_backward(x, mdl, B, nullptr));
    hipMemsetAsync(ggrad, 0, (size_t)small_n * 4, x.st);
    {
        GemmDesc d;
        d.A = x.f(w.dl1); d.lda = m.H2;
        d.B = D + dof[RG_GAN_D_W1S]; d.ldb = m.ks; d.b_kmajor = false;
        d.M = B; d.N = m.SN; d.K = m.H2;
        d.C = x.f(w.dlogit); d.ldc = m.ks;
        d.post = kPostTanhGrad; d.T = x.f(w.fake); d.ldt = m.ks; d.colsum = x.f(w.colsum);
        RG_TRY(gemm_small(x.st, d, x.f(x.w.part)));
        hipLaunchKernelGGL(sum_rows_kernel, dim3(blocks(m.SN)), dim3(256), 0, x.st, x.f(w.colsum),
                           (int)gemm_tiles_m(B), m.SN, m.SN, gslot(RG_GAN_G_BH));
    }
    // 3. da2 = dlogit WH (before WH moves), then through Dropout + LeakyReLU of layer 2
    {
        GemmDesc d;
        d.A = x.f(w.dlogit); d.lda = m.ks;
        d.B = G + go[RG_GAN_G_WH]; d.ldb = m.H; d.b_kmajor = false;
        d.M = B; d.N = m.H; d.K = m.ks;     // pad columns of dlogit and pad rows of WH are zero
        d.epi = kEpiPartial; d.splits = pick_splits(B, m.H, m.ks); d.C = x.f(w.part);
        RG_TRY(gemm_small(x.st, d, x.f(x.w.part)));
        hipLaunchKernelGGL(reduce_lrelu_grad_kernel, dim3(blocks((int64_t)B * m.H)), dim3(256), 0, x.st,
                           x.f(w.part), d.splits, (int64_t)B * m.H, x.f(w.d2), x.f(w.q2g), x.f(w.do2));
    }
    // 4. WH: gradient GEMM (dlogit^T a2) fused with the optimizer update in place
    {
        GemmDesc d;
        d.A = x.f(w.dlogit); d.lda = m.ks; d.a_kmajor = false;
        d.B = x.f(w.a2); d.ldb = m.H; d.b_kmajor = false;
        d.M = m.SN; d.N = m.H; d.K = B;
        d.epi = kEpiOpt;
        d.P = G + go[RG_GAN_G_WH]; d.ldp = m.H;
        d.Ms = mdl->g_m ? mdl->g_m + go[RG_GAN_G_WH] : nullptr;
        d.Vs = mdl->g_v ? mdl->g_v + go[RG_GAN_G_WH] : nullptr;
        d.opt = *opt;
        RG_TRY(gemm_small(x.st, d, x.f(x.w.part)));
    }
    // 5. BatchNorm 2 backward, layer 2 weights, back through layer 1
    hipLaunchKernelGGL(bn_bwd_kernel, dim3((unsigned)m.H), dim3(256), 0, x.st, x.f(w.do2), x.f(w.yh2), x.f(w.rs2),
                       G + go[RG_GAN_G_GAMMA2], B, (int)m.H, gslot(RG_GAN_G_GAMMA2), gslot(RG_GAN_G_BETA2),
                       x.f(w.dy2));
    {
        GemmDesc d;   // dW2 = dy2^T a1
        d.A = x.f(w.dy2); d.lda = m.H; d.a_kmajor = false;
        d.B = x.f(w.a1); d.ldb = m.H1; d.b_kmajor = false;
        d.M = m.H; d.N = m.H1; d.K = B;
        d.C = gslot(RG_GAN_G_W2); d.ldc = m.H1;
        RG_TRY(gemm_small(x.st, d, x.f(w.part)));
        colsum(x.st, x.f(w.dy2), B, m.H, m.H, nullptr, gslot(RG_GAN_G_B2));
        d = GemmDesc();  // do1 = (dy2 W2) * LeakyReLU'(d1) * mult1
        d.A = x.f(w.dy2); d.lda = m.H;
        d.B = G + go[RG_GAN_G_W2]; d.ldb = m.H1; d.b_kmajor = false;
        d.M = B; d.N = m.H1; d.K = m.H;
        d.C = x.f(w.do1); d.ldc = m.H1;
        d.post = kPostLreluGrad; d.T = x.f(w.d1); d.ldt = m.H1; d.Mult = x.f(w.q1g);
        RG_TRY(gemm_small(x.st, d, x.f(x.w.part)));
    }
    hipLaunchKernelGGL(bn_bwd_kernel, dim3((unsigned)m.H1), dim3(256), 0, x.st, x.f(w.do1), x.f(w.yh1), x.f(w.rs1),
                       G + go[RG_GAN_G_GAMMA1], B, (int)m.H1, gslot(RG_GAN_G_GAMMA1), gslot(RG_GAN_G_BETA1),
                       x.f(w.dy1));
    {
        GemmDesc d;   // dW1 = dy1^T a0
        d.A = x.f(w.dy1); d.lda = m.H1; d.a_kmajor = false;
        d.B = x.f(w.a0); d.ldb = m.kz; d.b_kmajor = false;
        d.M = m.H1; d.N = m.kz; d.K = B;
        d.C = gslot(RG_GAN_G_W1); d.ldc = m.kz;
        RG_TRY(gemm_small(x.st, d, x.f(w.part)));
        colsum(x.st, x.f(w.dy1), B, m.H1, m.H1, nullptr, gslot(RG_GAN_G_B1));
        d = GemmDesc();  // dx0 = (dy1 W1) * LeakyReLU'(x0)  (a0 > 0 iff x0 > 0)
        d.A = x.f(w.dy1); d.lda = m.H1;
        d.B = G + go[RG_GAN_G_W1]; d.ldb = m.kz; d.b_kmajor = false;
        d.M = B; d.N = m.kz; d.K = m.H1;
        d.C = x.f(w.dx0); d.ldc = m.kz;
        d.post = kPostLreluGrad; d.T = x.f(w.a0); d.ldt = m.kz;
        RG_TRY(gemm_small(x.st, d, x.f(x.w.part)));
    }
    // 6. history embedding of G: the e columns of dx0, grouped per item
    emb_grad(x.st, bt, x.f(w.dx0) + m.Z, m.kz, (int)m.E, gslot(RG_GAN_G_EMB));
    // 7. the remaining G parameters
    hipLaunchKernelGGL(opt_flat_kernel, dim3(blocks(small_n)), dim3(256), 0, x.st, G + small0, ggrad,
                       mdl->g_m ? mdl->g_m + small0 : nullptr, mdl->g_v ? mdl->g_v + small0 : nullptr, small_n,
                       *opt);
    RG_TRY(check_launch("rg_gan_g_step"));
    // 8. eval-mode inference on the same z (CGANs.py:404-406)
    if (slates) return rg_gan_generate(stream, mdl, workspace, bt, nz->z, slates);
    return 0;
}

extern "C" int rg_gan_generate(void *stream, const rg_gan_model_t *mdl, void *workspace, const rg_gan_batch_t *bt,
                               const float *z, float *slates) {
    RG_TRY(check_common(mdl, workspace, bt));
    if (!z || !slates) return fail_arg("rg_gan_generate: z and slates are required");
    const Dims m(mdl->dims);
    int64_t go[RG_GAN_G_END + 1], dof[RG_GAN_D_END + 1];
    const Ws w = make_ws(m, go, dof);
    const Ctx x{(hipStream_t)stream, m, go, dof, w, (char *)workspace};
    const int B = bt->rows;
    RG_TRY(g_forward(x, mdl, bt, z, nullptr, 0, false, false));
    if (m.N < kGemmBN) {   // heads narrower than a column tile: tanh outputs, then a row scan
        RG_TRY(g_heads(x, mdl, B));
        hipLaunchKernelGGL(argmax_rows_kernel, dim3(blocks((int64_t)B * m.S)), dim3(256), 0, x.st, x.f(w.fake),
                           m.ks, B, (int)m.S, m.N, slates);
        return check_launch("rg_gan_generate");
    }
    GemmDesc d;
    d.A = x.f(w.a2); d.lda = m.H;
    d.B = mdl->g + go[RG_GAN_G_WH]; d.ldb = m.H;
    d.M = B; d.N = m.SN; d.K = m.H;
    d.epi = kEpiArgmax; d.bias = mdl->g + go[RG_GAN_G_BH]; d.seg = m.N;
    d.amax = reinterpret_cast<float2 *>(x.f(w.amax));
    RG_TRY(gemm_small(x.st, d, x.f(x.w.part)));
    hipLaunchKernelGGL(argmax_final_kernel, dim3((unsigned)(((int64_t)B * m.S + 3) / 4)), dim3(256), 0, x.st, d.amax, B,
                       gemm_tiles_n(m.SN), (int)m.S, m.N, slates);
    return check_launch("rg_gan_generate");
}
