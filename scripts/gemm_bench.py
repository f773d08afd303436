"""Time the cGAN's large fp32 MFMA GEMM shapes through rg_gemm_f32 (C4 sizes):
python scripts/gemm_bench.py  ->  one line per shape: us per call, TFLOP/s, frac of 157.3."""
import ctypes
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from recommendation_gans_amd import _lib  # noqa: E402
from recommendation_gans_amd.gan_engine import ptr  # noqa: E402

L = _lib.load()
SN, B, H, H2 = 100540, 256, 256, 512
KS = 100544
dev = "cuda"


def run(name, A, lda, akm, Bm, ldb, bkm, M, N, K, ldc, splits=1, post=0, reps=20):
    C = torch.empty(M, ldc, device=dev)
    work = torch.empty(max(splits, 1) * M * N, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    args = (st, ptr(A), lda, akm, ptr(Bm), ldb, bkm, M, N, K, ptr(C), ldc, ptr(None), post, splits, ptr(work))
    _lib.check(L.rg_gemm_f32(*args), name)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        L.rg_gemm_f32(*args)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / reps * 1e3
    tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
    print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "splits": splits, "us": round(us, 1),
                      "tflops": round(tf, 2), "frac": round(tf / 157.3, 3)}), flush=True)


fake = torch.rand(B, KS, device=dev)
w1s = torch.rand(H2, KS, device=dev) * 0.01
wh = torch.rand(KS, H, device=dev) * 0.01
a2 = torch.rand(B, H, device=dev)
dl1 = torch.rand(B, H2, device=dev)
RMS_ONLY = "--rms-only" in sys.argv
for sp in (() if RMS_ONLY else (32, 64, 128)):
    run(f"D1 fwd split{sp} (AK,BK)", fake, KS, 1, w1s, KS, 1, B, H2, KS, H2, splits=sp)
if not RMS_ONLY:
    run("heads fwd tanh (AK,BK)", a2, H, 1, wh, H, 1, B, SN, H, KS, post=1)
    run("D1 dX (AK,BN)", dl1, H2, 1, w1s, KS, 0, B, SN, H2, KS)
    run("D1 dW (AM,BN)", dl1, H2, 0, fake, KS, 0, H2, SN, B, KS)
    run("heads dW (AM,BN)", fake, KS, 0, a2, H, 0, SN, H, B, H)
for sp in (() if RMS_ONLY else (64, 128)):
    run(f"heads dA split{sp} (AK,BN)", fake, KS, 1, wh, H, 0, B, H, KS, H, splits=sp)


def run_rms(name, A, lda, akm, Bm, ldb, bkm, M, N, K, reps=10):
    P = torch.rand(M, N, device=dev) * 0.01
    V = torch.rand(M, N, device=dev) * 1e-6
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    args = (st, ptr(A), lda, akm, ptr(Bm), ldb, bkm, M, N, K, ptr(P), ptr(V), N, 1e-3, 0.99, 1e-8)
    _lib.check(L.rg_gemm_f32_rms(*args), name)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        L.rg_gemm_f32_rms(*args)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / reps * 1e3
    print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "us": round(us, 1),
                      "pv_GBps": round(4 * 4 * M * N / (us * 1e-6) / 1e9, 1)}), flush=True)
    # the same P / V traffic as a plain streaming update (torch ops, reference point)
    g = torch.rand(M, N, device=dev)
    a.record()
    for _ in range(reps):
        V.mul_(0.99).addcmul_(g, g, value=0.01)
        P.addcdiv_(g, V.sqrt().add_(1e-8), value=-1e-3)
    b.record()
    torch.cuda.synchronize()
    us2 = a.elapsed_time(b) / reps * 1e3
    print(json.dumps({"shape": "torch rmsprop same size", "us": round(us2, 1)}), flush=True)


if "--ws-ab" in sys.argv:
    # the two forms of the optimizer GEMM (rg_gemm_ws_mode 0: the update in gemm_kernel's
    # epilogue, 1: the wave-specialised persistent kernel), alternating
    for mode in (0, 1, 0, 1):
        L.rg_gemm_ws_mode(mode)
        run_rms(f"ws{mode} D1 dW + RMSprop (AM,BN)", dl1, H2, 0, fake, KS, 0, H2, KS - 4, B)
        run_rms(f"ws{mode} heads dW + RMSprop (AM,BN)", fake, KS, 0, a2, H, 0, KS - 4, H, B)
    sys.exit(0)
if "--rms-sweep" in sys.argv:
    # wave quantization of the W1S update: 4 x ceil(N / 128) tiles on 256 CUs x 3 workgroups
    # (768 slots): N = 98,304 fills four rounds exactly, N = 100,540 (the model) spills 72 tiles
    # into a fifth
    # measured (round 5): 377 / 379 / 353 us at 2,976 / 3,072 / 3,076 tiles -- no round quantization
    for n_ in (98304 - 128 * 24, 98304, 98304 + 128, KS - 4):
        run_rms(f"D1 dW + RMSprop N={n_} tiles={4 * -(-n_ // 128)}", dl1, H2, 0, fake, KS, 0, H2, n_, B)
    sys.exit(0)
run_rms("D1 dW + RMSprop (AM,BN)", dl1, H2, 0, fake, KS, 0, H2, KS - 4, B)
run_rms("heads dW + RMSprop (AM,BN)", fake, KS, 0, a2, H, 0, KS - 4, H, B)
