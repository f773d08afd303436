"""Probe: fp32 GEMM rate of the ROCm libraries (torch.mm -> hipBLASLt / rocBLAS) at the cGAN's big
shapes, beside the repository's own gemm_kernel figures.  Timing only."""
import torch

def bench(M, N, K, ta=False, tb=False, it=20):
    a = torch.randn(K, M, device="cuda") if ta else torch.randn(M, K, device="cuda")
    b = torch.randn(N, K, device="cuda") if tb else torch.randn(K, N, device="cuda")
    A = a.t() if ta else a
    Bm = b.t() if tb else b
    for _ in range(3):
        torch.mm(A, Bm)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        torch.mm(A, Bm)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / it
    print(f"M={M} N={N} K={K} ta={ta} tb={tb}: {us:.1f} us, {2 * M * N * K / us / 1e6:.1f} TF", flush=True)

torch.backends.cuda.matmul.allow_tf32 = False
print(torch.backends.cuda.preferred_blas_library())
bench(256, 512, 100544)                # D layer-1 forward (fake slates x W1S^T)
bench(512, 100544, 256, ta=True)       # D layer-1 dW (dY^T X): 512 x 100544, K = batch 256
bench(256, 100544, 256)                # G heads forward (h x WH^T)
bench(256, 100544, 256, tb=True)
bench(100544, 256, 256, ta=True)       # heads dW
