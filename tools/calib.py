"""Calibration microbenchmarks on the GPU box (diagnostic, not part of the product):
achievable copy bandwidth and vendor-GEMM time for the 1x1-conv shapes of yolox_s."""
import torch

def t(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us

dev = "cuda"
for mb in (26, 52, 105, 210):
    n = mb * 2**20 // 2
    x = torch.randn(n, device=dev).to(torch.bfloat16)
    y = torch.empty_like(x)
    us = t(lambda: y.copy_(x))
    print(f"copy {mb} MB bf16: {us:.1f} us  {2 * n * 2 / us / 1e6:.2f} TB/s (read+write)")
    us = t(lambda: x.sum())
    print(f"sum  {mb} MB bf16: {us:.1f} us  {n * 2 / us / 1e6:.2f} TB/s (read)")
    y.fill_(1.0)
    us = t(lambda: y.fill_(2.0))
    print(f"fill {mb} MB bf16: {us:.1f} us  {n * 2 / us / 1e6:.2f} TB/s (write)")
for M, K, N in ((819200, 64, 64), (819200, 32, 32), (204800, 128, 128), (204800, 64, 64), (51200, 256, 256),
                (204800, 256, 128), (204800, 1152, 256), (204800, 1152, 128), (51200, 1152, 128), (12800, 1024, 512)):
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(K, N, device=dev).to(torch.bfloat16)
    us = t(lambda: a @ w)
    byt = (M * K + M * N + K * N) * 2
    print(f"gemm M={M} K={K} N={N}: {us:.1f} us  {2 * M * K * N / us / 1e6:.1f} TFLOP/s  {byt / us / 1e6:.2f} TB/s")
