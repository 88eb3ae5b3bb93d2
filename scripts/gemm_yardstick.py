#!/usr/bin/env python3
"""hipBLASLt (torch.mm, bf16) on the im2col GEMM shapes of the ResNet-18 convolutions, as a yardstick
for the implicit-GEMM kernels (scripts/convbench.py prints the same layers)."""
import torch


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        a.record()
        for _ in range(n):
            fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / n)
    return best


SHAPES = [  # name, M, N, K  (C[M][N] = A[M][K] @ B[K][N])
    ("square8192", 8192, 8192, 8192),
    ("l1 fwd", 262144, 64, 576),
    ("l2 fwd", 65536, 128, 1152),
    ("l3 fwd", 16384, 256, 2304),
    ("l4 fwd", 4096, 512, 4608),
    ("l1 wgrad", 64, 576, 262144),
    ("l2 wgrad", 128, 1152, 65536),
    ("l4 wgrad", 512, 4608, 4096),
]
for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    if "wgrad" in name:  # dY^T @ X: both operands m-major in memory
        at = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: torch.mm(at.t(), b))
    else:
        b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: torch.mm(a, b.t()))
    print(f"{name:10s} {t:8.1f} us {2.0 * M * N * K / t / 1e6:7.0f} TF/s", flush=True)
