#!/usr/bin/env python3
"""Keras CNN conv2 (26x26x32 -> 24x24x32, B=1024) forward: plain igemm64 (+ separate max-pool) vs
the pooled epilogue (igemm64 POOL), timed with HIP events."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distriflow_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B, H, C, N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024, 26, 32, 32
    x = torch.relu(torch.randn(B, H, H, C, device=dev)).to(torch.bfloat16)
    w = torch.zeros(N, 288, dtype=torch.bfloat16, device=dev)
    w[:, :288] = (torch.randn(N, 288, device=dev) / 17).to(torch.bfloat16)
    b = torch.zeros(N, device=dev)
    y = torch.empty(B, 24, 24, N, dtype=torch.bfloat16, device=dev)
    p = torch.empty(B, 12, 12, N, dtype=torch.bfloat16, device=dev)
    code = torch.empty(B, 12, 12, N, dtype=torch.uint8, device=dev)
    runs = {
        "conv": lambda: ops.conv_fwd(x, w, b, y, 3, 3, 1, 0, relu=True),
        "maxpool": lambda: ops.maxpool_fwd(y, p, 2),
        "conv_pool": lambda: ops.conv_pool_fwd(x, w, b, p, code, 3, 3, 1, 0, relu=True),
    }
    which = os.environ.get("ONLY")
    for name, fn in runs.items():
        if which and name != which:
            continue
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name:<10} {e0.elapsed_time(e1) / 50 * 1e3:8.1f} us")


if __name__ == "__main__":
    main()
