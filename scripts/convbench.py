#!/usr/bin/env python3
"""Per-conv timing of the ResNet-18 CIFAR convolutions (B=256): forward, data gradient and weight
gradient of each distinct layer shape through the engine's ops (HIP events around 20 launches)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distriflow_amd import ops  # noqa: E402

dev = "cuda"


def _r(a, b):
    return (a + b - 1) // b * b


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


SHAPES = [  # name, B, H, W, C, N, k, stride, pad
    ("l1", 256, 32, 32, 64, 64, 3, 1, 1),
    ("l2.0c1", 256, 32, 32, 64, 128, 3, 2, 1),
    ("l2", 256, 16, 16, 128, 128, 3, 1, 1),
    ("l3", 256, 8, 8, 256, 256, 3, 1, 1),
    ("l4", 256, 4, 4, 512, 512, 3, 1, 1),
]


def main():
    ws = torch.empty(1 << 25, device=dev)
    tot = 0.0
    only = sys.argv[1] if len(sys.argv) > 1 else None
    for name, B, H, W, C, N, k, s, p in SHAPES:
        if only and name != only:
            continue
        OH, OW = ops.conv_out_hw(H, W, k, k, s, p)
        x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
        w = torch.randn(N, k * k * C, device=dev) / (k * k * C) ** 0.5
        wp = torch.zeros(_r(N, 16), _r(k * k * C, 32), dtype=torch.bfloat16, device=dev)
        wp[:N, :k * k * C] = w.to(torch.bfloat16)
        wt3 = w.view(N, k * k, C).permute(2, 1, 0).reshape(C, k * k * N)
        wt = torch.zeros(_r(C, 16), _r(k * k * N, 32), dtype=torch.bfloat16, device=dev)
        wt[:C, :k * k * N] = wt3.to(torch.bfloat16)
        out = torch.empty(B, OH, OW, N, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(B, OH, OW, N, device=dev).to(torch.bfloat16)
        dx = torch.empty(B, H, W, C, device=dev, dtype=torch.bfloat16)
        gw = torch.empty(N, k * k * C, device=dev)
        flop = 2.0 * B * OH * OW * N * k * k * C
        tf = timeit(lambda: ops.conv_fwd(x, wp, None, out, k, k, s, p, False))
        td = timeit(lambda: ops.conv_dgrad(dy, None, wt, dx, k, k, s, p))
        tw = timeit(lambda: ops.conv_wgrad(dy, x, gw, None, ws, k, k, s, p))
        tot += tf + td + tw
        print(f"{name:8s} fwd {tf:7.1f} us {flop / tf / 1e6:6.0f} TF/s | dgrad {td:7.1f} us {flop / td / 1e6:6.0f} TF/s"
              f" | wgrad {tw:7.1f} us {flop / tw / 1e6:6.0f} TF/s", flush=True)
    print(f"total {tot:.1f} us")


if __name__ == "__main__":
    main()
