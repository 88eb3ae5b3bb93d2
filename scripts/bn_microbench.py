#!/usr/bin/env python3
"""Per-call time of the ResNet-18 BatchNorm consumer kernels (csrc/bn.hip bn_apply_acc / bn_dx_acc) at the
four stage shapes of CIFAR ResNet-18 (B = 256), inside a captured graph (as the engine runs them), against a
bf16 copy of the same tensor (the HBM yardstick).  Usage: python3 scripts/bn_microbench.py [nrep ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distriflow_amd import ops  # noqa: E402

SHAPES = [(64, 64), (64, 512), (256 * 32 * 32, 64), (256 * 16 * 16, 128), (256 * 8 * 8, 256), (256 * 4 * 4, 512)]


def timed(fn, n=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (5 * n)


def main():
    reps = [int(v) for v in sys.argv[1:]] or [8, 1]
    dev = "cuda"
    for M, C in SHAPES:
        x = torch.randn(M, C, device=dev).to(torch.bfloat16)
        g = torch.randn(M, C, device=dev).to(torch.bfloat16)
        y = torch.empty_like(x)
        gamma, beta = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
        mean, invstd = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        dgamma, dbeta, coef = torch.zeros(C, device=dev), torch.zeros(C, device=dev), torch.zeros(3 * C, device=dev)
        line = [f"M={M:7d} C={C:4d} {M * C * 2 / 1e6:6.1f} MB"]
        line.append(f"copy {timed(lambda: y.copy_(x)):6.2f} us")
        line.append(f"plain apply {timed(lambda: ops.bn_apply(x, y, gamma, beta, mean, invstd, relu=True)):6.2f} us")
        line.append(f"plain dx {timed(lambda: ops.bn_dx(x, g, y, coef)):6.2f} us")
        for nrep in reps:
            acc = torch.zeros(nrep, 2, C, dtype=torch.float64, device=dev)
            acc[:, 0] = 1.0
            acc[:, 1] = 2.0
            accb = torch.zeros(nrep, 2, C, dtype=torch.float64, device=dev)
            t_ap = timed(lambda: ops.bn_apply_acc(x, y, gamma, beta, acc, None, mean, invstd, rm, rv, relu=True))
            t_dx = timed(lambda: ops.bn_dx_acc(x, g, y, accb, None, gamma, mean, invstd, dgamma, dbeta, coef))
            line.append(f"nrep {nrep}: apply {t_ap:6.2f} us dx {t_dx:6.2f} us")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
