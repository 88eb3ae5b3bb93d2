#!/usr/bin/env python3
"""Phase attribution for the fused conv+pool kernels: time each kernel with phases skipped
(convpool_set_debug mask: 1 staging, 2 shifted-copy build, 4 MFMA, 8 stores)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distriflow_amd import native, ops  # noqa: E402


def timeit(fn, reps=20, iters=15):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None, help="conv1|conv2: run just this forward")
    ap.add_argument("--mask", type=int, default=0)
    ap.add_argument("--n", type=int, default=50)
    args = ap.parse_args()
    m = native.require()
    B = 4096
    dev = "cuda"
    data = torch.randint(0, 256, (60000, 28, 28, 1), dtype=torch.uint8, device=dev)
    idx = torch.randint(0, 60000, (B,), device=dev)
    g1 = ops.GatherRef(data, idx, 1 / 255, (28, 28, 1))
    x2 = torch.randn(B, 14, 14, 6, device=dev).to(torch.bfloat16)
    cases = [("conv1", g1, 1, 6, 5, 2, (14, 14)), ("conv2", x2, 6, 16, 5, 0, (5, 5))]
    for name, x, C, N, k, pad, (PH, PW) in cases:
        kp = ops.convpool_fwd_layout(28 if C == 1 else 14, 28 if C == 1 else 14, C, k, k, pad, N)[1]
        w = torch.randn(16, kp, device=dev).to(torch.bfloat16) * 0.1
        b = torch.zeros(N, device=dev)
        out = torch.empty(B, PH, PW, N, device=dev, dtype=torch.bfloat16)
        code = torch.empty(B, PH, PW, N, device=dev, dtype=torch.uint8)
        dp = torch.randn(B, PH, PW, N, device=dev).to(torch.bfloat16)
        gw = torch.empty(N, k * k * C, device=dev)
        gb = torch.empty(N, device=dev)
        ws = torch.empty(1 << 22, device=dev)
        if args.only:
            if args.only != name:
                continue
            m.convpool_set_debug(args.mask)
            for _ in range(args.n):
                ops.convpool_fwd(x, w, b, out, code, k, k, pad)
            torch.cuda.synchronize()
            print(name, "mask", args.mask, "done")
            return
        res = []
        for mask in (0, 1, 2, 3, 4, 8, 12, 15, 16, 32):
            m.convpool_set_debug(mask)
            t = timeit(lambda: ops.convpool_fwd(x, w, b, out, code, k, k, pad))
            res.append(f"m{mask}={t:.1f}")
        m.convpool_set_debug(0)
        ops.convpool_fwd(x, w, b, out, code, k, k, pad)
        tw = timeit(lambda: ops.convpool_wgrad(x, dp, code, gw, gb, ws, k, k, pad))
        print(f"{name} fwd(us) " + " ".join(res) + f" | wgrad+reduce {tw:.1f}", flush=True)
        if name == "conv2":
            wt = torch.randn(16, ops.convpool_dgrad_layout(14, 14, 6, k, k, pad, 16)[1], device=dev).to(torch.bfloat16) * 0.1
            dx = torch.empty(B, 14, 14, 6, device=dev, dtype=torch.bfloat16)
            td = timeit(lambda: ops.convpool_dgrad(dp, code, None, wt, dx, k, k, pad))
            print(f"{name} dgrad {td:.1f}", flush=True)
    e = torch.empty(16, device=dev)
    print(f"empty fill kernel {timeit(lambda: e.zero_()):.1f} us")


if __name__ == "__main__":
    main()
