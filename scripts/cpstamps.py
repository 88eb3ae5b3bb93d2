#!/usr/bin/env python3
"""Phase shares of the fused conv+pool kernels from in-kernel s_memtime stamps (diagnostic only:
stamps add waits, so read shares, not absolute lengths).  Slots: fwd 0 start, 1 setup done,
per group g: 2+3g staged, 3+3g shift-copies built, 4+3g tiles done, 31 end; wgrad 0, 1,
2+2g staged, 3+2g computed, 30 loop end, 31 end; dgrad 0, 1, 2+3g scattered, 3+3g computed,
4+3g cleared, 31 end."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distriflow_amd import native, ops  # noqa: E402


def report(name, st, grid, kind):
    st = st[:grid].cpu().numpy().astype("float64")
    import numpy as np

    valid = st[:, 0] > 0
    st = st[valid]
    t0 = st[:, 0].min()
    end = st[:, 31] - t0
    print(f"{name}: blocks {valid.sum()}  kernel span {end.max():.0f} clk  block start spread "
          f"{(st[:, 0] - t0).max():.0f} clk  median block life {np.median(st[:, 31] - st[:, 0]):.0f} clk")
    setup = np.median(st[:, 1] - st[:, 0])
    print(f"   setup {setup:.0f}")
    if kind == "fwd":
        g = 0
        while 4 + 3 * g < 31 and (st[:, 4 + 3 * g] > 0).any():
            m = st[:, 4 + 3 * g] > 0
            prev = st[m, 1] if g == 0 else st[m, 4 + 3 * (g - 1)]
            a = np.median(st[m, 2 + 3 * g] - prev)
            b = np.median(st[m, 3 + 3 * g] - st[m, 2 + 3 * g])
            c = np.median(st[m, 4 + 3 * g] - st[m, 3 + 3 * g])
            print(f"   group {g}: stage {a:.0f}  build {b:.0f}  tiles {c:.0f}   ({m.sum()} blocks)")
            g += 1
    elif kind == "wgrad":
        g = 0
        while 3 + 2 * g < 30 and (st[:, 3 + 2 * g] > 0).any():
            m = st[:, 3 + 2 * g] > 0
            prev = st[m, 1] if g == 0 else st[m, 3 + 2 * (g - 1)]
            a = np.median(st[m, 2 + 2 * g] - prev)
            b = np.median(st[m, 3 + 2 * g] - st[m, 2 + 2 * g])
            print(f"   group {g}: stage {a:.0f}  compute {b:.0f}   ({m.sum()} blocks)")
            g += 1
        print(f"   reduction {np.median(st[:, 31] - st[:, 30]):.0f}")
        m = st[:, 23] > 0
        if m.any():
            d = lambda a, b: np.median(st[m, b] - st[m, a])  # noqa: E731
            print(f"   group1 detail: writes {d(3, 20):.0f}  issue-loads {d(20, 21):.0f}  sync {d(21, 22):.0f}  "
                  f"build {d(22, 23):.0f}  sync {d(23, 4):.0f}")
    else:
        g = 0
        while 4 + 3 * g < 31 and (st[:, 4 + 3 * g] > 0).any():
            m = st[:, 4 + 3 * g] > 0
            prev = st[m, 1] if g == 0 else st[m, 4 + 3 * (g - 1)]
            a = np.median(st[m, 2 + 3 * g] - prev)
            b = np.median(st[m, 3 + 3 * g] - st[m, 2 + 3 * g])
            c = np.median(st[m, 4 + 3 * g] - st[m, 3 + 3 * g])
            print(f"   group {g}: scatter {a:.0f}  tiles {b:.0f}  clear {c:.0f}   ({m.sum()} blocks)")
            g += 1


def main():
    m = native.require()
    B, dev = 4096, "cuda"
    data = torch.randint(0, 256, (60000, 28, 28, 1), dtype=torch.uint8, device=dev)
    idx = torch.randint(0, 60000, (B,), device=dev)
    g1 = ops.GatherRef(data, idx, 1 / 255, (28, 28, 1))
    x2 = torch.randn(B, 14, 14, 6, device=dev).to(torch.bfloat16)
    buf = torch.zeros(4096 * 32, dtype=torch.int64, device=dev)
    for name, x, H, C, N, k, pad, PH in (("conv1", g1, 28, 1, 6, 5, 2, 14), ("conv2", x2, 14, 6, 16, 5, 0, 5)):
        kp = ops.convpool_fwd_layout(H, H, C, k, k, pad, N)[1]
        w = torch.randn(16, kp, device=dev).to(torch.bfloat16) * 0.1
        b = torch.zeros(N, device=dev)
        out = torch.empty(B, PH, PH, N, device=dev, dtype=torch.bfloat16)
        code = torch.empty(B, PH, PH, N, device=dev, dtype=torch.uint8)
        dp = torch.randn(B, PH, PH, N, device=dev).to(torch.bfloat16)
        gw = torch.empty(N, k * k * C, device=dev)
        gb = torch.empty(N, device=dev)
        ws = torch.empty(1 << 22, device=dev)
        for _ in range(3):
            ops.convpool_fwd(x, w, b, out, code, k, k, pad)
        for kind in ("fwd", "wgrad", "dgrad"):
            if kind == "dgrad" and name == "conv1":
                continue
            buf.zero_()
            m.convpool_set_stamps(buf)
            if kind == "fwd":
                ops.convpool_fwd(x, w, b, out, code, k, k, pad)
            elif kind == "wgrad":
                ops.convpool_wgrad(x, dp, code, gw, gb, ws, k, k, pad)
            else:
                wt = torch.randn(16, ops.convpool_dgrad_layout(14, 14, 6, k, k, pad, 16)[1], device=dev).to(torch.bfloat16) * 0.1
                dx = torch.empty(B, 14, 14, 6, device=dev, dtype=torch.bfloat16)
                ops.convpool_dgrad(dp, code, None, wt, dx, k, k, pad)
            torch.cuda.synchronize()
            m.convpool_set_stamps(None)
            report(f"{name} {kind}", buf.view(4096, 32), 4096, kind)


if __name__ == "__main__":
    main()
