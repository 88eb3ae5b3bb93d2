#!/usr/bin/env python3
"""Phase shares of the fused dense head train kernel (csrc/mlphead.hip) from in-kernel s_memtime
stamps, LeNet-5 head 400-120-84-10 at B=4096.  Slots: 0 start, 1 X staged, 2..4 forward layers,
6 softmax-CE, 7..9 backward layers (reverse order), 31 end.  Also times both launches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distriflow_amd import native, ops  # noqa: E402


def _r(a, b):
    return (a + b - 1) // b * b


def main():
    m = native.require()
    dev, B = "cuda", 4096
    dims = (400, 120, 84, 10)
    nl = len(dims) - 1
    x = torch.randn(B, dims[0], device=dev).clamp_min(0).to(torch.bfloat16)
    ws = [torch.randn(dims[i + 1], dims[i], device=dev) / dims[i] ** 0.5 for i in range(nl)]
    wp = []
    wtp = []
    for w in ws:
        N, K = w.shape
        a = torch.zeros(_r(N, 16), _r(K, 32), device=dev, dtype=torch.bfloat16)
        a[:N, :K] = w
        wp.append(a)
        t = torch.zeros(_r(K, 16), _r(N, 32), device=dev, dtype=torch.bfloat16)
        t[:K, :N] = w.t()
        wtp.append(t)
    bs = [torch.zeros(dims[i + 1], device=dev) for i in range(nl)]
    labels = torch.randint(0, 10, (60000,), device=dev, dtype=torch.int32)
    idx = torch.randint(0, 60000, (B,), device=dev)
    ldt = _r(B, 32)
    gw = [torch.empty(dims[i + 1], dims[i], device=dev) for i in range(nl)]
    gb = [torch.empty(dims[i + 1], device=dev) for i in range(nl)]
    hT = [torch.zeros(dims[i + 1], ldt, device=dev, dtype=torch.bfloat16) for i in range(nl - 1)] + [None]
    dzT = [torch.zeros(dims[i + 1], ldt, device=dev, dtype=torch.bfloat16) for i in range(nl)]
    xT = torch.zeros(dims[0], ldt, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(B, dims[0], device=dev, dtype=torch.bfloat16)
    loss_part = torch.zeros(2 * (B // 16), device=dev)
    stats = torch.zeros(2, device=dev)

    def run(ph):
        ops.head_train(wp, wtp, bs, gw, gb, hT, dzT, list(dims[:-1]), list(dims[1:]), x, True, xT, dx, None,
                       labels, idx, 1.0 / B, loss_part, stats, phases=ph)

    for ph, name in ((1, "train"), (2, "wgrad")):
        for _ in range(3):
            run(ph)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            run(ph)
        e1.record()
        torch.cuda.synchronize()
        print(f"{name}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us", flush=True)
    buf = torch.zeros(4096 * 32, dtype=torch.int64, device=dev)
    m.convpool_set_stamps(buf)
    run(1)
    torch.cuda.synchronize()
    m.convpool_set_stamps(None)
    st = buf.view(4096, 32)[: B // 16].cpu().numpy().astype("float64")
    t0 = st[:, 0].min()
    print(f"blocks {len(st)} span {(st[:, 31] - t0).max():.0f} clk start spread {(st[:, 0] - t0).max():.0f} "
          f"median life {np.median(st[:, 31] - st[:, 0]):.0f}")
    names = {1: "stage X", 2: "fwd L0", 3: "fwd L1", 4: "fwd L2", 6: "CE", 9: "bwd L2", 8: "bwd L1", 7: "bwd L0 (dx)",
             31: "end"}
    order = [0, 1, 2, 3, 4, 6, 9, 8, 7, 31]
    for a, b in zip(order[:-1], order[1:]):
        print(f"   {names[b]:12s} {np.median(st[:, b] - st[:, a]):8.0f}")


if __name__ == "__main__":
    main()
