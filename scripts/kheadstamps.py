#!/usr/bin/env python3
"""Phase breakdown of the reference CNN's dense-head launch (csrc/khead.hip) from in-kernel s_memtime
stamps (thread 0 of every workgroup, first job), B=1024 by default.  Slots: 0 job start, 1 P staged,
2 P^T written, 3 Z1 partial done, 4 ticket, 5 owner done (owners only), 6 dZ1 available, 7 dP in LDS,
8 end; slot 15 = owner flag.  Prints per-phase medians (owners / waiters) and the launch timeline
relative to the earliest workgroup start."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distriflow_amd import native, ops  # noqa: E402
from distriflow_amd.data.synthetic import synthetic_mnist  # noqa: E402
from distriflow_amd.models.zoo import build_model  # noqa: E402

NAMES = ["stage P", "P^T", "Z1 partial", "ticket", "owner / wait", "dgrad", "dP store"]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    m = native.require()
    net = build_model("keras_cnn", device="cuda", seed=0)
    assert net.khead
    data, labels = synthetic_mnist(60000, seed=1, device="cuda")
    idx = torch.randperm(60000, device="cuda")[:B]
    x, y = ops.GatherRef(data, idx, 1 / 255.0, (28, 28, 1)), ops.LabelRef(labels, idx)
    for _ in range(5):
        net.compute_gradients(x, y)
    torch.cuda.synchronize()
    buf = torch.zeros(1024 * 16, dtype=torch.int64, device="cuda")
    m.khead_set_stamps(buf)
    net.compute_gradients(x, y)
    torch.cuda.synchronize()
    m.khead_set_stamps(None)
    st = buf.view(1024, 16).cpu().numpy().astype(np.int64)
    G = int((st[:, 0] > 0).sum())
    st = st[:G]
    owner = st[:, 15] == 1
    t0 = st[:, 0].min()
    print(f"B={B}: {G} workgroups, {int(owner.sum())} owners; launch span {st[:, 8].max() - t0} clocks")
    # phase k = slot k+1 - slot k, except owner/wait = slot 6 - slot 4 (owners include their owner work)
    cols = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 6), (6, 7), (7, 8)]
    for name, (a, b) in zip(NAMES, cols):
        d = st[:, b] - st[:, a]
        print(f"  {name:<14} all med {np.median(d):7.0f} p90 {np.percentile(d, 90):7.0f} | owners med "
              f"{np.median(d[owner]):7.0f} | waiters med {np.median(d[~owner]):7.0f}")
    if owner.any():
        d = st[owner, 5] - st[owner, 4]
        print(f"  owner work     med {np.median(d):7.0f} p90 {np.percentile(d, 90):7.0f}")
    if (st[:, 9] > 0).any():
        za = st[:, 9] - st[:, 6]
        wt = st[:, 10] - st[:, 9]
        print(f"  dgrad split: dZ1 loads med {np.median(za):7.0f} | then W1^T loads med {np.median(wt):7.0f} | "
              f"MFMA + epilogue med {np.median(st[:, 7] - st[:, 10]):7.0f}")
    xcc = st[:, 14] & 0xF
    print(f"  XCC_ID == blockIdx % 8 for {(xcc == (np.arange(G) % 8)).mean() * 100:.0f}% of workgroups; "
          f"distinct (blockIdx%8 -> XCC) pairs {len(set(zip(np.arange(G) % 8, xcc)))}")
    print("timeline (clocks from the first start): slot median / max")
    for k in range(9):
        rel = st[:, k] - t0
        print(f"  slot {k}: med {np.median(rel):8.0f}  max {rel.max():8.0f}")


if __name__ == "__main__":
    main()
