#!/usr/bin/env python3
"""Phase breakdown of the reference CNN's fused conv-block backward (csrc/kcnn_fused.hip kcnn_bwd_kernel)
from in-kernel s_memtime stamps (thread 0 of every workgroup, its first two images), B = 1024 by default.
Slots: 0 image start, 1 dY2 expanded, 2 barrier, 3 conv1 recomputed, 4 barrier, 5 conv2 weight gradient,
6 dgrad weights loaded, 7 data gradient + conv1 weight gradient, 8 barrier.  Prints per-phase medians and
p90 per image (s_memtime: shader clocks) and the launch span."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distriflow_amd import native, ops  # noqa: E402
from distriflow_amd.data.synthetic import synthetic_mnist  # noqa: E402
from distriflow_amd.models.zoo import build_model  # noqa: E402

NAMES = ["dY2 expand", "barrier", "conv1 recompute", "barrier", "conv2 wgrad", "dgrad W load", "dgrad+conv1 wgrad",
         "barrier"]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    m = native.require()
    net = build_model("keras_cnn", device="cuda", seed=0)
    data, labels = synthetic_mnist(60000, seed=1, device="cuda")
    idx = torch.randperm(60000, device="cuda")[:B]
    x, y = ops.GatherRef(data, idx, 1 / 255.0, (28, 28, 1)), ops.LabelRef(labels, idx)
    for _ in range(20):
        net.compute_gradients(x, y)
    torch.cuda.synchronize()
    buf = torch.zeros(1024 * 32, dtype=torch.int64, device="cuda")
    m.kcnn_set_stamps(buf)
    for _ in range(3):  # the last one's stamps remain
        net.compute_gradients(x, y)
    torch.cuda.synchronize()
    m.kcnn_set_stamps(None)
    st = buf.view(1024, 2, 16).cpu().numpy().astype(np.int64)
    G = int((st[:, 0, 0] > 0).sum())
    st = st[:G]
    t0 = st[:, 0, 0].min()
    print(f"B={B}: {G} workgroups; span of the stamped images {st[:, :, 8].max() - t0} clocks (s_memtime)")
    for im in range(2):
        s = st[:, im]
        ok = s[:, 0] > 0
        s = s[ok]
        tot = s[:, 8] - s[:, 0]
        print(f"image {im}: {ok.sum()} workgroups, image time med {np.median(tot):.0f} p90 {np.percentile(tot, 90):.0f}")
        for k, name in enumerate(NAMES):
            d = s[:, k + 1] - s[:, k]
            print(f"  {name:<18} med {np.median(d):7.0f}  p90 {np.percentile(d, 90):7.0f}  "
                  f"share {np.median(d) / max(1, np.median(tot)) * 100:5.1f} %")
        gap = s[:, 0] - t0
        print(f"  start rel. to first: med {np.median(gap):.0f} max {gap.max():.0f}")


if __name__ == "__main__":
    main()
