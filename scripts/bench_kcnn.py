#!/usr/bin/env python3
"""Time the fused reference-CNN conv block (csrc/kcnn_fused.hip) at B=1024: forward, and the backward
with parts skipped (kcnn_set_debug) to attribute its time."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distriflow_amd import native, ops  # noqa: E402
from distriflow_amd.data.synthetic import synthetic_mnist  # noqa: E402
from distriflow_amd.models.zoo import build_model  # noqa: E402


def timed(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    m = native.require()
    net = build_model("keras_cnn", device="cuda", seed=0)
    blk = net.exec_layers[0]
    net.bind(B)
    data, labels = synthetic_mnist(60000, seed=1, device="cuda")
    idx = torch.randperm(60000, device="cuda")[:B]
    x = ops.GatherRef(data, idx, 1 / 255.0, (28, 28, 1))
    dy = (torch.randn(B, 12, 12, 32, device="cuda") * 1e-3).to(torch.bfloat16)
    for mask, name in [(0, "fwd (all)"), (32, "- stores"), (16, "- conv2"), (48, "- conv2+st"), (112, "- +conv1")]:
        m.kcnn_set_debug(mask)
        print(f"{name:<12} {timed(lambda: blk.forward(x, True)):8.1f} us")
    m.kcnn_set_debug(0)
    blk.forward(x, True)
    for mask, name in [(0, "bwd (all)"), (1, "- conv2 wgrad"), (2, "- dgrad+c1"), (3, "- both"), (7, "- +conv1"),
                       (15, "- +expand")]:
        m.kcnn_set_debug(mask)
        print(f"{name:<12} {timed(lambda: blk.backward(dy)):8.1f} us")
    m.kcnn_set_debug(0)


if __name__ == "__main__":
    main()
