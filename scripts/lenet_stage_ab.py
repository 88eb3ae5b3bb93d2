#!/usr/bin/env python3
"""A/B of the LeNet-5 train kernel's staging: batch rows read through the index vector (uint8 dataset +
idx: the index load, then the dependent row loads) against a pre-gathered bf16 batch (no index load).
Eager compute_gradients (train + reduce launches), B = 4096, hipEvent timing over 200 steps."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distriflow_amd import ops  # noqa: E402
from distriflow_amd.data.synthetic import synthetic_mnist  # noqa: E402
from distriflow_amd.models.zoo import build_model  # noqa: E402


def main():
    B = 4096
    net = build_model("lenet5", device="cuda", seed=0)
    data, labels = synthetic_mnist(60000, seed=1, device="cuda")
    idx = torch.randperm(60000, device="cuda")[:B]
    xg, yg = ops.GatherRef(data, idx, 1 / 255.0, (28, 28, 1)), ops.LabelRef(labels, idx)
    xb = (data.index_select(0, idx).float() / 255.0).to(torch.bfloat16).reshape(B, 28, 28, 1).contiguous()
    yb = labels.index_select(0, idx).contiguous()

    def wall(x, y, n=200):
        for _ in range(5):
            net.compute_gradients(x, y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            net.compute_gradients(x, y)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n * 1e3

    for rep in range(2):
        print(f"idx path {wall(xg, yg):.2f} us/step; pre-gathered bf16 {wall(xb, yb):.2f} us/step", flush=True)


if __name__ == "__main__":
    main()
