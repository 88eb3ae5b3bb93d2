#!/usr/bin/env python3
"""Yardstick (diagnostic only, not part of the framework): the same training step written in stock
PyTorch-ROCm (MIOpen convolutions, hipBLASLt GEMMs, bf16 autocast, channels_last), timed the same
way as bench.py, so our kernels have a local point of comparison.  Nothing in distriflow_amd uses it.

usage: python scripts/torch_yardstick.py --model resnet18_cifar --batch 256 --steps 30
"""
import argparse
import json
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Basic(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.b1 = nn.BatchNorm2d(cout)
        self.c2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.b2 = nn.BatchNorm2d(cout)
        self.sc = None
        if stride != 1 or cin != cout:
            self.sc = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        o = F.relu(self.b1(self.c1(x)))
        o = self.b2(self.c2(o))
        return F.relu(o + (self.sc(x) if self.sc is not None else x))


def resnet18():
    layers = [nn.Conv2d(3, 64, 3, 1, 1, bias=False), nn.BatchNorm2d(64), nn.ReLU()]
    cin = 64
    for f, s in [(64, 1), (128, 2), (256, 2), (512, 2)]:
        layers += [Basic(cin, f, s), Basic(f, f, 1)]
        cin = f
    layers += [nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(512, 10)]
    return nn.Sequential(*layers)


def lenet5():
    return nn.Sequential(nn.Conv2d(1, 6, 5, padding=2), nn.ReLU(), nn.MaxPool2d(2), nn.Conv2d(6, 16, 5), nn.ReLU(),
                         nn.MaxPool2d(2), nn.Flatten(), nn.Linear(400, 120), nn.ReLU(), nn.Linear(120, 84), nn.ReLU(),
                         nn.Linear(84, 10))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18_cifar")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda")
    if args.model == "resnet18_cifar":
        net, shape = resnet18(), (3, 32, 32)
    else:
        net, shape = lenet5(), (1, 28, 28)
    net = net.to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(net.parameters(), lr=0.01)
    x = torch.randn(args.batch, *shape, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (args.batch,), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(net(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    print(json.dumps({"yardstick": "stock PyTorch-ROCm eager (MIOpen/hipBLASLt, bf16 autocast, channels_last)",
                      "model": args.model, "batch": args.batch, "ms_per_step": round(dt * 1e3, 3),
                      "images_per_s": round(args.batch / dt, 1)}))


if __name__ == "__main__":
    main()
