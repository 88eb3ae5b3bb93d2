#!/usr/bin/env python3
"""Per-op GPU timing of the LeNet-5 / MNIST-CNN training step kernels (HIP events, median of N)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distriflow_amd import ops  # noqa: E402


def timeit(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="lenet5")
    ap.add_argument("-B", type=int, default=4096)
    args = ap.parse_args()
    from distriflow_amd.data.synthetic import synthetic_mnist, synthetic_cifar10
    from distriflow_amd.models.zoo import build_model

    net = build_model(args.model, "cuda")
    B = args.B
    if args.model == "resnet18_cifar":
        data, labels = synthetic_cifar10(8192, device="cuda")
    else:
        data, labels = synthetic_mnist(60000, device="cuda")
    idx = torch.randint(0, data.shape[0], (B,), device="cuda")
    x = ops.GatherRef(data, idx, 1 / 255, net.input_shape)
    if type(net.exec_layers[0]).__name__ != "FusedConvPool":  # only the fused first layer reads the dataset
        net.bind(B)
        x = x.materialise(net.x_buf)
    y = torch.empty(B, dtype=torch.int32, device="cuda")
    ops.gather_labels(labels, idx, y)
    net.compute_gradients(x, y)
    torch.cuda.synchronize()
    layers = net.exec_layers
    inputs = [x] + [l.out for l in layers[:-1]]
    douts = [l.dx for l in layers[1:]] + [net.dlogits]
    total = 0.0
    for i, l in enumerate(layers):
        xin = inputs[i]
        f = timeit(lambda: l.forward(xin, True))
        b = timeit(lambda: l.backward(douts[i].view_as(l.out) if douts[i] is not None else None))
        total += f + b
        print(f"{i:2d} {type(l).__name__:<16} {l.name:<14} fwd {f:8.1f} us  bwd {b:8.1f} us")
    t_ce = timeit(lambda: net.loss_and_grad(net.exec_layers[-1].out, y))
    t_sgd = timeit(lambda: net.store.sgd_step())
    print(f"softmax_ce {t_ce:.1f} us   sgd {t_sgd:.1f} us   layer total {total:.1f} us")
    full = timeit(lambda: (net.compute_gradients(x, y), net.store.sgd_step()), iters=30)
    print(f"full eager step {full:.1f} us  -> {B / full * 1e6 / 1e6:.2f} M img/s (eager, incl. launch overhead)")


if __name__ == "__main__":
    main()
