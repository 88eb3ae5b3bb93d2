"""Synthetic datasets with the exact shapes of the reference's workloads (no network, no downloads).

MNIST-shaped: 60,000 x 28x28x1 uint8 + labels in [0, 10) (/root/reference/experiment/mnist/mnist_data.ts:7-10).
CIFAR-10-shaped: 50,000 x 32x32x3 uint8.  Images are class prototypes plus noise, so a model can
actually learn them (used by convergence tests); benchmarks only need the shapes.
"""
from __future__ import annotations

import torch


def synthetic_images(n: int, shape: tuple, num_classes: int = 10, seed: int = 0, noise: float = 40.0,
                     device="cpu"):
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    protos = torch.rand((num_classes,) + tuple(shape), generator=g) * 255.0
    labels = torch.randint(0, num_classes, (n,), generator=g, dtype=torch.int64)
    out = torch.empty((n,) + tuple(shape), dtype=torch.uint8)
    step = 8192
    for s in range(0, n, step):
        lab = labels[s: s + step]
        img = protos[lab] + torch.randn((lab.numel(),) + tuple(shape), generator=g) * noise
        out[s: s + step] = img.clamp_(0, 255).to(torch.uint8)
    return out.to(device), labels.to(torch.int32).to(device)


def synthetic_mnist(n: int = 60000, seed: int = 0, device="cpu"):
    return synthetic_images(n, (28, 28, 1), 10, seed, device=device)


def synthetic_cifar10(n: int = 50000, seed: int = 0, device="cpu"):
    return synthetic_images(n, (32, 32, 3), 10, seed, device=device)


def non_iid_shards(labels: torch.Tensor, num_clients: int, classes_per_client: int = 2, seed: int = 0):
    """Pathological non-IID split (McMahan et al.): sort by label, cut into 2*clients shards, give each
    client ``classes_per_client`` shards.  Returns a list of index tensors."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    order = torch.argsort(labels.cpu().long() * labels.numel() + torch.randperm(labels.numel(), generator=g))
    nshards = num_clients * classes_per_client
    shards = list(torch.chunk(order, nshards))
    perm = torch.randperm(nshards, generator=g).tolist()
    out = []
    for c in range(num_clients):
        mine = [shards[perm[c * classes_per_client + j]] for j in range(classes_per_client)]
        out.append(torch.cat(mine))
    return out
