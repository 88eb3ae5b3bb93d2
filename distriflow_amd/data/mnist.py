"""MNIST IDX reader (reference: /root/reference/experiment/mnist/mnist_data.ts:20-72).

Big-endian IDX headers with magic 0x803 (images) / 0x801 (labels); images -> uint8 [N, rows, cols, 1]
(kept as uint8: the engine casts on the fly inside the first layer), labels -> int32 [N].  The
reference one-hot encodes labels (tf.oneHot(labels, 10)); the fused softmax-CE kernel takes class
indices directly, ``one_hot`` is provided for API parity.  No data ships with the reference or this
repo (no network): loaders take explicit paths, synthetic data is in :mod:`.synthetic`.
"""
from __future__ import annotations

import gzip
import os
import struct

import numpy as np
import torch


def _open(path):
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def read_idx_images(path: str) -> torch.Tensor:
    with _open(path) as f:
        magic, n, rows, cols = struct.unpack(">iiii", f.read(16))
        if magic != 0x00000803:
            raise ValueError(f"Training images file has invalid magic number 0x00000803 !== {magic:x}")
        data = np.frombuffer(f.read(n * rows * cols), dtype=np.uint8)
    return torch.from_numpy(data.copy()).view(n, rows, cols, 1)


def read_idx_labels(path: str) -> torch.Tensor:
    with _open(path) as f:
        magic, n = struct.unpack(">ii", f.read(8))
        if magic != 0x00000801:
            raise ValueError(f"Training labels file has invalid magic number 0x00000801 !== {magic:x}")
        data = np.frombuffer(f.read(n), dtype=np.uint8)
    return torch.from_numpy(data.astype(np.int32))


def load_mnist(data_dir: str, split: str = "train"):
    pre = "train" if split == "train" else "t10k"
    cand = lambda s: [os.path.join(data_dir, f"{pre}-{s}"), os.path.join(data_dir, f"{pre}-{s}.gz")]
    imgs = next((p for p in cand("images-idx3-ubyte") if os.path.exists(p)), None)
    labs = next((p for p in cand("labels-idx1-ubyte") if os.path.exists(p)), None)
    if imgs is None or labs is None:
        raise FileNotFoundError(f"MNIST {split} IDX files not found in {data_dir}")
    x, y = read_idx_images(imgs), read_idx_labels(labs)
    if x.shape[0] != y.shape[0]:
        raise ValueError(f"{x.shape[0]} images but {y.shape[0]} labels")
    return x, y


def write_idx(path_images: str, path_labels: str, x: torch.Tensor, y: torch.Tensor):
    """Inverse of the readers (used by tests to round-trip the format)."""
    n, r, c = x.shape[0], x.shape[1], x.shape[2]
    with open(path_images, "wb") as f:
        f.write(struct.pack(">iiii", 0x803, n, r, c))
        f.write(x.to(torch.uint8).contiguous().numpy().tobytes())
    with open(path_labels, "wb") as f:
        f.write(struct.pack(">ii", 0x801, n))
        f.write(y.to(torch.uint8).contiguous().numpy().tobytes())


def one_hot(labels: torch.Tensor, num_classes: int = 10) -> torch.Tensor:
    return torch.nn.functional.one_hot(labels.long(), num_classes).float()
