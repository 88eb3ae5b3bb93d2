"""Flat-variable checkpoint format of DistributedServerDynamicModel.

/root/reference/src/server/models.ts:198-267 (SURVEY §5.4 format B): ``<dir>/meta.json`` =
``{"meta": [{"shape": [...], "dtype": "float32"}, ...], "byteOffsets": [...]}`` and ``<dir>/data.bin``
= the raw little-endian buffers concatenated.  (The reference's ``load`` never assigns what it reads,
SURVEY §2.9 item 4 — here it does.)
"""
from __future__ import annotations

import json
import os
from typing import Sequence

import numpy as np
import torch

from ..protocol import dtype_name, serialize_var, torch_dtype, deserialize_var, SerializedVariable


def flat_serialize(tensors: Sequence[torch.Tensor]):
    """-> (meta dict, bytes)"""
    meta, offsets, blobs = [], [], []
    off = 0
    for t in tensors:
        s = serialize_var(t)
        meta.append({"shape": s.shape, "dtype": s.dtype})
        offsets.append(off)
        blobs.append(s.data)
        off += len(s.data)
    return {"meta": meta, "byteOffsets": offsets}, b"".join(blobs)


def flat_deserialize(meta: dict, data: bytes, device="cpu") -> list[torch.Tensor]:
    out = []
    offs = list(meta["byteOffsets"]) + [len(data)]
    for i, m in enumerate(meta["meta"]):
        out.append(deserialize_var(SerializedVariable(m["dtype"], m["shape"], data[offs[i]: offs[i + 1]]), device))
    return out


def save_flat(directory: str, tensors: Sequence[torch.Tensor]):
    os.makedirs(directory, exist_ok=True)
    meta, data = flat_serialize(tensors)
    with open(os.path.join(directory, "data.bin"), "wb") as f:
        f.write(data)
    tmp = os.path.join(directory, "meta.json.tmp")
    with open(tmp, "w") as f:
        json.dump(meta, f)
    os.replace(tmp, os.path.join(directory, "meta.json"))


def load_flat(directory: str, device="cpu") -> list[torch.Tensor]:
    with open(os.path.join(directory, "meta.json")) as f:
        meta = json.load(f)
    with open(os.path.join(directory, "data.bin"), "rb") as f:
        data = f.read()
    return flat_deserialize(meta, data, device)
