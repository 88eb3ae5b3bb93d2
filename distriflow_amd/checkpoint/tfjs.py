"""tf.js ``LayersModel`` checkpoint format (model.json + binary weight shards), read and write.

What the reference saves with ``model.save('file://<dir>')`` / loads with ``tf.loadLayersModel``
(/root/reference/src/server/models.ts:132-150, SURVEY §5.4 formats A and C):

  model.json = {"modelTopology": {... Keras Sequential config ...},
                "weightsManifest": [{"paths": ["weights.bin"], "weights": [{"name", "shape", "dtype"}, ...]}],
                "format": "layers-model", "generatedBy": ..., "convertedBy": ...}
  weights.bin = little-endian float32 values of every weight, concatenated in manifest order.

Keras layouts are converted at this boundary only: Conv2D kernel HWIO [kh][kw][cin][cout] <-> engine
OHWI [cout][kh][kw][cin]; Dense kernel [in][out] <-> engine [out][in]; BatchNormalization
gamma/beta(/moving_mean/moving_variance).  Weights are always stored fp32 on disk even when training
runs in bf16.  Multi-shard manifests (``group1-shard1of1`` ... as in model.json:1) are read too.
"""
from __future__ import annotations

import json
import os
from typing import Optional

import numpy as np
import torch

from ..models.keras import keras_config_from_layers
from ..models.layers import BatchNorm, Conv2D, ConvPoolGemm, Dense, FusedConvPool, KerasConvBlock, ResidualBlock

FORMAT = "layers-model"
GENERATED_BY = "distriflow_amd"


def _engine_to_keras(spec_name: str, value: torch.Tensor, layer) -> np.ndarray:
    v = value.detach().float().cpu()
    conv = isinstance(layer, (Conv2D, FusedConvPool, ConvPoolGemm, KerasConvBlock))
    if spec_name.endswith("/kernel") and conv:
        return v.permute(1, 2, 3, 0).contiguous().numpy()          # OHWI -> HWIO
    if spec_name.endswith("/kernel") and isinstance(layer, Dense):
        return v.t().contiguous().numpy()                          # [out][in] -> [in][out]
    return v.contiguous().numpy()


def _keras_to_engine(spec_name: str, arr: np.ndarray, layer, engine_shape) -> torch.Tensor:
    t = torch.from_numpy(np.ascontiguousarray(arr)).float()
    conv = isinstance(layer, (Conv2D, FusedConvPool, ConvPoolGemm, KerasConvBlock))
    if spec_name.endswith("/kernel") and conv:
        t = t.permute(3, 0, 1, 2)                                  # HWIO -> OHWI
    elif spec_name.endswith("/kernel") and isinstance(layer, Dense):
        t = t.t()
    return t.contiguous().reshape(engine_shape)


def _weight_layers(net):
    """[(spec_name, layer)] in parameter order, plus BN moving statistics entries."""
    out = []
    for l in net.exec_layers:
        subs = l.sublayers() if hasattr(l, "sublayers") else [l]
        for s in subs:
            for spec in s.specs():
                out.append((spec.name, s))
            if isinstance(s, BatchNorm):
                out.append((f"{s.name}/moving_mean", s))
                out.append((f"{s.name}/moving_variance", s))
    return out


def _bn_stat(layer: BatchNorm, which: str, device) -> torch.Tensor:
    if not hasattr(layer, "run_mean"):
        layer.run_mean = torch.zeros(layer.C, device=device)
        layer.run_var = torch.ones(layer.C, device=device)
    return layer.run_mean if which == "moving_mean" else layer.run_var


def save_layers_model(net, directory: str, topology: Optional[dict] = None, shard_bytes: int = 0) -> str:
    """Write ``directory/model.json`` + weight shard(s).  Returns the model.json path."""
    os.makedirs(directory, exist_ok=True)
    entries = []
    blobs = []
    for name, layer in _weight_layers(net):
        if name.endswith("/moving_mean") or name.endswith("/moving_variance"):
            arr = _bn_stat(layer, name.rsplit("/", 1)[1], net.device).float().cpu().numpy()
        else:
            arr = _engine_to_keras(name, net.store[name], layer)
        arr = np.ascontiguousarray(arr, dtype="<f4")
        entries.append({"name": name, "shape": list(arr.shape), "dtype": "float32"})
        blobs.append(arr.tobytes())
    data = b"".join(blobs)
    if shard_bytes and len(data) > shard_bytes:
        n = (len(data) + shard_bytes - 1) // shard_bytes
        paths = [f"group1-shard{i + 1}of{n}.bin" for i in range(n)]
        for i, p in enumerate(paths):
            with open(os.path.join(directory, p), "wb") as f:
                f.write(data[i * shard_bytes:(i + 1) * shard_bytes])
    else:
        paths = ["weights.bin"]
        with open(os.path.join(directory, "weights.bin"), "wb") as f:
            f.write(data)
    if topology is None:
        topology = getattr(net, "topology", None)
    if topology is None:
        topology = {"model_config": keras_config_from_layers(net.layers_all, net.input_shape, net.name),
                    "keras_version": "2.1.4", "backend": "tensorflow"}
    doc = {
        "modelTopology": topology,
        "weightsManifest": [{"paths": paths, "weights": entries}],
        "format": FORMAT,
        "generatedBy": GENERATED_BY,
        "convertedBy": None,
    }
    path = os.path.join(directory, "model.json")
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(doc, f)
    os.replace(tmp, path)
    return path


def read_manifest_weights(model_json: str) -> dict:
    """-> {weight name: np.ndarray (Keras layout)} for every manifest group (shards concatenated)."""
    with open(model_json) as f:
        doc = json.load(f)
    base = os.path.dirname(model_json)
    out = {}
    for group in doc.get("weightsManifest", []):
        raw = b""
        for p in group["paths"]:
            with open(os.path.join(base, p), "rb") as f:
                raw += f.read()
        off = 0
        for w in group["weights"]:
            dt = {"float32": "<f4", "int32": "<i4", "bool": "u1"}[w.get("dtype", "float32")]
            n = int(np.prod(w["shape"])) if w["shape"] else 1
            size = n * np.dtype(dt).itemsize
            out[w["name"]] = np.frombuffer(raw[off: off + size], dtype=dt).reshape(w["shape"]).copy()
            off += size
    return out


def load_layers_model_weights(net, model_json: str, strict: bool = True):
    """Load weights of a tf.js LayersModel checkpoint into an engine model (layout conversion included)."""
    weights = read_manifest_weights(model_json)
    missing = []
    for name, layer in _weight_layers(net):
        if name not in weights:
            missing.append(name)
            continue
        if name.endswith("/moving_mean") or name.endswith("/moving_variance"):
            _bn_stat(layer, name.rsplit("/", 1)[1], net.device).copy_(torch.from_numpy(weights[name]))
            continue
        t = _keras_to_engine(name, weights[name], layer, net.store.spec(name).shape)
        net.store[name].copy_(t.to(net.store.master.device))
    if missing and strict:
        raise KeyError(f"checkpoint {model_json} lacks weights {missing}")
    net.store.refresh_compute()
    return net


def load_topology(model_json: str) -> dict:
    with open(model_json) as f:
        return json.load(f)["modelTopology"]
