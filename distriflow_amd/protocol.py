"""Wire protocol: serialised tensors, the reference's message types, and their binary encoding.

Reference: /root/reference/src/common/utils.ts:
  * ``SerializedVariable = {dtype, shape, data: ArrayBuffer}`` with dtype in {float32, int32, bool}
    (utils.ts:7-17) — here also bfloat16 / uint8 / int64 / float16;
  * ``serializeVar(s)`` = device->host readback + copy (utils.ts:32-51), ``deserializeVar(s)``
    (utils.ts:77-84), ``stackSerialized`` = per-weight concatenation into [numUpdates, ...shape]
    (utils.ts:53-75);
  * messages ``ModelMsg{version, vars}``, ``GradientMsg{version, vars}``, ``DataMsg{batch, epoch, x, y}``,
    ``UploadMsg{clientId, gradients?, batch?, metrics?}``, ``DownloadMsg{model, hyperparams, data?}``
    and ``Events.Download/Upload`` (utils.ts:115-155).

On the MI355X data plane tensors never go through host memory: a message is encoded as ONE fixed
size int64 header tensor (kind, ids, version, counts, payload dtypes/sizes) plus up to four flat
payload tensors sent with RCCL/gloo point-to-point; small JSON side data (client id, hyper-params,
version strings) rides as a uint8 payload.  See :mod:`distriflow_amd.parallel.transport`.
"""
from __future__ import annotations

import json
import struct
from dataclasses import dataclass, field
from enum import Enum
from typing import Any, Optional, Sequence

import numpy as np
import torch


class Events(str, Enum):
    Download = "downloadVars"
    Upload = "uploadVars"


_DTYPES = {
    "float32": torch.float32,
    "int32": torch.int32,
    "bool": torch.bool,
    "bfloat16": torch.bfloat16,
    "float16": torch.float16,
    "uint8": torch.uint8,
    "int64": torch.int64,
}
_NAMES = {v: k for k, v in _DTYPES.items()}


def dtype_name(dt: torch.dtype) -> str:
    if dt not in _NAMES:
        raise ValueError(f"unsupported dtype {dt}")
    return _NAMES[dt]


def torch_dtype(name: str) -> torch.dtype:
    if name not in _DTYPES:
        raise ValueError(f"unsupported dtype {name!r}")
    return _DTYPES[name]


@dataclass
class SerializedVariable:
    dtype: str
    shape: list
    data: bytes

    def nbytes(self) -> int:
        return len(self.data)


def serialize_var(t: torch.Tensor) -> SerializedVariable:
    """Device -> host readback of one tensor (a copy, never a view of engine memory)."""
    t = t.detach()
    name = dtype_name(t.dtype)
    host = t.contiguous().cpu()
    if t.dtype == torch.bfloat16:
        raw = host.view(torch.int16).numpy().tobytes()
    elif t.dtype == torch.bool:
        raw = host.to(torch.uint8).numpy().tobytes()
    else:
        raw = host.numpy().tobytes()
    return SerializedVariable(name, list(t.shape), raw)


def serialize_vars(vs: Sequence[torch.Tensor]) -> list[SerializedVariable]:
    return [serialize_var(v) for v in vs]


def serialized_to_array(s: SerializedVariable) -> np.ndarray:
    n = int(np.prod(s.shape)) if len(s.shape) else 1
    if s.dtype == "bfloat16":
        return np.frombuffer(s.data, dtype=np.int16, count=n).reshape(s.shape)
    if s.dtype == "bool":
        return np.frombuffer(s.data, dtype=np.uint8, count=n).reshape(s.shape)
    np_dt = {"float32": np.float32, "int32": np.int32, "float16": np.float16, "uint8": np.uint8,
             "int64": np.int64}[s.dtype]
    return np.frombuffer(s.data, dtype=np_dt, count=n).reshape(s.shape)


def deserialize_var(s: SerializedVariable, device="cpu") -> torch.Tensor:
    arr = serialized_to_array(s).copy()
    t = torch.from_numpy(arr)
    if s.dtype == "bfloat16":
        t = t.view(torch.bfloat16)
    elif s.dtype == "bool":
        t = t.to(torch.bool)
    return t.to(device)


def deserialize_vars(vs: Sequence[SerializedVariable], device="cpu") -> list[torch.Tensor]:
    return [deserialize_var(v, device) for v in vs]


def stack_serialized(updates: Sequence[Sequence[SerializedVariable]]) -> list[SerializedVariable]:
    """[numUpdates][numWeights] -> per weight one SerializedVariable of shape [numUpdates, ...shape]."""
    if not updates:
        return []
    n_up = len(updates)
    out = []
    for w in range(len(updates[0])):
        first = updates[0][w]
        parts = []
        for u in range(n_up):
            v = updates[u][w]
            if v.dtype != first.dtype or list(v.shape) != list(first.shape):
                raise ValueError(f"update {u} weight {w}: {v.dtype}{v.shape} != {first.dtype}{first.shape}")
            parts.append(v.data)
        out.append(SerializedVariable(first.dtype, [n_up] + list(first.shape), b"".join(parts)))
    return out


# ------------------------------------------------------------------------------------------ messages
@dataclass
class ModelMsg:
    version: str
    vars: Any  # list[SerializedVariable] | flat torch.Tensor (device)


@dataclass
class GradientMsg:
    version: str
    vars: Any


@dataclass
class DataMsg:
    batch: int
    epoch: int
    x: Any = None   # tensor / SerializedVariable, or None when workers hold the data (indices only)
    y: Any = None
    start: int = 0  # row range of the batch in the (worker-resident) dataset
    size: int = 0
    indices: Any = None  # example ids of a shuffled batch (list of int) when only ids travel


@dataclass
class UploadMsg:
    client_id: str
    gradients: Optional[GradientMsg] = None
    batch: Optional[int] = None
    epoch: Optional[int] = None
    metrics: Optional[list] = None
    num_examples: int = 0

    # reference spelling
    @property
    def clientId(self):
        return self.client_id


@dataclass
class DownloadMsg:
    model: ModelMsg
    hyperparams: dict = field(default_factory=dict)
    data: Optional[DataMsg] = None


# ------------------------------------------------------------------------------------------ binary header
# int64[HEADER_LEN]: [magic, kind, src, version_id, batch, epoch, n_metrics, num_examples,
#                     n_payloads, (dtype_code, numel) x 4, metrics (float64 bits) x 8, reserved...]
HEADER_LEN = 32
MAGIC = 0x44464C57  # 'DFLW'
MAX_PAYLOADS = 4
MAX_METRICS = 8


class Kind:
    HELLO = 1        # client -> server: I joined (json: client_id)
    DOWNLOAD = 2     # server -> client: model (+ data / batch assignment, + json: version, hyperparams)
    UPLOAD = 3       # client -> server: gradients / weights (+ batch, metrics)
    BYE = 4          # either direction: leave / shut down
    ACK = 5          # server -> client: upload received (reference ack(true))
    DONE = 6         # server -> client: dataset exhausted, stop


_DT_CODES = {torch.float32: 1, torch.bfloat16: 2, torch.int32: 3, torch.int64: 4, torch.uint8: 5, torch.float16: 6,
             torch.bool: 7}
_CODE_DT = {v: k for k, v in _DT_CODES.items()}


def encode_header(kind: int, src: int, version_id: int = 0, batch: int = -1, epoch: int = -1,
                  metrics: Optional[Sequence[float]] = None, num_examples: int = 0,
                  payloads: Sequence[torch.Tensor] = ()) -> torch.Tensor:
    h = torch.zeros(HEADER_LEN, dtype=torch.int64)
    ms = list(metrics or [])[:MAX_METRICS]
    if len(payloads) > MAX_PAYLOADS:
        raise ValueError("too many payloads")
    h[0], h[1], h[2], h[3], h[4], h[5] = MAGIC, kind, src, version_id, batch, epoch
    h[6], h[7], h[8] = len(ms), num_examples, len(payloads)
    for i, p in enumerate(payloads):
        h[9 + 2 * i] = _DT_CODES[p.dtype]
        h[10 + 2 * i] = p.numel()
    for i, m in enumerate(ms):
        h[17 + i] = struct.unpack("<q", struct.pack("<d", float(m)))[0]
    return h


def decode_header(h: torch.Tensor) -> dict:
    v = h.cpu().tolist()
    if v[0] != MAGIC:
        raise ValueError(f"bad message magic {v[0]:#x}")
    n_m = v[6]
    n_p = v[8]
    return {
        "kind": v[1], "src": v[2], "version_id": v[3], "batch": v[4], "epoch": v[5],
        "metrics": [struct.unpack("<d", struct.pack("<q", v[17 + i]))[0] for i in range(n_m)],
        "num_examples": v[7],
        "payloads": [(_CODE_DT[v[9 + 2 * i]], v[10 + 2 * i]) for i in range(n_p)],
    }


def json_payload(obj) -> torch.Tensor:
    return torch.frombuffer(bytearray(json.dumps(obj).encode()), dtype=torch.uint8).clone()


def payload_json(t: torch.Tensor):
    return json.loads(bytes(t.cpu().numpy().tobytes()).decode())
