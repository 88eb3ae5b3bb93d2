"""DistriWorker roles: the worker side of FedSGD, asynchronous SGD and federated averaging.

Reference: ``AbstractClient`` (/root/reference/src/client/abstract_client.ts:1-181), ``FederatedClient``
(federated_client.ts:22-149), ``AsynchronousSGDClient`` (asynchronousSGD_client.ts:8-85);
SURVEY §2.3 K4-K6, §3.2, §3.3.

Preserved behaviour: client identity = config clientId, else a persisted id, else uuid4; the first
Download must arrive within CONNECTION_TIMEOUT (10 s); ``model_version()`` is ``'unsynced'`` before it;
``DistributedUpdate(x, y)`` buffers examples and uploads one gradient per ``examplesPerUpdate`` of them,
tagged with the version it was computed on, optionally with pre-update metrics (``sendMetrics``);
weights change only through server downloads; per-version upload counters
(``num_updates`` / ``num_versions``); hyper-parameter precedence local config -> server -> defaults.

MI355X design: the example buffer is a preallocated device FIFO (``utils.tensors.ExampleRing``: no
per-call concat/slice reallocation), gradients are the engine's flat HBM buffer sent straight over RCCL, received weights are written into the flat
master buffer and the bf16 compute copies refreshed by one kernel.  The async worker can hold the
dataset itself (HBM resident) so only batch ids travel (``DataMsg.x is None``).
"""
from __future__ import annotations

import os
import time
import uuid
from typing import Callable, Optional

import torch

from ..config import DEFAULT_CLIENT_HYPERPARAMS, compile_args
from ..models.distri_model import ClientModel, is_client_model
from ..protocol import GradientMsg, Kind, UploadMsg
from ..utils.logging import Logger
from .transport import Message, Transport

CONNECTION_TIMEOUT = 10.0
UPLOAD_TIMEOUT = 5.0
COOKIE_NAME = "Distributed-learner-uuid"


def _persisted_client_id() -> Optional[str]:
    """Browser-cookie equivalent: a per-user file (reference getCookie/setCookie, client/utils.ts:49-64)."""
    p = os.path.join(os.path.expanduser("~"), ".distriflow_client_id")
    try:
        if os.path.exists(p):
            with open(p) as f:
                v = f.read().strip()
                return v or None
        v = str(uuid.uuid4())
        with open(p, "w") as f:
            f.write(v)
        return v
    except OSError:
        return None


class AbstractWorker:
    role = "Distributed Client"

    def __init__(self, transport: Transport, model, config: Optional[dict] = None, server_rank: int = 0):
        config = dict(config or {})
        allowed = {"modelCompileConfig", "hyperparams", "verbose", "clientId", "sendMetrics", "metricsFile",
                   "connectionTimeout", "ack"}
        for k in config:
            if k not in allowed:
                raise ValueError(f'Unrecognized client config key "{k}"')
        if not is_client_model(model):
            model = ClientModel(model, config.get("modelCompileConfig") or {})
        self.transport = transport
        self.server_rank = server_rank
        self.model = model
        self.verbose = bool(config.get("verbose"))
        self.send_metrics = bool(config.get("sendMetrics"))
        self.client_id = config.get("clientId") or _persisted_client_id() or str(uuid.uuid4())
        self.hyperparams = dict(config.get("hyperparams") or {})
        self.logger = Logger(self.role, self.verbose, config.get("metricsFile"))
        self.connection_timeout = float(config.get("connectionTimeout", CONNECTION_TIMEOUT))
        self.ack = bool(config.get("ack", False))
        self.msg: Optional[Message] = None
        self.version_callbacks: list[Callable] = [lambda v1, v2: self.log(f"Updated model: {v1} -> {v2}")]
        self.upload_callbacks: list[Callable] = []
        self.version_update_counts: dict = {}
        self.done = False
        self._connected = False

    # ------------------------------------------------------------------ reference API
    def model_version(self) -> str:
        return "unsynced" if self.msg is None else self.msg.meta.get("version", str(self.msg.version_id))

    modelVersion = model_version

    def on_new_version(self, cb):
        self.version_callbacks.append(cb)

    def on_upload(self, cb):
        self.upload_callbacks.append(cb)

    onNewVersion = on_new_version
    onUpload = on_upload

    def evaluate(self, x, y):
        return self.model.evaluate(x, y)

    def predict(self, x):
        return self.model.predict(x)

    def num_updates(self) -> int:
        return sum(self.version_update_counts.values())

    def num_versions(self) -> int:
        return len(self.version_update_counts)

    numUpdates = num_updates
    numVersions = num_versions

    def dispose(self):
        if self._connected:
            self.transport.send(self.server_rank, Message(Kind.BYE, meta={"client_id": self.client_id}))
            self._connected = False
        self.log("Disconnected")

    @property
    def input_shape(self):
        return self.model.input_shape

    @property
    def output_shape(self):
        return self.model.output_shape

    def log(self, *args):
        self.logger.log(*args)

    def time(self, msg, fn):
        return self.logger.time(msg, fn)

    def hyperparam(self, key: str):
        if self.hyperparams.get(key) is not None:
            return self.hyperparams[key]
        server = (self.msg.meta.get("hyperparams") if self.msg else None) or {}
        if server.get(key) is not None:
            return server[key]
        return DEFAULT_CLIENT_HYPERPARAMS[key]

    # ------------------------------------------------------------------ plumbing
    def _apply_download(self, m: Message):
        old = self.model_version()
        self.msg = m
        self.model.set_flat(m.tensors[0])
        new = self.model_version()
        self.version_update_counts.setdefault(new, 0)
        for cb in self.version_callbacks:
            cb(None if old == "unsynced" else old, new)

    def connect(self):
        self.transport.send(self.server_rank, Message(Kind.HELLO, meta={"client_id": self.client_id}))
        t0 = time.perf_counter()
        while True:
            m = self.transport.recv(0.05)
            if m is not None:
                if m.kind == Kind.DOWNLOAD:
                    self._connected = True
                    return m
                if m.kind == Kind.DONE:
                    self._connected = True
                    self.done = True
                    return None
            if time.perf_counter() - t0 > self.connection_timeout:
                raise TimeoutError(f"no model download from the server within {self.connection_timeout:.0f}s")

    def setup(self):
        self.time("Initial model setup", self.model.setup)
        m = self.time("Download weights from server", self.connect)
        if m is not None:
            self._apply_download(m)

    def poll(self, timeout: float = 0.0) -> Optional[Message]:
        """Process pending server messages; returns the last DOWNLOAD handled (if any)."""
        last = None
        while True:
            m = self.transport.recv(timeout)
            timeout = 0.0
            if m is None:
                return last
            if m.kind == Kind.DOWNLOAD:
                self._apply_download(m)
                last = m
            elif m.kind in (Kind.DONE, Kind.BYE):
                self.done = True
                return last

    def _upload(self, grad: torch.Tensor, version_id: int, batch: int = -1, epoch: int = -1, metrics=None,
                num_examples: int = 0) -> UploadMsg:
        up = UploadMsg(self.client_id, GradientMsg(self.model_version(), grad), batch if batch >= 0 else None,
                       epoch if epoch >= 0 else None, metrics, num_examples)
        m = Message(Kind.UPLOAD, version_id=version_id, batch=batch, epoch=epoch, metrics=list(metrics or []),
                    num_examples=num_examples, tensors=[grad])
        self.time("Upload weights to server", lambda: self.transport.send(self.server_rank, m))
        if self.ack:
            self._wait_ack()
        for cb in self.upload_callbacks:
            cb(up)
        return up

    def _wait_ack(self):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < UPLOAD_TIMEOUT:
            m = self.transport.recv(0.01)
            if m is None:
                continue
            if m.kind == Kind.ACK:
                return
            if m.kind == Kind.DOWNLOAD:
                self._apply_download(m)
            elif m.kind in (Kind.DONE, Kind.BYE):
                self.done = True
                return
        raise TimeoutError("uploadVars timed out")


class FederatedClient(AbstractWorker):
    """Synchronous FedSGD worker: ``distributed_update(x, y)`` buffers examples and uploads one gradient
    per ``examplesPerUpdate`` examples, tagged with the current model version."""

    def setup(self):
        from ..utils.tensors import ExampleRing

        super().setup()
        shape = tuple(self.model.input_shape)
        dev = getattr(self.model, "device", "cpu")
        self.ring_x = ExampleRing(shape, torch.float32, dev)
        self.ring_y = ExampleRing((), torch.int64, dev)

    def distributed_update(self, x: torch.Tensor, y: torch.Tensor):
        dev = self.ring_x.buf.device
        y = y.to(dev)
        single = tuple(x.shape) == self.ring_x.unit_shape  # one example (reference addRows accepts both)
        if y.dim() > 1 or (single and y.numel() > 1):  # one-hot labels -> class ids
            y = y.argmax(dim=-1)
        self.ring_x.push(x.to(dev, torch.float32))
        self.ring_y.push(y.long().reshape(-1))
        if len(self.ring_x) != len(self.ring_y):
            raise ValueError("examples and labels must have the same number of rows")
        per = int(self.hyperparam("examplesPerUpdate"))
        while len(self.ring_x) >= per:
            self.poll(0.0)
            version = self.model_version()
            vid = self.msg.version_id if self.msg else 0
            xt, yt = self.ring_x.peek(per), self.ring_y.peek(per)
            metrics = self.model.evaluate(xt, yt) if self.send_metrics else None
            grad = self.time("Fit model", lambda: self.model.fit_flat(xt, yt))
            self._upload(grad, vid, metrics=metrics, num_examples=per)
            self.version_update_counts[version] = self.version_update_counts.get(version, 0) + 1
            self.ring_x.pop(per)
            self.ring_y.pop(per)
        self.poll(0.0)

    DistributedUpdate = distributed_update

    @property
    def x(self) -> torch.Tensor:
        """Buffered, not yet uploaded examples (oldest first): an independent copy.  The zero-copy view
        of the ring (``ring_x.peek``) is for the internal fit path only; a later push / peek or a ring
        growth would change a view under a caller that keeps it."""
        return self.ring_x.peek(len(self.ring_x)).clone()

    @property
    def y(self) -> torch.Tensor:
        return self.ring_y.peek(len(self.ring_y)).clone()

    def num_examples(self) -> int:
        return len(self.ring_x)

    def num_examples_per_update(self) -> int:
        return int(self.hyperparam("examplesPerUpdate"))

    def num_examples_remaining(self) -> int:
        return self.num_examples_per_update() - self.num_examples()


class AsynchronousSGDClient(AbstractWorker):
    """Asynchronous SGD worker: every download carries fresh weights + the next microbatch (shipped
    tensors, or a row range of the worker-resident dataset); compute its gradient and upload it with
    the version it was computed on, until the server says DONE."""

    def __init__(self, transport: Transport, model, config: Optional[dict] = None, server_rank: int = 0,
                 data: Optional[torch.Tensor] = None, labels: Optional[torch.Tensor] = None, data_scale: float = 1.0):
        super().__init__(transport, model, config)
        self.server_rank = server_rank
        self.data, self.labels, self.data_scale = data, labels, data_scale

    def _batch_tensors(self, m: Message):
        d = m.meta.get("data") or {}
        if len(m.tensors) >= 3:
            x, y = m.tensors[1], m.tensors[2]
            shape = tuple(self.model.input_shape)
            return x.reshape((-1,) + shape), y
        if self.data is None:
            raise RuntimeError("download carries no data and this worker holds no dataset")
        if d.get("indices") is not None:  # shuffled epoch: gather the permuted rows on the device
            idx = torch.tensor(d["indices"], dtype=torch.int64, device=self.data.device)
            x, y = self.data.index_select(0, idx), self.labels.index_select(0, idx.to(self.labels.device))
        else:
            s, n = int(d["start"]), int(d["size"])
            x, y = self.data[s: s + n], self.labels[s: s + n]
        if x.dtype == torch.uint8:
            x = x.float() * self.data_scale
        return x, y

    def distributed_update(self):
        m = self.msg
        if m is None or "data" not in m.meta:
            return
        x, y = self._batch_tensors(m)
        metrics = self.model.evaluate(x, y) if self.send_metrics else None
        grad = self.time("Fit model", lambda: self.model.fit_flat(x, y))
        version = self.model_version()
        self._upload(grad, m.version_id, batch=m.batch, epoch=m.epoch, metrics=metrics, num_examples=int(y.shape[0]))
        self.version_update_counts[version] = self.version_update_counts.get(version, 0) + 1

    DistributedUpdate = distributed_update

    def run(self, max_updates: Optional[int] = None, timeout: Optional[float] = None):
        """Work loop: compute on the current download, then wait for the next, until DONE."""
        t0 = time.perf_counter()
        n = 0
        handled = self.msg
        while not self.done:
            if self.msg is not None and self.msg is handled:
                self.distributed_update()
                n += 1
                if max_updates is not None and n >= max_updates:
                    break
            handled = None
            m = self.poll(0.05)
            if m is not None:
                handled = m
            elif timeout is not None and time.perf_counter() - t0 > timeout:
                break
        return n


class FedAvgClient(AbstractWorker):
    """Federated-averaging worker: each round, train ``local_steps`` SGD steps (or ``local_epochs`` passes)
    on its own shard starting from the global weights, then upload the resulting weights + #examples."""

    def __init__(self, transport: Transport, model, x: torch.Tensor, y: torch.Tensor, config: Optional[dict] = None,
                 server_rank: int = 0, batch_size: int = 32, local_steps: int = 0, local_epochs: int = 1,
                 data_scale: float = 1.0, seed: int = 0):
        super().__init__(transport, model, config)
        self.server_rank = server_rank
        self.x, self.y = x, y
        self.batch_size, self.local_steps, self.local_epochs = batch_size, local_steps, local_epochs
        self.data_scale = data_scale
        self.gen = torch.Generator(device="cpu")
        self.gen.manual_seed(seed)
        self.rounds_done = 0

    def _local_train(self):
        n = self.x.shape[0]
        steps = self.local_steps or max(1, self.local_epochs * (n // self.batch_size))
        perm = torch.randperm(n, generator=self.gen)
        seen = 0
        for s in range(steps):
            j = (s * self.batch_size) % max(1, n - self.batch_size + 1)
            idx = perm[j: j + self.batch_size].to(self.x.device)
            xb = self.x.index_select(0, idx)
            if xb.dtype == torch.uint8:
                xb = xb.float() * self.data_scale
            g = self.model.fit_flat(xb, self.y.index_select(0, idx))
            self.model.update_flat(g, 1.0)
            seen += idx.numel()
        return seen

    def run(self, timeout: Optional[float] = None):
        t0 = time.perf_counter()
        handled = self.msg
        while not self.done:
            if self.msg is not None and self.msg is handled:
                vid = self.msg.version_id
                seen = self.time("Local training", self._local_train)
                self._upload(self.model.get_flat(), vid, num_examples=int(self.x.shape[0]))
                self.rounds_done += 1
            handled = self.poll(0.05)
            if handled is None and timeout is not None and time.perf_counter() - t0 > timeout:
                break
        return self.rounds_done


# reference names
DistriWorker = FederatedClient
