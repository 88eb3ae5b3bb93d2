"""DistriServer roles: the parameter server side of synchronous (FedSGD), asynchronous (bounded
staleness) and federated-averaging training.

Reference: ``AbstractServer`` (/root/reference/src/server/abstract_server.ts:24-116),
``FederatedServer`` (federated_server.ts:26-118), ``AsynchronousSGDServer``
(asynchronousSGD_server.ts:14-110); SURVEY §2.2 S6-S8, §3.1, §3.3.

Preserved behaviour: callbacks ``on_new_version(old, new)`` / ``on_upload(msg)``, counters
``num_clients`` / ``num_updates`` / ``updates``, the ``updating`` guard, version-gated uploads and the
count barrier ``minUpdatesPerVersion`` (FedSGD), FCFS microbatch dispatch with re-dispatch (async),
hyper-parameters pushed to clients in every download, verbose logging + ms timers, default
checkpointed server model under ``<cwd>/saved-models``.

MI355X design: messages ride :mod:`.transport` (RCCL point-to-point between GPU ranks, or in-process
queues); gradients arrive as flat fp32 HBM buffers and are aggregated by ONE ``sum_buffers`` kernel
with the 1/K mean folded in, then applied by the fused SGD kernel; the new weights leave as the
engine's flat master buffer (no host serialisation).  Fixes: upload callbacks get the
message (item 7); the async server sends the next batch + weights only to the worker that uploaded
(item 6: the reference broadcast the same batch to everyone; ``broadcast_downloads=True`` restores
it); bounded staleness ``maximumStaleness`` (README.md:27) is enforced with a native gate.
"""
from __future__ import annotations

import os
import time
from typing import Callable, Optional

import torch

from .. import native, ops
from ..config import client_hyperparams, server_hyperparams, verbose_from_env
from ..models.distri_model import CheckpointedServerModel, InMemoryServerModel, is_server_model
from ..protocol import DataMsg, GradientMsg, Kind, UploadMsg
from ..utils.logging import Logger
from .transport import Message, Transport


class AbstractServer:
    role = "Distributed Server"

    def __init__(self, transport: Transport, model, config: Optional[dict] = None):
        config = dict(config or {})
        allowed = {"clientHyperparams", "serverHyperparams", "updatesPerVersion", "modelDir", "modelCompileArgs",
                   "verbose", "broadcastDownloads", "saveEvery", "keepLast", "ack", "metricsFile"}
        for k in config:
            if k not in allowed:
                raise ValueError(f'Unrecognized server config key "{k}"')
        if not is_server_model(model):
            model_dir = config.get("modelDir")
            compile_cfg = config.get("modelCompileArgs") or {}
            if model_dir is False:
                model = InMemoryServerModel(model, compile_cfg)
            else:
                model_dir = model_dir or os.path.join(os.getcwd(), "saved-models")
                model = CheckpointedServerModel(model_dir, model, compile_cfg, keep_last=config.get("keepLast"),
                                                save_every=config.get("saveEvery", 1))
        self.transport = transport
        self.model = model
        self.config = config
        self.verbose = verbose_from_env(config.get("verbose"))
        self.client_hyperparams = client_hyperparams(config.get("clientHyperparams") or {})
        self.server_hyperparams = server_hyperparams(config.get("serverHyperparams") or {})
        self.logger = Logger(self.role, self.verbose, config.get("metricsFile"))
        self.num_clients = 0
        self.num_updates = 0
        self.updates: list = []
        self.updating = False
        self.clients: dict = {}  # rank -> client id
        self.version_callbacks: list[Callable] = [lambda v1, v2: self.log(f"updated model: {v1} -> {v2}")]
        self.upload_callbacks: list[Callable] = []
        self.version_id = 0
        self.ack = bool(config.get("ack", False))
        self._running = False

    # ------------------------------------------------------------------ reference API
    def on_new_version(self, cb: Callable[[Optional[str], str], None]):
        self.version_callbacks.append(cb)

    def on_upload(self, cb: Callable[[UploadMsg], None]):
        self.upload_callbacks.append(cb)

    onNewVersion = on_new_version
    onUpload = on_upload

    def log(self, *args):
        self.logger.log(*args)

    def time(self, msg: str, fn: Callable):
        return self.logger.time(msg, fn)

    def perform_version_callbacks(self, old: Optional[str] = None):
        self.time("performing callbacks", lambda: [c(old, self.model.version) for c in self.version_callbacks])

    def perform_upload_callbacks(self, msg: UploadMsg):
        self.time("upload callbacks", lambda: [c(msg) for c in self.upload_callbacks])

    # ------------------------------------------------------------------ messages
    def download_message(self, data: Optional[DataMsg] = None) -> Message:
        meta = {"version": self.model.version, "hyperparams": self.client_hyperparams}
        if data is not None:
            meta["data"] = {"batch": data.batch, "epoch": data.epoch, "start": data.start, "size": data.size}
            if data.indices is not None:
                meta["data"]["indices"] = [int(i) for i in data.indices]
        tensors = [self.model.get_flat()]
        if data is not None and data.x is not None:
            tensors += [data.x, data.y]
        return Message(Kind.DOWNLOAD, version_id=self.version_id,
                       batch=data.batch if data else -1, epoch=data.epoch if data else -1, tensors=tensors, meta=meta)

    def _upload_msg(self, m: Message) -> UploadMsg:
        grads = m.tensors[0] if m.tensors else None
        return UploadMsg(client_id=self.clients.get(m.src, str(m.src)),
                         gradients=GradientMsg(str(m.version_id), grads) if grads is not None else None,
                         batch=m.batch if m.batch >= 0 else None, epoch=m.epoch if m.epoch >= 0 else None,
                         metrics=list(m.metrics) or None, num_examples=m.num_examples)

    def setup(self):
        self.time("setting up model", self.model.setup)
        self.perform_version_callbacks()

    def _new_version(self):
        old = self.model.version
        self.model.save()
        self.version_id += 1
        self.perform_version_callbacks(old)

    # ------------------------------------------------------------------ event loop
    def handle_connect(self, m: Message):
        self.num_clients += 1
        self.clients[m.src] = m.meta.get("client_id", str(m.src))
        self.log(f"connection: {self.num_clients} clients")

    def handle_disconnect(self, m: Message):
        if m.src in self.clients:
            self.clients.pop(m.src)
            self.num_clients -= 1
        self.log(f"disconnection: {self.num_clients} clients")

    def handle_upload(self, m: Message):
        raise NotImplementedError

    def handle(self, m: Message):
        if m.kind == Kind.HELLO:
            self.handle_connect(m)
        elif m.kind == Kind.UPLOAD:
            if self.ack:
                self.transport.send(m.src, Message(Kind.ACK, version_id=self.version_id))
            self.handle_upload(m)
        elif m.kind == Kind.BYE:
            self.handle_disconnect(m)

    def step(self, timeout: Optional[float] = 0.0) -> bool:
        m = self.transport.recv(timeout)
        if m is None:
            return False
        self.handle(m)
        return True

    def serve(self, until: Optional[Callable[[], bool]] = None, timeout: Optional[float] = None,
              idle_timeout: Optional[float] = None):
        """Event loop until ``until()`` is true, all clients left, or a timeout."""
        self._running = True
        t0 = time.perf_counter()
        last = t0
        while self._running:
            got = self.step(0.01)
            now = time.perf_counter()
            if got:
                last = now
            if until is not None and until():
                break
            if timeout is not None and now - t0 > timeout:
                break
            if idle_timeout is not None and now - last > idle_timeout:
                break
        self._running = False

    def stop(self):
        self._running = False

    def shutdown(self):
        for r in list(self.clients):
            self.transport.send(r, Message(Kind.DONE, version_id=self.version_id))


class FederatedServer(AbstractServer):
    """Synchronous FedSGD parameter server: accept only gradients computed on the current version,
    and after ``minUpdatesPerVersion`` of them apply their mean and publish a new version to all."""

    def setup(self):
        super().setup()

    def handle_connect(self, m: Message):
        super().handle_connect(m)
        self.transport.send(m.src, self.download_message())

    def should_update(self) -> bool:
        return self.num_updates >= int(self.server_hyperparams["minUpdatesPerVersion"])

    def handle_upload(self, m: Message):
        msg = self._upload_msg(m)
        if m.version_id != self.version_id or self.updating:
            self.log(f"dropped stale update from {msg.client_id} (version {m.version_id} != {self.version_id})")
            return
        self.log(f"new update from {msg.client_id}")
        self.updates.append(m.tensors[0])
        self.num_updates += 1
        self.perform_upload_callbacks(msg)
        if self.should_update():
            self.update_model()
            self.transport.broadcast(self.download_message(), list(self.clients))

    def update_model(self):
        self.updating = True
        agg = self.server_hyperparams["aggregation"]
        if agg != "mean":
            raise ValueError(f"unsupported aggregation {agg}")

        def _apply():
            k = len(self.updates)
            g = aggregate_sum(self.updates)
            self.model.update_flat(g, scale=1.0 / k)

        self.time("computing new weights", _apply)
        self.updates = []
        self.num_updates = 0
        self._new_version()
        self.updating = False


def aggregate_sum(bufs: list) -> torch.Tensor:
    """Sum K flat gradient buffers: one native kernel on GPU (pointer table), torch on CPU."""
    if len(bufs) == 1:
        return bufs[0]
    b0 = bufs[0]
    if b0.is_cuda:
        ptrs = torch.tensor([b.data_ptr() for b in bufs], dtype=torch.int64, device=b0.device)
        out = torch.empty_like(b0)
        native.require().sum_buffers(ptrs, len(bufs), out, 1.0)
        return out
    return torch.stack(bufs).sum(0)


class AsynchronousSGDServer(AbstractServer):
    """Asynchronous SGD parameter server with a server-owned FCFS dataset and bounded staleness.

    Every admitted gradient is applied on arrival (w -= lr * g) and starts a new version; a gradient
    computed on version v arriving at version V is admitted iff ``V - v <= maximumStaleness``
    (-1 = unbounded, the reference behaviour).  The uploading worker immediately gets the new weights
    plus its next microbatch (ids only when workers hold the data: ``ship_data=False``).
    """

    def __init__(self, transport: Transport, model, dataset, config: Optional[dict] = None, ship_data: bool = False):
        super().__init__(transport, model, config)
        self.dataset = dataset
        self.ship_data = ship_data
        self.broadcast_downloads = bool(self.config.get("broadcastDownloads", False))
        self.gate = native.require().StalenessGate(int(self.server_hyperparams["maximumStaleness"]))
        self.rejected = 0
        self.finished_clients = set()
        self.admitted_batches: list = []  # (epoch, batch) of every applied gradient, in order

    def _dispense(self) -> Optional[DataMsg]:
        from ..data.dataset import batch_to_data_msg

        if self.ship_data:
            b, done = self.dataset.next()
            if done:
                return None
            return DataMsg(b.batch, b.epoch, b.x, b.y, b.start, b.size)
        r = self.dataset.next_id()
        if r is None:
            return None
        b, epoch, start, size = r
        # a shuffled dataset's batch is its permuted example ids, not the row range [start, start+size)
        idx = self.dataset.example_indices(b).tolist() if self.dataset.shuffle else None
        return DataMsg(b, epoch, None, None, start, size, idx)

    def _send_work(self, dst: int):
        data = self._dispense()
        if data is None:
            self.transport.send(dst, Message(Kind.DONE, version_id=self.version_id))
            self.finished_clients.add(dst)
            return
        self.log(f"epoch: {data.epoch} batch: {data.batch}")
        msg = self.download_message(data)
        if self.broadcast_downloads:
            self.transport.broadcast(msg, list(self.clients))
        else:
            self.transport.send(dst, msg)

    def handle_connect(self, m: Message):
        super().handle_connect(m)
        self._send_work(m.src)

    def handle_upload(self, m: Message):
        msg = self._upload_msg(m)
        self.log(f"new update from {msg.client_id}")
        self.num_updates += 1
        self.perform_upload_callbacks(msg)
        if self.gate.admit(int(m.version_id), int(self.version_id)):
            # a microbatch counts as done only once its gradient is applied: a rejected (too stale)
            # gradient leaves the batch incomplete, so the dispenser hands it out again
            # (at-least-once, /root/reference/src/server/dataset.ts:47-67)
            if m.batch >= 0:
                self.dataset.complete_batch(m.batch, m.epoch if m.epoch >= 0 else None)
            self.admitted_batches.append((int(m.epoch), int(m.batch)))
            self.update_model(m.tensors[0])
        else:
            self.rejected += 1
            self.log(f"rejected update: staleness {self.version_id - m.version_id} > "
                     f"{self.server_hyperparams['maximumStaleness']}")
        self._send_work(m.src)

    def update_model(self, grad: torch.Tensor):
        self.updating = True
        self.time("computing new weights", lambda: self.model.update_flat(grad, 1.0))
        self._new_version()
        self.updating = False

    def all_done(self) -> bool:
        """Dataset exhausted and every connected worker has been told DONE (or has left)."""
        return self.num_updates > 0 and self.dataset.done and set(self.clients) <= self.finished_clients


class FedAvgServer(AbstractServer):
    """Federated averaging (McMahan et al.): each round the server sends the global weights, every
    participating client trains locally on its own (non-IID) data and returns weights + example count;
    the new global model is the example-weighted mean.  The reference only has the API shape for this
    (``FederatedClient.DistributedUpdate``, /root/reference/README.md:6 "stretch goal")."""

    def __init__(self, transport: Transport, model, config: Optional[dict] = None, rounds: int = 10,
                 clients_per_round: Optional[int] = None):
        super().__init__(transport, model, config)
        self.rounds = rounds
        self.round = 0
        self.clients_per_round = clients_per_round
        self._pending: dict = {}
        self._acc = None
        self._acc_n = 0

    def handle_connect(self, m: Message):
        super().handle_connect(m)

    def start_round(self):
        ranks = sorted(self.clients)
        if self.clients_per_round:
            ranks = ranks[: self.clients_per_round]
        self._pending = {r: True for r in ranks}
        self._acc = None
        self._acc_n = 0
        msg = self.download_message()
        msg.meta["round"] = self.round
        self.transport.broadcast(msg, ranks)

    def handle_upload(self, m: Message):
        if m.version_id != self.version_id or m.src not in self._pending:
            return
        msg = self._upload_msg(m)
        self.perform_upload_callbacks(msg)
        w = m.tensors[0].float()
        n = max(1, int(m.num_examples))
        self._acc = w * n if self._acc is None else self._acc.add_(w, alpha=n)
        self._acc_n += n
        self._pending.pop(m.src)
        self.num_updates += 1
        if not self._pending:
            self.model.set_flat(self._acc / self._acc_n)
            self._new_version()
            self.round += 1
            if self.round < self.rounds:
                self.start_round()

    def finished(self) -> bool:
        return self.round >= self.rounds


# reference names
DistriServer = FederatedServer
