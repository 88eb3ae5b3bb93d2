"""Message transports for the parameter-server roles (DistriServer / DistriWorker).

The reference moves every message through socket.io websockets in a star around the server, with
JSON framing and host-side ArrayBuffers (/root/reference/src/server/federated_server.ts:60-85,
/root/reference/src/client/abstract_client.ts:148-173).  Here:

* :class:`DistTransport` — ``torch.distributed`` point-to-point between ranks of ONE node: RCCL over
  xGMI when the process group is ``nccl`` (tensors go GPU->GPU, never through host memory), gloo
  on CPU.  A message = one fixed-size int64 header + up to 4 flat payloads (the model / gradient
  payload is the engine's flat HBM buffer itself).  Receiving is first-come-first-serve over all
  peers: one header ``irecv`` is kept posted per peer and polled, so the server handles whichever
  worker finishes first (RCCL has no any-source receive).
* :class:`LocalHub` / :class:`LocalTransport` — in-process queues with identical semantics, for
  single-process use and the protocol tests (the reference's loopback test shape,
  /root/reference/src/test/federated_api_test.ts).

Both deliver per-pair FIFO order, like a socket.
"""
from __future__ import annotations

import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Optional, Sequence

import torch
import torch.distributed as dist

from ..protocol import HEADER_LEN, Kind, decode_header, encode_header, json_payload, payload_json

META_FLAG = 0x100  # kind bit: last payload is a JSON dict


@dataclass
class Message:
    kind: int
    src: int = -1
    version_id: int = 0
    batch: int = -1
    epoch: int = -1
    metrics: list = field(default_factory=list)
    num_examples: int = 0
    tensors: list = field(default_factory=list)
    meta: dict = field(default_factory=dict)


class Transport:
    rank: int
    peers: list

    def send(self, dst: int, msg: Message) -> None:
        raise NotImplementedError

    def recv(self, timeout: Optional[float] = None) -> Optional[Message]:
        raise NotImplementedError

    def broadcast(self, msg: Message, dsts: Optional[Sequence[int]] = None) -> None:
        for d in (self.peers if dsts is None else dsts):
            self.send(d, msg)

    def close(self) -> None:
        pass


# ------------------------------------------------------------------------------------------ in-process
class LocalHub:
    """Shared mailboxes for endpoints 0..n-1 living in one process (threads or cooperative loops)."""

    def __init__(self, n: int):
        self.n = n
        self.boxes = [queue.Queue() for _ in range(n)]
        self.closed = [False] * n

    def endpoint(self, rank: int, peers: Optional[Sequence[int]] = None) -> "LocalTransport":
        return LocalTransport(self, rank, peers)


class LocalTransport(Transport):
    def __init__(self, hub: LocalHub, rank: int, peers: Optional[Sequence[int]] = None):
        self.hub, self.rank = hub, rank
        self.peers = list(peers) if peers is not None else [r for r in range(hub.n) if r != rank]

    def send(self, dst: int, msg: Message) -> None:
        if self.hub.closed[dst]:
            return
        # messages own their tensors (a socket would have serialised them)
        m = Message(msg.kind, self.rank, msg.version_id, msg.batch, msg.epoch, list(msg.metrics), msg.num_examples,
                    [t.detach().clone() for t in msg.tensors], dict(msg.meta))
        self.hub.boxes[dst].put(m)

    def recv(self, timeout: Optional[float] = None) -> Optional[Message]:
        try:
            if timeout is not None and timeout <= 0:
                return self.hub.boxes[self.rank].get_nowait()
            return self.hub.boxes[self.rank].get(timeout=timeout)
        except queue.Empty:
            return None

    def close(self) -> None:
        self.hub.closed[self.rank] = True


# ------------------------------------------------------------------------------------------ torch.distributed
class DistTransport(Transport):
    """Point-to-point messages over a torch.distributed process group (RCCL on GPUs, gloo on CPU)."""

    def __init__(self, peers: Sequence[int], device=None, group=None, poll_interval: float = 50e-6):
        if not dist.is_initialized():
            raise RuntimeError("DistTransport needs an initialised process group")
        self.group = group
        self.rank = dist.get_rank()
        self.peers = list(peers)
        self.backend = dist.get_backend(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
        self.device = torch.device(device)
        self.poll_interval = poll_interval
        self._hdr = {}
        self._work = {}
        self._lock = threading.Lock()
        for p in self.peers:
            self._post(p)

    def _post(self, peer: int):
        h = torch.empty(HEADER_LEN, dtype=torch.int64, device=self.device)
        self._hdr[peer] = h
        self._work[peer] = dist.irecv(h, src=peer, group=self.group)

    def send(self, dst: int, msg: Message) -> None:
        payloads = [t.detach().reshape(-1) for t in msg.tensors]
        kind = msg.kind
        if msg.meta:
            payloads.append(json_payload(msg.meta))
            kind |= META_FLAG
        payloads = [p if p.device == self.device else p.to(self.device) for p in payloads]
        payloads = [p.contiguous() for p in payloads]
        h = encode_header(kind, self.rank, msg.version_id, msg.batch, msg.epoch, msg.metrics, msg.num_examples,
                          payloads).to(self.device)
        with self._lock:
            dist.send(h, dst, group=self.group)
            for p in payloads:
                if p.numel():
                    dist.send(p, dst, group=self.group)

    def _complete(self, peer: int) -> Message:
        hd = decode_header(self._hdr[peer])
        tensors = []
        for dt, n in hd["payloads"]:
            t = torch.empty(n, dtype=dt, device=self.device)
            if n:
                dist.recv(t, src=peer, group=self.group)
            tensors.append(t)
        self._post(peer)
        kind = hd["kind"]
        meta = {}
        if kind & META_FLAG:
            meta = payload_json(tensors.pop())
            kind &= ~META_FLAG
        return Message(kind, hd["src"], hd["version_id"], hd["batch"], hd["epoch"], hd["metrics"],
                       hd["num_examples"], tensors, meta)

    def recv(self, timeout: Optional[float] = None) -> Optional[Message]:
        t0 = time.perf_counter()
        while True:
            for peer in self.peers:
                w = self._work.get(peer)
                if w is not None and w.is_completed():
                    w.wait()
                    return self._complete(peer)
            if timeout is not None and time.perf_counter() - t0 >= timeout:
                return None
            time.sleep(self.poll_interval)

    def close(self) -> None:
        # posted header receives are abandoned with the process group
        self._work.clear()
