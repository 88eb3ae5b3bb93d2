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
    """Point-to-point messages over torch.distributed (RCCL over xGMI on GPUs, gloo on CPU).

    Every (server, worker) pair gets TWO 2-rank process groups, one per direction.  RCCL runs all
    point-to-point traffic of a communicator on one stream, so a permanently posted header receive
    would otherwise block the same pair's sends in the other direction; with a group per direction
    each stream only ever carries one direction's messages in order.  Sends are non-blocking
    (``isend`` on a snapshot of the payload, completed in the background) so two peers that send to
    each other at the same time cannot deadlock.  Create with :func:`make_star_transports` (collective).
    """

    CLOSE = 0x7F  # channel-level kind: the peer closed its sending side

    def __init__(self, rank: int, channels: dict, device=None, poll_interval: float = 50e-6):
        self.rank = rank
        self.channels = channels  # peer -> (send_group, recv_group)
        self.peers = sorted(channels)
        self.backend = dist.get_backend()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
        self.device = torch.device(device)
        self.poll_interval = poll_interval
        self._inflight = []
        self._closed = False
        # RCCL: header receives stay posted and are polled through their completion events (never
        # blocking a stream the compute path uses).  gloo: point-to-point work only completes inside
        # wait(), so one receiver thread per peer blocks on its channel and queues whole messages.
        self._threaded = self.backend != "nccl"
        if self._threaded:
            self._q: "queue.Queue" = queue.Queue()
            self._threads = []
            for p in self.peers:
                t = threading.Thread(target=self._rx_loop, args=(p,), daemon=True)
                t.start()
                self._threads.append(t)
        else:
            self._hdr = {}
            self._work = {}
            for p in self.peers:
                self._post(p)

    # ---- receive side
    def _post(self, peer: int):
        h = torch.empty(HEADER_LEN, dtype=torch.int64, device=self.device)
        self._hdr[peer] = h
        self._work[peer] = dist.irecv(h, src=peer, group=self.channels[peer][1])

    def _read_body(self, peer: int, hdr: torch.Tensor) -> Message:
        hd = decode_header(hdr)
        g = self.channels[peer][1]
        tensors = []
        for dt, n in hd["payloads"]:
            t = torch.empty(n, dtype=dt, device=self.device)
            if n:
                dist.recv(t, src=peer, group=g)
            tensors.append(t)
        kind = hd["kind"]
        meta = {}
        if kind & META_FLAG:
            meta = payload_json(tensors.pop())
            kind &= ~META_FLAG
        return Message(kind, hd["src"], hd["version_id"], hd["batch"], hd["epoch"], hd["metrics"],
                       hd["num_examples"], tensors, meta)

    def _rx_loop(self, peer: int):
        g = self.channels[peer][1]
        while True:
            h = torch.empty(HEADER_LEN, dtype=torch.int64, device=self.device)
            try:
                dist.recv(h, src=peer, group=g)
                m = self._read_body(peer, h)
            except Exception as e:  # process group torn down
                self._q.put(e)
                return
            if m.kind == self.CLOSE:
                return
            self._q.put(m)

    def recv(self, timeout: Optional[float] = None) -> Optional[Message]:
        if self._threaded:
            self._reap()
            try:
                if timeout is not None and timeout <= 0:
                    m = self._q.get_nowait()
                else:
                    m = self._q.get(timeout=timeout)
            except queue.Empty:
                return None
            if isinstance(m, Exception):
                raise m
            return m
        t0 = time.perf_counter()
        while True:
            self._reap()
            for peer in self.peers:
                w = self._work.get(peer)
                if w is not None and w.is_completed():
                    w.wait()
                    m = self._read_body(peer, self._hdr[peer])
                    self._post(peer)
                    if m.kind == self.CLOSE:
                        self._work.pop(peer, None)
                        continue
                    return m
            if timeout is not None and time.perf_counter() - t0 >= timeout:
                return None
            time.sleep(self.poll_interval)

    # ---- send side
    def _reap(self):
        if self._inflight:
            self._inflight = [(w, keep) for (w, keep) in self._inflight if not w.is_completed()]

    def send(self, dst: int, msg: Message) -> None:
        payloads = [t.detach().reshape(-1) for t in msg.tensors]
        kind = msg.kind
        if msg.meta:
            payloads.append(json_payload(msg.meta))
            kind |= META_FLAG
        # snapshot semantics (a socket copies too): the caller may update the weights right after
        payloads = [p.to(self.device, copy=True).contiguous() for p in payloads]
        h = encode_header(kind, self.rank, msg.version_id, msg.batch, msg.epoch, msg.metrics, msg.num_examples,
                          payloads).to(self.device)
        g = self.channels[dst][0]
        self._reap()
        if self._threaded:
            # gloo isend completes only inside wait(): keep ordering with a blocking send on the
            # channel (the receiver thread of the peer always drains it, so this cannot deadlock)
            dist.send(h, dst, group=g)
            for p in payloads:
                if p.numel():
                    dist.send(p, dst, group=g)
            return
        self._inflight.append((dist.isend(h, dst, group=g), h))
        for p in payloads:
            if p.numel():
                self._inflight.append((dist.isend(p, dst, group=g), p))

    def flush(self, timeout: float = 60.0):
        """Wait until every send of this endpoint has been delivered."""
        t0 = time.perf_counter()
        while self._inflight and time.perf_counter() - t0 < timeout:
            self._reap()
            time.sleep(self.poll_interval)

    def close(self) -> None:
        """Collective with the peers' close(): tells every peer's receiver this channel is finished."""
        if self._closed:
            return
        self._closed = True
        for p in self.peers:
            try:
                self.send(p, Message(self.CLOSE))
            except Exception:
                pass
        self.flush()
        if self._threaded:
            for t in self._threads:
                t.join(timeout=30)


def make_star_transports(server_rank: int = 0, device=None) -> DistTransport:
    """Collective (every rank calls it): a star of per-direction channels around ``server_rank``.
    Returns this rank's endpoint (the server's peers are all workers, a worker's peer is the server)."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    up, down = {}, {}
    for c in range(world):
        if c == server_rank:
            continue
        pair = sorted([server_rank, c])
        up[c] = dist.new_group(pair)    # worker -> server
        down[c] = dist.new_group(pair)  # server -> worker
    if rank == server_rank:
        channels = {c: (down[c], up[c]) for c in up}
    else:
        channels = {server_rank: (up[rank], down[rank])}
    return DistTransport(rank, channels, device)
