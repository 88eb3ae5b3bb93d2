"""One-shot xGMI all-reduce for small gradient buckets (kernel: csrc/allreduce_p2p.hip).

The reference's synchronous aggregation is a host-side stack + mean on the parameter server
(/root/reference/src/server/federated_server.ts:92-117 with /root/reference/src/common/utils.ts:53-75).
Here every rank keeps the full gradient in HBM and the mean becomes an all-reduce.  For the
reference's payloads (31.8 KB MLP, 247 KB LeNet-5, 2.4 MB Keras CNN) the cost is latency, not
bandwidth.  A ring all-reduce makes 2(W-1) dependent hops over single links.  The one-shot kernel
reads all W-1 peer copies at once over the fully connected xGMI mesh (7 links per MI355X), so one
flag round is the only synchronisation.

Setup is collective: every rank allocates an IPC-exportable buffer, the handles go round the
process group (``all_gather_object``), each rank maps its peers, and a self-test checks the
sums against a host reference.  All ranks then agree, through a MIN all-reduce of a status flag, whether the
path is usable.  If any rank fails (IPC refused, ranks on different nodes, a peer flag timed out)
every rank falls back to RCCL.  The kernel never spins forever: a peer missing for ``timeout_s``
sets a sticky error word, and :meth:`check` raises on it.
"""
from __future__ import annotations

import os
import socket
from typing import Optional

import torch
import torch.distributed as dist

from .. import native


def _agree(ok: bool, group, device) -> bool:
    if dist.get_backend(group) == "gloo":
        device = torch.device("cpu")
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


class P2PAllReduce:
    """In-place SUM all-reduce of fp32 GPU tensors of up to ``max_bytes`` over IPC-mapped peer buffers."""

    def __init__(self, group=None, max_bytes: int = 8 << 20, timeout_s: float = 30.0, self_test: bool = True,
                 ll_slots: int = 256):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.max_floats = max_bytes // 4
        self.comm = None
        self.reason = ""
        ok, why = True, ""
        if self.world > 8:
            ok, why = False, "more than 8 ranks"
        hosts = [None] * self.world
        dist.all_gather_object(hosts, socket.gethostname(), group=group)
        if len(set(hosts)) != 1:
            ok, why = False, "ranks span several nodes"
        comm, handle = None, b""
        if ok:
            try:
                # + ll_slots slots of the in-kernel LL exchange (csrc/ll_exchange.h) for kernels that
                # fold the all-reduce into their own epilogue (the fused LeNet-5 reduce)
                comm = native.require().P2PComm(self.rank, self.world, self.max_floats, timeout_s, ll_slots)
                handle = comm.handle()
            except Exception as e:  # e.g. IPC export refused by the driver
                ok, why = False, f"alloc/export: {e!r}"
        if not _agree(ok, group, self.device):
            self.reason = why or "a peer could not set up"
            return
        handles = [None] * self.world
        dist.all_gather_object(handles, handle, group=group)
        try:
            comm.open(handles)
        except Exception as e:
            ok, why = False, f"open: {e!r}"
        if not _agree(ok, group, self.device):
            self.reason = why or "a peer could not map the buffers"
            return
        self.comm = comm
        if self_test:
            # a broken peer path shows up as a flag timeout: fail the self-test within seconds, not minutes
            comm.set_timeout(min(timeout_s, 5.0))
            passed = self._self_test() and self._ll_self_test()
            comm.set_timeout(timeout_s)
            if not passed:
                self.comm = None
                self.reason = self.reason or "self-test mismatch"
        self._probe = None
        if self.comm is not None:
            from .watchdog import register_owner_probe

            self._probe = register_owner_probe(
                "p2p_allreduce", self, lambda o: o.comm.host_error() if o.comm is not None else 0)

    def close(self):
        """Release the IPC mappings and stop the watchdog reading this communicator's error word."""
        from .watchdog import unregister_probe

        if getattr(self, "_probe", None):
            unregister_probe(self._probe)
            self._probe = None
        self.comm = None

    @property
    def ok(self) -> bool:
        return self.comm is not None

    def capacity(self) -> int:
        return self.comm.max_floats if self.comm is not None else 0

    def all_reduce(self, t: torch.Tensor, scale: float = 1.0):
        """In place on the current stream (graph-capturable)."""
        self.comm.allreduce(t, scale)

    def check(self):
        """Raise if any launch saw a peer-flag timeout (the sticky device error word)."""
        if self.comm is not None and self.comm.error() != 0:
            raise RuntimeError("p2p all-reduce: a peer flag timed out (peer dead or stalled)")

    def _ll_self_test(self) -> bool:
        """The in-kernel LL exchange (csrc/ll_exchange.h) that the fused LeNet-5 reduce launch folds into
        its epilogue, on its first slots, both parities.  A failure (mismatch or peer timeout: the error word
        is shared with the all-reduce) disables the whole communicator, so the trainer falls back to RCCL."""
        ok = True
        try:
            ns = min(4, int(self.comm.ll_slots))
            if ns <= 0:
                return True
            n = ns * 1024  # kLLSlot granules per slot
            g = torch.Generator(device="cpu")
            for it in range(3):
                g.manual_seed(4321 + it)
                base = torch.randn(self.world, n, generator=g)
                out = torch.empty(n, device=self.device)
                self.comm.ll_selftest(base[self.rank].to(self.device), out)
                torch.cuda.synchronize(self.device)
                if self.comm.error() != 0:
                    self.reason, ok = "peer timeout in the LL exchange self-test", False
                    break
                # rank-order fp32 sums: every rank must hold the same bits
                ref = base[0].clone()
                for r in range(1, self.world):
                    ref += base[r]
                if not torch.equal(out.cpu(), ref):
                    self.reason, ok = "LL exchange self-test mismatch", False
                    break
        except Exception as e:
            self.reason, ok = f"LL self-test: {e!r}", False
        return _agree(ok, self.group, self.device)

    def _self_test(self) -> bool:
        ok = True
        try:
            g = torch.Generator(device="cpu")
            for n in sorted({min(k, self.max_floats) for k in (1, 5, 2048, 2049, 70001, 1 << 20)}):
                g.manual_seed(1234 + n)
                base = torch.randn(self.world, n, generator=g)
                mine = base[self.rank].to(self.device)
                for _ in range(3):  # both staging halves, epoch advance
                    x = mine.clone()
                    self.all_reduce(x)
                    torch.cuda.synchronize(self.device)
                    ref = base.sum(0)
                    if self.comm.error() != 0:
                        self.reason = "peer flag timeout in self-test"
                        ok = False
                        break
                    if not torch.allclose(x.cpu(), ref, rtol=1e-5, atol=1e-5):
                        self.reason = f"self-test mismatch at n={n}"
                        ok = False
                        break
                if not ok:
                    break
        except Exception as e:
            self.reason, ok = f"self-test: {e!r}", False
        return _agree(ok, self.group, self.device)


def make_p2p(group=None, max_bytes: int = 8 << 20, timeout_s: float = 30.0) -> Optional[P2PAllReduce]:
    """``DISTRIFLOW_ALLREDUCE=rccl`` disables the one-shot path; returns None when it is unusable."""
    if os.environ.get("DISTRIFLOW_ALLREDUCE", "auto").lower() == "rccl":
        return None
    if not (dist.is_initialized() and dist.get_world_size(group) > 1 and torch.cuda.is_available()):
        return None
    p = P2PAllReduce(group, max_bytes=max_bytes, timeout_s=timeout_s)
    return p if p.ok else None
