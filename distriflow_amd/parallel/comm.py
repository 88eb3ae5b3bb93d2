"""Process-group plumbing: one process per GPU, RCCL (``backend="nccl"`` on ROCm) for the data plane,
gloo for CPU-only runs / control metadata, TCPStore rendezvous on 127.0.0.1.

Replaces the reference's socket.io transport and its connection handshake (SURVEY §2.5 M1-M2,
/root/reference/src/client/abstract_client.ts:166-173: ``connectTo`` + first Download within 10 s)
with ``init_process_group`` + a timeout.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1 and dist.is_initialized()

    @property
    def is_main(self) -> bool:
        return self.rank == 0


_ENV: Optional[DistEnv] = None


def init_distributed(backend: Optional[str] = None, timeout_s: float = 600.0, device: Optional[str] = None,
                     watchdog: bool = False) -> DistEnv:
    """Initialise from torchrun-style env vars (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT).

    backend: "nccl" (RCCL over xGMI, GPUs), "gloo" (CPU), or None = nccl if GPUs are visible else gloo.
    watchdog: start the dead-peer watchdog (parallel/watchdog.py) once the group is up, so a lost
    rank ends the job within ``DISTRIFLOW_DEAD_AFTER_S`` (30 s) instead of the collective timeout.
    """
    global _ENV
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = (device or ("cuda" if torch.cuda.is_available() else "cpu")).startswith("cuda")
    # DISTRIFLOW_BACKEND=gloo on a GPU box: rehearsal mode, several ranks may share a GPU (rank r on
    # GPU r % device_count) with gloo as the control plane; RCCL refuses two ranks on one device
    backend = backend or os.environ.get("DISTRIFLOW_BACKEND") or None
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    if use_gpu and backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    dev = torch.device(f"cuda:{local}") if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(dev)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    _ENV = DistEnv(rank, world, local, backend if world > 1 else "none", dev)
    if watchdog and world > 1:
        from .watchdog import start_watchdog

        start_watchdog(rank, world)
    return _ENV


def env() -> DistEnv:
    return _ENV or DistEnv()


def shutdown():
    global _ENV
    from .watchdog import active

    from .watchdog import clear_probes

    wd = active()
    if wd is not None:
        # normal completion: peers stop watching this rank, but this rank keeps watching them until the
        # final barrier returns (a peer that dies during shutdown still ends the job promptly)
        wd.mark_done()
    if dist.is_initialized():
        try:
            dist.barrier()
        except Exception:
            pass
    if wd is not None:
        wd.stop()
    clear_probes()
    if dist.is_initialized():
        dist.destroy_process_group()
    _ENV = None


def broadcast_params(flat: torch.Tensor, src: int = 0, group=None):
    """Initial weight sync (reference M1: every connecting client first downloads the weights)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat, src=src, group=group)


def allreduce_max_scalar(v: float, device) -> float:
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return v
    t = torch.tensor([v], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
