"""Rank setup shared by the multi-process GPU tests.

On a node with at least ``world`` GPUs every rank gets its own device (``cuda:rank``) and the process
group runs on RCCL (``backend="nccl"``), so the IPC mappings, the one-shot / in-kernel LL exchanges and
the parameter server really travel over xGMI between distinct devices.  On a smaller box (the one-GPU
test pool) the ranks share ``cuda:0`` and the control plane is gloo (RCCL refuses two ranks on one
device): the same protocol code runs, with local HBM under the peer loads and stores.
"""
import os
import socket

import torch


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def real_devices(world: int) -> bool:
    """True when every rank can have a GPU of its own (device_count does not initialise HIP)."""
    return torch.cuda.device_count() >= world


def init_rank(rank: int, world: int, port: int) -> torch.device:
    """Join the test's process group; returns this rank's device."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if real_devices(world):
        dev = torch.device("cuda", rank)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return dev


def finish():
    import torch.distributed as dist

    dist.barrier()
    dist.destroy_process_group()
