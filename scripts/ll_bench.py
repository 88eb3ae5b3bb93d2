#!/usr/bin/env python3
"""In-kernel LL exchange microbenchmark (csrc/ll_exchange.h through the ll_selftest kernel: one slot of
1024 fp32 values per workgroup, each value pushed to every peer as an 8-byte {value, epoch} granule,
then polled and summed in rank order).  W ranks share cuda:0 over gloo (the one-GPU pool), so the
pushes land in local HBM: the numbers are the protocol's own cost (push issue, poll, sum), not xGMI.
Prints per payload size: median us per exchange, us per MB of values, granule bytes per peer."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def worker(rank, world, port, q):
    from mp_util import finish, init_rank

    dev = init_rank(rank, world, port)
    from distriflow_amd.parallel.p2p import P2PAllReduce

    p = P2PAllReduce(max_bytes=1 << 20, ll_slots=256)
    assert p.ok, p.reason
    comm = p.comm
    out = []
    for ns in (16, 64, 128, 256):
        inp = torch.randn(ns * 1024, device=dev)
        o = torch.empty_like(inp)
        for _ in range(5):
            comm.ll_selftest(inp, o)
        torch.cuda.synchronize()
        ts = []
        for _ in range(20):
            dist.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            comm.ll_selftest(inp, o)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        med = ts[len(ts) // 2]
        mb = ns * 1024 * 4 / 1e6
        out.append((ns, mb, med, med / mb, ns * 1024 * 8 / 1e3))
    if rank == 0:
        q.put(out)
    finish()


def main():
    from mp_util import free_port

    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.spawn(worker, args=(world, free_port(), q), nprocs=world, join=True)
    rows = q.get()
    print(f"LL exchange, {world} ranks sharing one MI355X (local HBM under the peer stores):")
    print(f"{'slots':>6} {'MB values':>10} {'us/exchange':>12} {'us/MB':>8} {'KB granules/peer':>17}")
    for ns, mb, med, per, kb in rows:
        print(f"{ns:6d} {mb:10.3f} {med:12.2f} {per:8.2f} {kb:17.0f}")


if __name__ == "__main__":
    main()
