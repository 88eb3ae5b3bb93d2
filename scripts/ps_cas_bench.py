#!/usr/bin/env python3
"""Throughput of the parameter server's element adds (csrc/ps_device.h ps_add) against process count.

P processes (sharing this box's GPU, gloo control plane) each apply K gradients of n elements to the
sharded master with max_staleness unbounded (every gradient admitted), all at once.  At P >= 2 every add
is a system-scope compare-and-swap on uncached, IPC-mapped memory (the N > 1 path of the async PS); P = 1
is the exclusive plain read-modify-write path.  Prints one JSON line per P: aggregate element adds per
microsecond, per-process apply time, CAS retries.  On one GPU the "remote" shards are local HBM, so this
prices CAS contention and the uncached path, not xGMI link latency.

usage: python scripts/ps_cas_bench.py [--procs 1,2,4,8] [--n 61708] [--steps 50]
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _worker(rank, world, port, n, steps, q):
    import torch
    import torch.distributed as dist

    from mp_util import init_rank
    from test_async_ps_gpu import _open_ps

    dev = init_rank(rank, world, port)
    ps = _open_ps(rank, world, n)
    ps.init_master(torch.zeros(n, device=dev))
    g = torch.full((n,), -1e-3, device=dev)
    for _ in range(3):
        ps.apply(g, 1.0, -1)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        ps.apply(g, 1.0, -1)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    dist.barrier()
    t1 = time.perf_counter()
    st = ps.stats()
    q.put((rank, el, t1 - t0, st[4], st[5]))
    dist.barrier()
    dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp

    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", default="1,2,4,8")
    ap.add_argument("--n", type=int, default=61708)
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    ctx = mp.get_context("spawn")
    for P in [int(p) for p in args.procs.split(",")]:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        q = ctx.Queue()
        mp.start_processes(_worker, args=(P, port, args.n, args.steps, q), nprocs=P, join=True, start_method="spawn")
        res = sorted(q.get() for _ in range(P))
        wall = max(r[2] for r in res)
        adds = P * args.steps * args.n
        print(json.dumps({"procs": P, "path": "exclusive RMW" if P == 1 else "system-scope CAS",
                          "n": args.n, "steps": args.steps, "wall_s": round(wall, 5),
                          "adds_per_us": round(adds / wall / 1e6, 1),
                          "apply_us_per_proc": round(max(r[1] for r in res) / args.steps * 1e6, 2),
                          "cas_retries": sum(r[3] for r in res), "err": sum(r[4] for r in res)}), flush=True)


if __name__ == "__main__":
    main()
