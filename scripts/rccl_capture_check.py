#!/usr/bin/env python3
"""Does this ROCm/RCCL stack support capturing collectives in a hipGraph?  (1-rank communicator.)
Mirrors DataParallelTrainer's full-graph path: async all_reduce issued mid-step, waited at the end."""
import os
import time

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29611")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
x = torch.ones(61706, device="cuda")
y = torch.zeros_like(x)
dist.all_reduce(x)  # warm the communicator
torch.cuda.synchronize()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        y.add_(1.0)
        w = dist.all_reduce(x, async_op=True)
        y.mul_(2.0)
        w.wait()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
ok = True
try:
    with torch.cuda.graph(g):
        y.add_(1.0)
        w = dist.all_reduce(x, async_op=True)
        y.mul_(2.0)
        w.wait()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
except Exception as e:  # noqa: BLE001
    ok = False
    print("capture failed:", repr(e))
print("capture ok:", ok, "x[0]", float(x[0]))
# eager small all-reduce latency (1 rank: pure RCCL launch overhead)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(200):
    dist.all_reduce(x)
torch.cuda.synchronize()
print(f"eager all_reduce(247 KB) 1 rank: {(time.perf_counter() - t0) / 200 * 1e6:.1f} us")
dist.destroy_process_group()
