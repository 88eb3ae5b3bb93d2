#!/usr/bin/env python3
"""Does the fused-exchange self-test perturb later steps?  2 ranks on cuda:0 (gloo): 8 steps with the
self-test on / off, single-step replays and 4-step graphs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def worker(rank, world, port):
    from mp_util import init_rank, finish
    dev = init_rank(rank, world, port)
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer

    data, labels = synthetic_mnist(4096, seed=3, device=dev)
    g = torch.Generator().manual_seed(5)
    rows = torch.stack([torch.randperm(4096, generator=g)[:128] for _ in range(12)])[:, rank * 64:(rank + 1) * 64]
    res = {}
    for name, st_on, multi in (("on_single", 1, False), ("off_single", 0, False), ("on_single2", 1, False),
                               ("off_single2", 0, False), ("on_single3", 1, False)):
        os.environ["DISTRIFLOW_DIAG"] = f"fused_selftest={st_on}"
        net = build_model("lenet5", device=dev, seed=0)
        tr = DataParallelTrainer(net, lr=0.05, graph="full", allreduce="p2p")
        tr.bind_dataset(data, labels, 64, scale=1.0 / 255.0)
        tr.bind_index_stream(rows.contiguous().to(dev))
        if multi:
            tr.prepare_run(4)
            tr.run(8)
        else:
            for _ in range(8):
                tr.step()
        torch.cuda.synchronize()
        res[name] = net.store.master.clone()
        tk = net.lenet_dense_part[-100:]
        res[name + "_tickets"] = int((tk != 0).sum())
    base = res["off_single"]
    print(f"rank {rank}: " + ", ".join(f"{k}: maxdiff {float((v - base).abs().max()):.3e}" for k, v in res.items()
                                       if not k.endswith("_tickets")) +
          " tickets nonzero " + str({k: v for k, v in res.items() if k.endswith("_tickets")}), flush=True)
    finish()


if __name__ == "__main__":
    from mp_util import free_port
    mp.spawn(worker, args=(2, free_port()), nprocs=2, join=True)
