"""One-shot xGMI all-reduce (csrc/allreduce_p2p.hip, parallel/p2p.py) on a real MI355X.

On a node with a GPU per rank every rank gets its own device and the process group is RCCL, so the
peer loads and flags cross xGMI (tests/mp_util.py).  On the one-GPU test box the ranks are processes
sharing cuda:0: the IPC export/import, the flag protocol, the double-buffered staging and graph
capture are all exercised exactly as on an 8-GPU node (only the transport under the peer loads
differs: local HBM instead of xGMI), with a gloo control plane (RCCL refuses two ranks on one device).
"""
import os
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from mp_util import free_port, init_rank

pytestmark = pytest.mark.gpu


def _port():
    return free_port()


def _init(rank, world, port):
    """cuda:rank + RCCL when the box has a GPU per rank, else ranks share cuda:0 over gloo (mp_util)."""
    import torch.distributed as dist

    global DEV
    DEV = init_rank(rank, world, port)
    return dist


DEV = torch.device("cuda", 0)


def _primitive_worker(rank, world, port, out_dir):
    dist = _init(rank, world, port)
    from distriflow_amd.parallel.p2p import P2PAllReduce

    p = P2PAllReduce(max_bytes=1 << 20, timeout_s=10.0)
    res = {"ok": p.ok, "reason": p.reason}
    if p.ok:
        dev = DEV
        g = torch.Generator().manual_seed(7)
        base = torch.randn(world, 100_003, generator=g)
        # eager, with scale
        x = base[rank].to(dev)
        p.all_reduce(x, scale=0.5)
        torch.cuda.synchronize()
        res["eager_err"] = float((x.cpu() - 0.5 * base.sum(0)).abs().max())
        res["eager_bits"] = x.cpu()
        # graph capture + replays: epochs must keep advancing on the device
        y = torch.zeros(100_003, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            y.copy_(base[rank].to(dev))
            p.all_reduce(y)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        src = base[rank].to(dev)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            y.copy_(src)
            p.all_reduce(y)
        errs = []
        for i in range(5):
            src.mul_(-1.0)
            gr.replay()
            torch.cuda.synchronize()
            sign = -1.0 if i % 2 == 0 else 1.0
            errs.append(float((y.cpu() - sign * base.sum(0)).abs().max()))
        res["graph_err"] = max(errs)
        res["dev_error"] = p.comm.error()
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _timeout_worker(rank, world, port, out_dir):
    dist = _init(rank, world, port)
    from distriflow_amd.parallel.p2p import P2PAllReduce

    p = P2PAllReduce(max_bytes=64 << 10, timeout_s=0.5, self_test=False)
    flag = None
    if p.ok and rank == 0:
        x = torch.ones(4096, device=DEV)
        p.all_reduce(x)  # rank 1 never joins
        # the host-mapped mirror shows the timeout while the kernel may still be running, with no HIP
        # call (this is what the watchdog thread polls)
        import time

        t0 = time.time()
        while p.comm.host_error() == 0 and time.time() - t0 < 10.0:
            time.sleep(0.01)
        host_flag = p.comm.host_error()
        torch.cuda.synchronize()
        flag = p.comm.error()
    else:
        host_flag = None
    torch.save({"ok": p.ok, "flag": flag, "host_flag": host_flag}, os.path.join(out_dir, f"t{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _trainer_worker(rank, world, port, out_dir):
    _init(rank, world, port)
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer, epoch_permutations

    dev = DEV
    net = build_model("lenet5", device=dev, seed=rank)  # different init: the broadcast must fix it
    data, labels = synthetic_mnist(4096, seed=3, device=dev)
    tr = DataParallelTrainer(net, lr=0.05, graph="full", allreduce="p2p")
    tr.bind_dataset(data, labels, 256, scale=1.0 / 255.0)
    tr.bind_index_stream(epoch_permutations(4096, 256, 40, dev, seed=rank))
    losses = []
    for _ in range(40):
        st = tr.step()
        losses.append(float(st[0].item()) / 256)
    torch.cuda.synchronize()
    tr.check_comm()
    torch.save({"w": net.store.master.cpu(), "losses": losses, "path": tr.allreduce_path,
                "graph": tr.graph_mode}, os.path.join(out_dir, f"w{rank}.pt"))
    import torch.distributed as dist

    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 8])
def test_p2p_allreduce_procs_sharing_one_gpu(world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_primitive_worker, args=(world, _port(), d), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"r{i}.pt"), weights_only=True) for i in range(world)]
    assert all(x["ok"] for x in r), [x["reason"] for x in r]
    for x in r:
        assert x["eager_err"] < 1e-4 and x["graph_err"] < 1e-4 and x["dev_error"] == 0
    for x in r[1:]:
        assert torch.equal(r[0]["eager_bits"], x["eager_bits"])  # rank-order sums: bit-identical replicas


@pytest.mark.timeout(120)
def test_p2p_peer_timeout_sets_error_instead_of_hanging():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_timeout_worker, args=(2, _port(), d), nprocs=2, join=True)
        t0 = torch.load(os.path.join(d, "t0.pt"), weights_only=True)
    assert t0["ok"]
    assert t0["flag"] == 1 and t0["host_flag"] == 1


@pytest.mark.timeout(240)
def test_p2p_data_parallel_graph_training():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_trainer_worker, args=(2, _port(), d), nprocs=2, join=True)
        w = [torch.load(os.path.join(d, f"w{i}.pt"), weights_only=True) for i in range(2)]
    assert w[0]["path"] == "p2p" and w[0]["graph"] == "full"
    assert torch.equal(w[0]["w"], w[1]["w"])  # replicas stay bit-identical
    l0 = w[0]["losses"]
    assert sum(l0[-5:]) < sum(l0[:5])


def _fedavg_gpu_worker(rank, world, port, out_dir):
    _init(rank, world, port)
    from distriflow_amd.data.synthetic import non_iid_shards, synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.fedavg import FedAvgTrainer

    dev = DEV
    data, labels = synthetic_mnist(8192, seed=3, device=dev)
    shard = non_iid_shards(labels, world, 5, seed=0)[rank].to(dev)
    B, rounds, local = 256, 10, 20
    g = torch.Generator().manual_seed(rank)
    reps = rounds * local * B // shard.numel() + 1
    stream = torch.cat([shard[torch.randperm(shard.numel(), generator=g).to(dev)] for _ in range(reps)])
    stream = stream[: rounds * local * B].view(rounds * local, B)
    net = build_model("lenet5", device=dev, seed=rank)
    tr = FedAvgTrainer(net, lr=0.1, local_steps=local, graph="full", allreduce="p2p")
    tr.bind_dataset(data, labels, B, scale=1.0 / 255.0)
    tr.bind_index_stream(stream)
    loss0, acc0 = net.evaluate(data[:2048].float() / 255.0, labels[:2048])
    for _ in range(rounds):
        tr.run_round()
    torch.cuda.synchronize()
    tr.check_comm()
    loss, acc = net.evaluate(data[:2048].float() / 255.0, labels[:2048])
    acc = acc if loss < loss0 else -1.0
    torch.save({"w": net.store.master.cpu(), "acc": float(acc), "graph": tr.graph_mode},
               os.path.join(out_dir, f"a{rank}.pt"))
    import torch.distributed as dist

    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_fedavg_device_engine_two_procs():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_fedavg_gpu_worker, args=(2, _port(), d), nprocs=2, join=True)
        r = [torch.load(os.path.join(d, f"a{i}.pt"), weights_only=True) for i in range(2)]
    assert r[0]["graph"] == "full"
    assert torch.equal(r[0]["w"], r[1]["w"])  # every rank ends a round with the same averaged model
    assert r[0]["acc"] > 0.3  # loss fell and the averaged model beats chance well on all 10 classes


def _fedavg_average_worker(rank, world, port, out_dir):
    _init(rank, world, port)
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.fedavg import FedAvgTrainer

    dev = DEV
    net = build_model("lenet5", device=dev, seed=0)
    tr = FedAvgTrainer(net, lr=0.1, local_steps=1, graph="none", allreduce="p2p")
    g = torch.Generator().manual_seed(100 + rank)
    mine = torch.randn(net.store.total, generator=g)
    net.store.master.copy_(mine.to(dev))
    tr.average()
    torch.cuda.synchronize()
    tr.check_comm()
    torch.save({"mine": mine, "avg": net.store.master.cpu(), "path": tr.allreduce_path},
               os.path.join(out_dir, f"f{rank}.pt"))
    import torch.distributed as dist

    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_fedavg_average_is_the_mean_of_rank_masters():
    """the device FedAvg engine's average() equals the CPU mean of the ranks' masters
    (one-shot xGMI all-reduce, rank-order sums, then the 1/world scale), on every rank."""
    world = 3
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_fedavg_average_worker, args=(world, _port(), d), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"f{i}.pt"), weights_only=True) for i in range(world)]
    ref = torch.stack([x["mine"] for x in r]).double().mean(0).float()
    for x in r:
        assert x["path"] == "p2p"
        torch.testing.assert_close(x["avg"], ref, rtol=1e-6, atol=1e-6)
    assert torch.equal(r[0]["avg"], r[1]["avg"]) and torch.equal(r[0]["avg"], r[2]["avg"])
