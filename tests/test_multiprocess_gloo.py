"""Multi-process tests on the CPU gloo backend: synchronous all-reduce data parallelism, and the
parameter-server roles over the torch.distributed transport (RCCL on GPUs uses the same code)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from distriflow_amd.parallel.comm import init_distributed

    return init_distributed(backend="gloo", device="cpu", timeout_s=120)


def _dp_worker(rank, world, port, out_dir):
    _init(rank, world, port)
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer

    torch.manual_seed(0)
    net = build_model("lenet5", "cpu", seed=rank)  # different init per rank: broadcast must fix it
    x, y = synthetic_mnist(64, seed=5)
    tr = DataParallelTrainer(net, lr=0.1, graph="none", bucket_mb=0.05)  # several buckets -> overlap path
    assert len(tr.buckets) > 1
    xb = (x[rank * 32:(rank + 1) * 32].float() / 255)
    tr.train_step(xb, y[rank * 32:(rank + 1) * 32])
    torch.save(net.store.master.clone(), os.path.join(out_dir, f"w{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_data_parallel_allreduce_matches_full_batch():
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model

    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dp_worker, args=(2, _port(), d), nprocs=2, join=True)
        w0 = torch.load(os.path.join(d, "w0.pt"), weights_only=True)
        w1 = torch.load(os.path.join(d, "w1.pt"), weights_only=True)
    assert torch.equal(w0, w1)
    ref = build_model("lenet5", "cpu", seed=0)
    x, y = synthetic_mnist(64, seed=5)
    ref.compute_gradients(x.float() / 255, y)
    ref.store.set_hyper(0.1)
    ref.store.sgd_step()
    torch.testing.assert_close(w0, ref.store.master, rtol=1e-4, atol=1e-6)


def _ps_worker(rank, world, port, mode, out_dir):
    _init(rank, world, port)
    from distriflow_amd.data.dataset import DistriDataset
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.distri_model import ClientModel, InMemoryServerModel
    from distriflow_amd.parallel.server import AsynchronousSGDServer, FederatedServer
    from distriflow_amd.parallel.transport import make_star_transports
    from distriflow_amd.parallel.worker import AsynchronousSGDClient, FederatedClient

    x, y = synthetic_mnist(256, seed=7)
    result = {}
    tp = make_star_transports(0)
    if rank == 0:
        model = InMemoryServerModel("mlp_mnist", {"learningRate": 0.05}, device="cpu")
        if mode == "sync":
            srv = FederatedServer(tp, model, {"modelDir": False, "serverHyperparams": {"minUpdatesPerVersion": 2},
                                              "clientHyperparams": {"examplesPerUpdate": 16}})
            srv.setup()
            srv.serve(until=lambda: srv.num_clients == 0 and srv.num_updates == 0 and srv.version_id > 0, timeout=120)
            result = {"versions": srv.version_id}
        else:
            ds = DistriDataset(x, y, {"batchSize": 32, "epochs": 1})
            srv = AsynchronousSGDServer(tp, model, ds, {"modelDir": False, "serverHyperparams": {"maximumStaleness": 2}})
            srv.setup()
            srv.serve(until=lambda: srv.all_done() and srv.num_clients == 0, timeout=120)
            result = {"updates": srv.num_updates, "done": ds.done, "hist": srv.gate.histogram()}
    else:
        cm = ClientModel("mlp_mnist", device="cpu")
        if mode == "sync":
            c = FederatedClient(tp, cm, {"clientId": f"c{rank}"})
            c.setup()
            for i in range(8):
                c.distributed_update(x[i * 16:(i + 1) * 16].float() / 255, y[i * 16:(i + 1) * 16])
            c.poll(0.5)
            result = {"versions_seen": c.num_versions(), "uploads": c.num_updates()}
        else:
            c = AsynchronousSGDClient(tp, cm, {"clientId": f"a{rank}"}, data=x, labels=y, data_scale=1 / 255)
            c.setup()
            c.run(timeout=100)
            result = {"uploads": c.num_updates()}
        c.dispose()
    tp.close()
    torch.save(result, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["sync", "async"])
def test_parameter_server_over_gloo(mode):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ps_worker, args=(3, _port(), mode, d), nprocs=3, join=True)
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=False) for r in range(3)]
    if mode == "sync":
        assert res[0]["versions"] >= 2  # 16 uploads, barrier 2, stale ones dropped
        assert all(r["uploads"] == 8 for r in res[1:])
    else:
        assert res[0]["done"]
        assert res[0]["updates"] == sum(r["uploads"] for r in res[1:]) >= 8
        assert len(res[0]["hist"]) <= 3


def _fedavg_worker(rank, world, port, out_dir):
    _init(rank, world, port)
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.fedavg import FedAvgTrainer

    net = build_model("mlp_mnist", "cpu", seed=0)
    tr = FedAvgTrainer(net, lr=0.1, local_steps=3, graph="none")
    # after the initial broadcast every rank diverges: perturb rank-specifically, then average
    before = net.store.master.clone()
    net.store.master.add_(float(rank + 1))
    tr.average()
    torch.save({"before": before, "after": net.store.master.clone()}, os.path.join(out_dir, f"f{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_fedavg_average_is_the_mean_of_ranks():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_fedavg_worker, args=(2, _port(), d), nprocs=2, join=True)
        r = [torch.load(os.path.join(d, f"f{i}.pt"), weights_only=True) for i in range(2)]
    assert torch.equal(r[0]["before"], r[1]["before"])  # broadcast init
    torch.testing.assert_close(r[0]["after"], r[0]["before"] + 1.5)  # mean of +1 and +2
    assert torch.equal(r[0]["after"], r[1]["after"])


def _fedsgd_worker(rank, world, port, out_dir, k, steps):
    _init(rank, world, port)
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer, fedsgd_rows

    net = build_model("mlp_mnist", "cpu", seed=0)
    x, y = synthetic_mnist(512, seed=5)
    tr = DataParallelTrainer(net, lr=0.1, graph="none", min_updates_per_version=k)
    tr.bind_dataset(x, y, 16, scale=1.0 / 255)
    g = torch.Generator().manual_seed(3)
    micro = torch.randperm(512, generator=g)[: 16 * k * steps].view(k * steps, 16)
    tr.bind_index_stream(fedsgd_rows(micro, k, rank, world))
    for _ in range(steps):
        tr.step()
    torch.save({"w": net.store.master.clone(), "B": tr.B, "images": tr.images_per_step},
               os.path.join(out_dir, f"f{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("k", [8, 5])
def test_fedsgd_count_barrier_equals_union_of_k_microbatches(k):
    """Device FedSGD count barrier (reference FederatedServer: the mean of minUpdatesPerVersion
    microbatch gradients per version, federated_server.ts:73-90): W = 2 ranks sharing K microbatches of
    16 rows per version (K = 5: 3 + 2, uneven) equal one rank stepping on the union of the K microbatches,
    for every version."""
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model

    world, steps = 2, 3
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_fedsgd_worker, args=(world, _port(), d, k, steps), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"f{i}.pt"), weights_only=True) for i in range(world)]
    assert torch.equal(r[0]["w"], r[1]["w"])
    assert r[0]["B"] == 16 * (k // 2 + k % 2) and r[1]["B"] == 16 * (k // 2)
    assert r[0]["images"] == 16 * k
    ref = build_model("mlp_mnist", "cpu", seed=0)
    x, y = synthetic_mnist(512, seed=5)
    g = torch.Generator().manual_seed(3)
    micro = torch.randperm(512, generator=g)[: 16 * k * steps].view(k * steps, 16)
    ref.store.set_hyper(0.1)
    for v in range(steps):
        rows = micro[v * k:(v + 1) * k].reshape(-1)
        ref.compute_gradients(x[rows].float() / 255, y[rows])
        ref.store.sgd_step()
    torch.testing.assert_close(r[0]["w"], ref.store.master, rtol=1e-5, atol=1e-7)
