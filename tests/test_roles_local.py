"""Server <-> worker protocol over the in-process transport (reference federated_api_test.ts shape),
plus asynchronous SGD (FCFS dataset, bounded staleness) and FedAvg with the real engine on CPU."""
import threading
import time

import pytest
import torch

from distriflow_amd.data.dataset import DistriDataset
from distriflow_amd.data.synthetic import non_iid_shards, synthetic_mnist
from distriflow_amd.models.distri_model import InMemoryServerModel, ClientModel
from distriflow_amd.models.mock import MockModel
from distriflow_amd.parallel.server import AsynchronousSGDServer, FedAvgServer, FederatedServer
from distriflow_amd.parallel.transport import LocalHub
from distriflow_amd.parallel.worker import AsynchronousSGDClient, FedAvgClient, FederatedClient

INIT = [torch.ones(2, 2), torch.tensor([[1.0, 2, 3, 4]])]


def wait_for(cond, timeout=10.0):
    t0 = time.time()
    while not cond():
        if time.time() - t0 > timeout:
            raise TimeoutError("condition not reached")
        time.sleep(0.005)


@pytest.fixture
def fed(tmp_path):
    hub = LocalHub(2)
    server_model = MockModel(INIT)
    server_model.version = "initial"
    client_vars = [torch.zeros_like(t) for t in INIT]
    client_model = MockModel(client_vars)
    server = FederatedServer(hub.endpoint(0), server_model, {
        "modelDir": str(tmp_path), "serverHyperparams": {"minUpdatesPerVersion": 2},
        "clientHyperparams": {"examplesPerUpdate": 1}})
    server.setup()
    th = threading.Thread(target=server.serve, kwargs={"timeout": 30}, daemon=True)
    th.start()
    client = FederatedClient(hub.endpoint(1), client_model, {"clientId": "c1"})
    client.setup()
    yield server, client, client_model
    client.dispose()
    server.stop()
    th.join(5)


def test_transmits_model_version_on_startup(fed):
    server, client, cm = fed
    assert client.model_version() == "initial"
    assert torch.equal(cm.vars[0], INIT[0])  # weights downloaded


def test_transmits_updates(fed):
    server, client, cm = fed
    assert len(server.updates) == 0
    cm.vars[0].copy_(torch.full((2, 2), 2.0))
    client.distributed_update(torch.zeros(1, 1), torch.zeros(1))
    wait_for(lambda: len(server.updates) == 1)
    assert server.num_clients == 1 and server.clients[1] == "c1"


def test_triggers_download_after_enough_uploads(fed):
    server, client, cm = fed
    seen, server_versions = [], []
    client.on_new_version(lambda old, new: seen.append((old, new)))
    server.on_new_version(lambda old, new: server_versions.append(new))
    cm.vars[0].copy_(torch.full((2, 2), 2.0))
    client.distributed_update(torch.zeros(1, 1), torch.zeros(1))
    client.distributed_update(torch.zeros(3, 1), torch.zeros(3))
    wait_for(lambda: (client.poll(0.01) or True) and len(seen) > 0)
    old, new = seen[0]
    # the client may already have uploaded the last two examples on the bumped version, in which case
    # the server bumps twice; the first new version the client sees is the server's first bump
    assert old == "initial" and new != "initial" and new == server_versions[0]
    # 4 uploads, barrier 2: uploads computed on a stale version after a bump are dropped
    assert client.num_updates() == 4


def test_async_sgd_fcfs_bounded_staleness():
    x, y = synthetic_mnist(512, seed=1)
    hub = LocalHub(3)
    ds = DistriDataset(x, y, {"batchSize": 32, "epochs": 2})
    smodel = InMemoryServerModel("mlp_mnist", {"learningRate": 0.05}, device="cpu")
    server = AsynchronousSGDServer(hub.endpoint(0), smodel, ds,
                                   {"modelDir": False, "serverHyperparams": {"maximumStaleness": 1}})
    server.setup()
    th = threading.Thread(target=server.serve, kwargs={"until": server.all_done, "timeout": 60}, daemon=True)
    th.start()
    workers, threads = [], []
    for r in (1, 2):
        w = AsynchronousSGDClient(hub.endpoint(r, [0]), ClientModel("mlp_mnist", device="cpu"),
                                  {"clientId": f"w{r}"}, data=x, labels=y, data_scale=1 / 255)
        workers.append(w)
    for w in workers:
        t = threading.Thread(target=lambda w=w: (w.setup(), w.run(timeout=60)), daemon=True)
        t.start()
        threads.append(t)
    for t in threads:
        t.join(60)
    th.join(10)
    assert ds.done
    assert server.num_updates >= ds.batches * 2  # every batch of both epochs completed at least once
    hist = server.gate.histogram()
    assert len(hist) <= 2  # staleness never above the bound
    assert server.gate.accepted + server.gate.rejected == server.num_updates
    assert sum(w.num_updates() for w in workers) == server.num_updates


def test_fedavg_rounds_non_iid():
    x, y = synthetic_mnist(800, seed=2)
    shards = non_iid_shards(y, 2, 2)
    hub = LocalHub(3)
    smodel = InMemoryServerModel("mlp_mnist", device="cpu")
    server = FedAvgServer(hub.endpoint(0), smodel, {"modelDir": False}, rounds=3)
    server.setup()
    clients = [FedAvgClient(hub.endpoint(r, [0]), ClientModel("mlp_mnist", {"learningRate": 0.05}, device="cpu"),
                            x[shards[r - 1]], y[shards[r - 1]], {"clientId": f"f{r}", "connectionTimeout": 30},
                            batch_size=32, local_steps=5, data_scale=1 / 255, seed=r) for r in (1, 2)]
    ths = [threading.Thread(target=lambda c=c: (c.setup(), c.run(timeout=60)), daemon=True) for c in clients]
    for t in ths:
        t.start()
    wait_for(lambda: server.step(0.01) is not None and server.num_clients == 2, 20)
    v0 = smodel.get_flat().clone()
    server.start_round()
    server.serve(until=server.finished, timeout=60)
    server.shutdown()
    for t in ths:
        t.join(10)
    assert server.round == 3 and server.version_id == 3
    assert all(c.rounds_done == 3 for c in clients)
    assert not torch.equal(v0, smodel.get_flat())


def test_async_sgd_rejected_batches_are_redispatched():
    """maximumStaleness 0 with 3 racing workers rejects many gradients; every (epoch, batch) must still
    end with exactly one ADMITTED gradient (at-least-once dispatch, /root/reference/src/server/
    dataset.ts:47-67), and a shuffled dataset's workers train on the permuted example ids."""
    x, y = synthetic_mnist(384, seed=3)
    hub = LocalHub(4)
    ds = DistriDataset(x, y, {"batchSize": 32, "epochs": 2}, shuffle=True, seed=5)
    smodel = InMemoryServerModel("mlp_mnist", {"learningRate": 0.05}, device="cpu")
    server = AsynchronousSGDServer(hub.endpoint(0), smodel, ds,
                                   {"modelDir": False, "serverHyperparams": {"maximumStaleness": 0}})
    seen_idx = []
    server.setup()
    th = threading.Thread(target=server.serve, kwargs={"until": server.all_done, "timeout": 90}, daemon=True)
    th.start()
    workers = [AsynchronousSGDClient(hub.endpoint(r, [0]), ClientModel("mlp_mnist", device="cpu"),
                                     {"clientId": f"w{r}"}, data=x, labels=y, data_scale=1 / 255) for r in (1, 2, 3)]
    orig = workers[0]._batch_tensors

    def spy(m):
        seen_idx.append(list((m.meta.get("data") or {}).get("indices") or []))
        return orig(m)
    workers[0]._batch_tensors = spy
    threads = [threading.Thread(target=lambda w=w: (w.setup(), w.run(timeout=90)), daemon=True) for w in workers]
    for t in threads:
        t.start()
    for t in threads:
        t.join(90)
    th.join(10)
    assert ds.done
    admitted = server.admitted_batches
    assert sorted(admitted) == sorted((e, b) for e in range(2) for b in range(ds.batches))
    assert server.gate.rejected > 0  # the race really produced stale gradients
    assert server.gate.accepted == len(admitted)
    assert seen_idx and all(len(i) == 32 for i in seen_idx)
    assert any(i != list(range(i[0], i[0] + 32)) for i in seen_idx)  # permuted, not row ranges
