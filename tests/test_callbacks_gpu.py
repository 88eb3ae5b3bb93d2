"""Version / upload callbacks of the device engines (VERDICT r2 Missing 3, next-round #7).

Reference: AbstractServer.onNewVersion / onUpload fire on every update with the clients' metrics
(/root/reference/src/server/abstract_server.ts:67-79,105-115, asynchronousSGD_server.ts:66-70).  Here
they fire once per graph replay from device counters that the step's own last launch accumulates (no
extra launch inside the step), read back asynchronously."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


def _data():
    from distriflow_amd.data.synthetic import synthetic_mnist

    return synthetic_mnist(4096, seed=3, device=dev)


@pytest.mark.parametrize("model", ["lenet5", "mlp_mnist"])
def test_sync_callbacks_follow_the_version_counter(model):
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer, epoch_permutations

    data, labels = _data()
    net = build_model(model, device=dev, seed=0)
    tr = DataParallelTrainer(net, lr=0.05, graph="full")
    tr.bind_dataset(data, labels, 256, scale=1.0 / 255.0)
    tr.bind_index_stream(epoch_permutations(4096, 256, 16, dev, seed=1))
    versions, uploads = [], []
    tr.on_new_version(lambda o, n: versions.append((o, n)))
    tr.onUpload(uploads.append)  # reference spelling
    tr.prepare_run(4)
    tr.run(10)  # two 4-step replays + two single steps
    tr.flush_callbacks()
    assert versions == [(0, 4), (4, 8), (8, 9), (9, 10)]
    assert [u["version"] for u in uploads] == [4, 8, 9, 10]
    assert [u["updates"] for u in uploads] == [4, 4, 1, 1]  # counted on the device
    assert all(u["images"] == u["steps"] * 256 and math.isfinite(u["loss"]) and 0 <= u["accuracy"] <= 1
               for u in uploads)
    # the last replay's loss is the last step's loss
    assert abs(uploads[-1]["loss"] - float(tr.stats[0]) / 256) < 1e-4


def test_async_callbacks_report_ps_counters():
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.async_ps import AsyncPSTrainer
    from distriflow_amd.parallel.data_parallel import epoch_permutations

    data, labels = _data()
    net = build_model("lenet5", device=dev, seed=0)
    tr = AsyncPSTrainer(net, lr=0.05, max_staleness=2, graph="full")
    tr.bind_dataset(data, labels, 256, scale=1.0 / 255.0)
    tr.bind_schedule(epoch_permutations(4096, 256, 16, dev, seed=1))
    ups = []
    tr.on_upload(ups.append)
    tr.prepare_run(4)
    tr.run(12)
    tr.flush_callbacks()
    st = tr.ps_stats()
    assert [u["version"] for u in ups] == [4, 8, 12]
    assert sum(u["accepted"] for u in ups) == st["accepted"] == st["version"] == 12  # one worker: all admitted
    assert sum(u["rejected"] for u in ups) == 0
    assert all(math.isfinite(u["loss"]) for u in ups)


@pytest.mark.parametrize("graph", ["full", "none"])
def test_preprocess_callback_runs_inside_the_device_step(graph):
    """A dataset preprocess callback (reference dataset.ts:87-96) runs on every batch of the device
    engine, captured into the step's hipGraph: 3 fused LeNet-5 steps with an invert-images callback give
    bit-identical weights to 3 steps on explicitly inverted batches."""
    from distriflow_amd import ops
    from distriflow_amd.data.dataset import DistriDataset
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer

    data, labels = _data()
    ds = DistriDataset(data, labels, {"batchSize": 256, "epochs": 1}, shuffle=False)
    calls = []

    def invert(b):
        calls.append(1)
        b.x.mul_(-1.0).add_(1.0)
        return b

    ds.add_preprocess_callback(invert)
    a = build_model("lenet5", device=dev, seed=0)
    b = build_model("lenet5", device=dev, seed=0)
    tr = DataParallelTrainer(a, lr=0.05, graph=graph)
    tr.bind_distri_dataset(ds)
    ref = DataParallelTrainer(b, lr=0.05, graph="none")
    xs = torch.empty(256, 28, 28, 1, dtype=torch.bfloat16, device=dev)
    ys = torch.empty(256, dtype=torch.int32, device=dev)
    for k in range(3):
        tr.step()
        idx = torch.arange(256 * k, 256 * (k + 1), device=dev)
        ops.gather_batch(data, labels, idx, xs, ys, 1.0 / 255.0)
        ref.train_step((1.0 - xs.float()).to(torch.bfloat16), ys)
    torch.cuda.synchronize()
    assert calls  # traced (graph) or called per step (eager)
    assert torch.equal(a.store.master, b.store.master)
