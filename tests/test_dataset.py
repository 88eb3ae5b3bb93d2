"""DistriDataset FCFS semantics (reference dataset.ts) on the native dispenser."""
import torch

from distriflow_amd.data.dataset import DistriDataset, batch_to_data_msg
from distriflow_amd.data.mnist import load_mnist, one_hot, write_idx
from distriflow_amd.data.synthetic import non_iid_shards, synthetic_mnist


def _ds(n=100, bs=32, epochs=2, small=False, shuffle=False):
    x = torch.arange(n, dtype=torch.float32).view(n, 1)
    y = torch.arange(n)
    return DistriDataset(x, y, {"batchSize": bs, "epochs": epochs, "smallLastBatch": small}, shuffle=shuffle)


def test_sequential_dispatch_and_epochs():
    d = _ds(96, 32, 2)
    assert d.batches == 3
    seen = []
    while True:
        b, done = d.next()
        if done:
            break
        seen.append((b.epoch, b.batch))
        assert b.x.shape[0] == 32 and float(b.x[0]) == b.batch * 32
        d.complete_batch(b.batch)
    assert seen == [(0, 0), (0, 1), (0, 2), (1, 0), (1, 1), (1, 2)]


def test_redispatch_of_unacknowledged_batches():
    d = _ds(96, 32, 1)
    got = [d.next()[0].batch for _ in range(3)]
    assert got == [0, 1, 2]
    d.complete_batch(0)
    d.complete_batch(2)
    b, _ = d.next()           # cursor ran off the end: batch 1 (never completed) is re-dispatched
    assert b.batch == 1
    d.complete_batch(1)
    assert d.next() == (None, True)


def test_small_last_batch_and_drop():
    assert _ds(100, 32, 1, small=False).batches == 3
    d = _ds(100, 32, 1, small=True)
    assert d.batches == 4
    for _ in range(3):
        d.next()
    b, _ = d.next()
    assert b.batch == 3 and b.x.shape[0] == 4


def test_preprocess_and_state_roundtrip():
    d = _ds(64, 16, 3, shuffle=True)
    d.add_preprocess_callback(lambda b: (setattr(b, "x", b.x * 2) or b))
    b, _ = d.next()
    assert torch.equal(b.x, d.x.index_select(0, b.indices) * 2)
    d.complete_batch(b.batch)
    st = d.state()
    e = _ds(64, 16, 3, shuffle=True)
    e.load_state(st)
    assert e.epoch == d.epoch and e.remaining == d.remaining
    assert e.next()[0].batch == d.next()[0].batch
    msg = batch_to_data_msg(b)
    assert msg.x.shape == list(b.x.shape)


def test_idx_round_trip(tmp_path):
    x, y = synthetic_mnist(50)
    write_idx(str(tmp_path / "train-images-idx3-ubyte"), str(tmp_path / "train-labels-idx1-ubyte"), x, y)
    x2, y2 = load_mnist(str(tmp_path), "train")
    assert torch.equal(x2, x) and torch.equal(y2, y)
    assert one_hot(y2[:3]).shape == (3, 10)


def test_non_iid_shards_cover_each_example_once():
    _, y = synthetic_mnist(1000)
    shards = non_iid_shards(y, 8, 2)
    allidx = torch.cat(shards).sort().values
    assert torch.equal(allidx, torch.arange(1000))
    assert all(len(torch.unique(y[s])) <= 4 for s in shards)


def test_index_stream_covers_epochs_and_splits_ranks():
    """The sync engine's device schedule comes from the dispenser: every full batch of every epoch
    exactly once, batch k on rank k % world, per-epoch shuffles, and the dispenser ends done."""
    import torch

    from distriflow_amd.data.dataset import DistriDataset

    n, B, E = 100, 8, 3  # 12 full batches + a ragged one per epoch
    x, y = torch.arange(n).float().view(n, 1), torch.arange(n)
    streams = []
    for r in range(2):
        ds = DistriDataset(x, y, {"batchSize": B, "epochs": E}, shuffle=True, seed=7)
        streams.append(ds.index_stream(rank=r, world=2))
        assert ds.done
    a, b = streams
    assert a.shape == b.shape == (E * 12 // 2, B)
    for e in range(E):  # per epoch the two ranks' batches are disjoint rows of one permutation
        rows = torch.cat([a[e * 6:(e + 1) * 6].flatten(), b[e * 6:(e + 1) * 6].flatten()])
        assert rows.unique().numel() == 96
    assert not torch.equal(a[:6], a[6:12])  # reshuffled per epoch


def test_index_stream_refuses_preprocess_callbacks():
    import pytest
    import torch

    from distriflow_amd.data.dataset import DistriDataset

    ds = DistriDataset(torch.zeros(16, 1), torch.zeros(16), {"batchSize": 4, "epochs": 1})
    ds.add_preprocess_callback(lambda b: b)
    with pytest.raises(ValueError):
        ds.index_stream()


def test_trainer_binds_a_distri_dataset_cpu():
    import torch

    from distriflow_amd.data.dataset import DistriDataset
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer

    net = build_model("mlp_mnist", device="cpu", seed=0)
    data, labels = synthetic_mnist(512, seed=0, device="cpu")
    ds = DistriDataset(data, labels, {"batchSize": 64, "epochs": 2}, shuffle=True, seed=1)
    tr = DataParallelTrainer(net, lr=0.1, graph="none")
    steps = tr.bind_distri_dataset(ds)
    assert steps == 16 and tr.steps_per_epoch == 8
    losses = [float(tr.step()[0]) / 64 for _ in range(steps)]
    assert losses[-1] < losses[0]


def test_trainer_runs_dataset_preprocess_callbacks_cpu():
    """The device engines run the dataset's preprocess chain on every batch (reference
    /root/reference/src/server/dataset.ts:87-96): a step with a callback equals a plain step on the
    batch the callback produced."""
    import torch

    from distriflow_amd.data.dataset import DistriDataset
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer

    data, labels = synthetic_mnist(256, seed=3, device="cpu")
    seen = []

    def invert_and_shift(b):
        seen.append((int(b.batch[0]), b.epoch, tuple(b.x.shape)))
        b.x = 1.0 - b.x
        b.y = (b.y + 1) % 10
        return b

    ds = DistriDataset(data, labels, {"batchSize": 32, "epochs": 1}, shuffle=False)
    ds.add_preprocess_callback(invert_and_shift)
    a = build_model("mlp_mnist", device="cpu", seed=0)
    b = build_model("mlp_mnist", device="cpu", seed=0)
    tr = DataParallelTrainer(a, lr=0.1, graph="none")
    assert tr.bind_distri_dataset(ds) == 8
    ref = DataParallelTrainer(b, lr=0.1, graph="none")
    for k in range(3):
        st = tr.step()
        rows = torch.arange(32 * k, 32 * (k + 1))
        x = 1.0 - data[rows].float().reshape(32, 28, 28, 1) / 255.0
        y = ((labels[rows] + 1) % 10).to(torch.int32)
        st_ref = ref.train_step(x.to(b.dtype).float(), y)
        torch.testing.assert_close(st, st_ref)
        torch.testing.assert_close(a.store.master, b.store.master)
    assert [s[0] for s in seen] == [0, 1, 2] and all(s[1] == -1 and s[2] == (32, 28, 28, 1) for s in seen)


def test_preprocess_callback_must_keep_shapes_cpu():
    import pytest
    import torch

    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer, epoch_permutations

    data, labels = synthetic_mnist(128, seed=3, device="cpu")
    tr = DataParallelTrainer(build_model("mlp_mnist", device="cpu", seed=0), lr=0.1, graph="none")
    tr.bind_dataset(data, labels, 32, scale=1 / 255.0)
    tr.bind_index_stream(epoch_permutations(128, 32, 4, "cpu", seed=0))

    def crop(b):
        b.x = b.x[:, :20]
        return b

    tr.add_preprocess_callback(crop)
    with pytest.raises(ValueError):
        tr.step()
