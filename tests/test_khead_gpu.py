"""The reference CNN's dense head as one split-K launch (csrc/khead.hip) + the fused head weight-gradient
launch, against the per-layer path it replaces (igemm64 dense1 forward / split-K epilogue, mlphead dense2
+ softmax-CE, igemm64 dense1 data gradient, igemm weight gradient + slab reduction).  Same epilogue order
and roundings; fp32 sums differ in order only, so the data / weight gradients agree to bf16 rounding."""
import pytest
import torch

from distriflow_amd import ops

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


def _pair(monkeypatch, seed=3):
    from distriflow_amd.models.zoo import build_model

    f = build_model("keras_cnn", device=dev, seed=seed)
    assert f.khead
    monkeypatch.setenv("DISTRIFLOW_DIAG", "khead_fused=0")
    p = build_model("keras_cnn", device=dev, seed=seed)
    monkeypatch.delenv("DISTRIFLOW_DIAG")
    assert not p.khead
    p.store.set_flat(f.store.master.clone())
    return f, p


def _rel(a, b):
    return float((a.double() - b.double()).norm() / (b.double().norm() + 1e-30))


@pytest.mark.parametrize("B", [64, 200, 1024])
def test_khead_matches_per_layer_head(monkeypatch, B):
    from distriflow_amd.data.synthetic import synthetic_mnist

    f, p = _pair(monkeypatch)
    data, labels = synthetic_mnist(4096, seed=5, device=dev)
    idx = torch.randperm(4096, device=dev)[:B]
    x, y = ops.GatherRef(data, idx, 1 / 255.0, (28, 28, 1)), ops.LabelRef(labels, idx)
    f.step_dev.fill_(5)
    p.step_dev.fill_(5)
    sf = f.compute_gradients(x, y).clone()
    sp = p.compute_gradients(x, y).clone()
    torch.cuda.synchronize()
    assert torch.equal(f.exec_layers[0].out, p.exec_layers[0].out)  # same pooled (+ dropout) map
    assert abs(float(sf[0]) - float(sp[0])) <= 1e-3 * abs(float(sp[0])) + 1e-3, (sf, sp)
    assert abs(float(sf[1]) - float(sp[1])) <= max(2.0, 0.01 * B), (sf, sp)
    lf, lp = f.exec_layers[-1].out, p.exec_layers[-1].out
    assert _rel(lf, lp) < 1e-2, _rel(lf, lp)
    d1 = f.exec_layers[-2]
    assert _rel(d1.dx, p.exec_layers[-2].dx) < 2e-2, _rel(d1.dx, p.exec_layers[-2].dx)
    for s in f.store.specs:
        gf, gp = f.store.gradient(s.name), p.store.gradient(s.name)
        assert torch.isfinite(gf).all(), s.name
        assert _rel(gf, gp) < 2e-2, (s.name, _rel(gf, gp))


def test_khead_repeatable_across_launches(monkeypatch):
    """The flags compare against a per-launch tag: back-to-back steps on the same inputs give identical
    results (no stale flag, no lost ticket), batch not a multiple of the 32-row tile."""
    from distriflow_amd.data.synthetic import synthetic_mnist

    f, _ = _pair(monkeypatch)
    data, labels = synthetic_mnist(1024, seed=2, device=dev)
    xb = (data[:333].float() / 255.0).to(torch.bfloat16)
    yb = labels[:333]
    outs = []
    for _ in range(3):
        f.step_dev.fill_(7)
        s = f.compute_gradients(xb, yb).clone()
        torch.cuda.synchronize()
        outs.append((s, f.store.grad.clone(), f.exec_layers[-2].dx.clone()))
    for s, g, dx in outs[1:]:
        assert torch.equal(s, outs[0][0])
        assert torch.equal(g, outs[0][1])
        assert torch.equal(dx, outs[0][2])
    # no row tile's flag wait timed out (the bounded wait's sticky error word)
    from distriflow_amd import ops

    assert ops.khead_error(f.khead_ws, 333) == 0


def test_khead_training_in_graph(monkeypatch):
    """Captured into a hipGraph and replayed: the per-launch tag lives on the device, so replays stay
    correct; a few SGD steps reduce the loss."""
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer, epoch_permutations

    f, _ = _pair(monkeypatch)
    data, labels = synthetic_mnist(2048, seed=1, device=dev)
    tr = DataParallelTrainer(f, lr=0.05, graph="full")
    tr.bind_dataset(data, labels, 256, scale=1.0 / 255.0)
    tr.bind_index_stream(epoch_permutations(2048, 256, 30, dev, seed=0))
    losses = [float(tr.step()[0].item()) / 256 for _ in range(30)]
    assert tr.graph_mode == "full"
    assert sum(losses[-5:]) < 0.9 * sum(losses[:5]), losses
