"""The reference CNN's fused conv block (csrc/kcnn_fused.hip) against the per-layer kernels it replaces
(conv1 image-resident kernel, conv2 igemm64 with the pooled epilogue, unpool + conv2 weight / data
gradient + conv1 weight gradient).  The fused block computes conv1 on MFMA (the per-layer kernel: VALU FMA
chains), so the 9-tap fp32 sums differ in order: the pooled maps agree to bf16 rounding (a handful of
elements one bf16 step apart, an argmax code flipped where two window values tie within it), the loss and
every gradient to fp32 / bf16 summation order."""
import pytest
import torch

from distriflow_amd import ops

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


def _pair(monkeypatch, seed=3):
    from distriflow_amd.models.layers import KerasConvBlock
    from distriflow_amd.models.zoo import build_model

    f = build_model("keras_cnn", device=dev, seed=seed)
    assert isinstance(f.exec_layers[0], KerasConvBlock)
    monkeypatch.setenv("DISTRIFLOW_DIAG", "kcnn_fused=0")
    p = build_model("keras_cnn", device=dev, seed=seed)
    monkeypatch.delenv("DISTRIFLOW_DIAG")
    assert not isinstance(p.exec_layers[0], KerasConvBlock)
    p.store.set_flat(f.store.master.clone())
    return f, p


def _rel(a, b):
    return float((a.double() - b.double()).norm() / (b.double().norm() + 1e-30))


@pytest.mark.parametrize("B", [64, 200])
def test_kcnn_block_matches_per_layer_path(monkeypatch, B):
    from distriflow_amd.data.synthetic import synthetic_mnist

    f, p = _pair(monkeypatch)
    data, labels = synthetic_mnist(4096, seed=5, device=dev)
    idx = torch.randperm(4096, device=dev)[:B]
    x, y = ops.GatherRef(data, idx, 1 / 255.0, (28, 28, 1)), ops.LabelRef(labels, idx)
    # same dropout masks: the fused step's masks read counter + 1 and its reduce advances the counter at
    # the end; the per-layer step's gather advances it first
    f.step_dev.fill_(5)
    p.step_dev.fill_(5)
    sf = f.compute_gradients(x, y).clone()
    sp = p.compute_gradients(x, y).clone()
    torch.cuda.synchronize()
    assert int(f.step_dev.item()) == 6 and int(p.step_dev.item()) == 6
    of, op = f.exec_layers[0].out, p.exec_layers[1].out  # pooled (+ dropout) map
    assert _rel(of, op) < 2e-3, _rel(of, op)
    assert (of != op).float().mean().item() < 2e-3
    assert (f.exec_layers[0].code != p.exec_layers[1].code).float().mean().item() < 1e-3
    assert abs(float(sf[0]) - float(sp[0])) <= 1e-3 * abs(float(sp[0])) and abs(float(sf[1]) - float(sp[1])) <= 1
    for s in f.store.specs:
        gf, gp = f.store.gradient(s.name), p.store.gradient(s.name)
        assert _rel(gf, gp) < 5e-3, (s.name, _rel(gf, gp))


def test_kcnn_block_bf16_batch_input_and_training(monkeypatch):
    """A bf16 batch (no index) takes the same path; a few SGD steps reduce the loss."""
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer, epoch_permutations

    f, p = _pair(monkeypatch)
    data, labels = synthetic_mnist(2048, seed=1, device=dev)
    xb = (data[:96].float() / 255.0).to(torch.bfloat16)
    yb = labels[:96]
    f.step_dev.fill_(2)  # masks read 3, then the block's reduce advances the counter
    p.step_dev.fill_(2)  # advanced (torch add) to 3 before the per-layer step reads it
    sf = f.compute_gradients(xb, yb).clone()
    sp = p.compute_gradients(xb, yb).clone()
    torch.cuda.synchronize()
    assert abs(float(sf[0]) - float(sp[0])) <= 1e-3 * abs(float(sp[0]))
    tr = DataParallelTrainer(f, lr=0.05, graph="full")
    tr.bind_dataset(data, labels, 256, scale=1.0 / 255.0)
    tr.bind_index_stream(epoch_permutations(2048, 256, 30, dev, seed=0))
    losses = [float(tr.step()[0].item()) / 256 for _ in range(30)]
    assert tr.graph_mode == "full"
    assert sum(losses[-5:]) < 0.9 * sum(losses[:5]), losses
