"""Branching Keras graphs on MI355X: the merge kernels (csrc/merge.hip) against the fp32 torch reference
of the same op on bf16-rounded inputs, and a whole branching model's gradients against the CPU fp32
engine on the same weights."""
import pytest
import torch

from distriflow_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", list(ops.MERGE_KINDS))
@pytest.mark.parametrize("n", [2, 3])
def test_merge_kernels_match_fp32_reference(kind, n):
    if kind == "Subtract" and n != 2:
        pytest.skip("Subtract takes two inputs")
    g = torch.Generator().manual_seed(7)
    widths = [5, 8, 3][:n] if kind == "Concatenate" else [12] * n
    xs = [torch.randn(6, 4, 4, w, generator=g).to(torch.bfloat16) for w in widths]
    xs[0].view(-1)[:7] = xs[1].view(-1)[:7] if kind != "Concatenate" else xs[0].view(-1)[:7]  # ties
    dy = torch.randn(6, 4, 4, sum(widths) if kind == "Concatenate" else 12, generator=g).to(torch.bfloat16)
    dev = [x.cuda() for x in xs]
    out = torch.empty(dy.shape, dtype=torch.bfloat16, device="cuda")
    ops.merge_fwd(dev, out, kind)
    ref = torch.empty(dy.shape, dtype=torch.bfloat16)
    ops.merge_fwd(xs, ref, kind)
    torch.testing.assert_close(out.cpu().float(), ref.float(), rtol=1e-2, atol=1e-2)
    gd = [torch.empty_like(x) for x in dev]
    ops.merge_bwd(dev, dy.cuda(), gd, kind)
    gr = [torch.empty_like(x) for x in xs]
    ops.merge_bwd(xs, dy, gr, kind)
    for a, b in zip(gd, gr):
        torch.testing.assert_close(a.cpu().float(), b.float(), rtol=1e-2, atol=1e-2)


def test_branching_model_gpu_matches_cpu_fp32():
    from test_keras_graph import _functional
    from distriflow_amd.models.keras import layers_from_keras
    from distriflow_amd.models.net import Net

    topo = _functional([
        ("Conv2D", "c1", {"filters": 16, "kernel_size": [3, 3], "activation": "relu", "padding": "same"}, ["inp"]),
        ("Conv2D", "a1", {"filters": 16, "kernel_size": [3, 3], "activation": "relu", "padding": "same"}, ["c1"]),
        ("Conv2D", "b1", {"filters": 16, "kernel_size": [1, 1]}, ["c1"]),
        ("Add", "m", {}, ["a1", "b1"]),
        ("Concatenate", "cat", {"axis": -1}, ["m", "c1"]),
        ("MaxPooling2D", "p", {"pool_size": [2, 2]}, ["cat"]),
        ("Flatten", "f", {}, ["p"]),
        ("Dense", "d", {"units": 10, "activation": "softmax"}, ["f"]),
    ], (12, 12, 3), "d")
    lg, shape = layers_from_keras(topo)
    lc, _ = layers_from_keras(topo)
    gpu = Net(lg, shape, device="cuda", seed=2)
    cpu = Net(lc, shape, device="cpu", seed=2)
    cpu.store.master.copy_(gpu.store.master.cpu())
    x = torch.rand(32, 12, 12, 3)
    y = torch.randint(0, 10, (32,))
    sg = gpu.compute_gradients(x.cuda().to(torch.bfloat16), y.cuda().to(torch.int32))
    sc = cpu.compute_gradients(x, y)
    torch.cuda.synchronize()
    assert abs(float(sg[0]) - float(sc[0])) / 32 < 2e-2
    for s in cpu.store.specs:
        a, b = gpu.store.gradient(s.name).float().cpu().reshape(-1), cpu.store.gradient(s.name).reshape(-1)
        cos = float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-12))
        assert cos > 0.99, (s.name, cos)
