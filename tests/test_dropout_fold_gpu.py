"""Dropout folded into its producer (Net._fold_dropout): the Dense+ReLU epilogues (plain and split-K)
and the max-pool kernel write exactly what the standalone dropout launch wrote after them, and the
Keras CNN (model.json: pool -> dropout -> dense -> dropout -> dense) runs with no dropout launch while
its gradients still match the fp32 CPU reference."""
import pytest
import torch

from distriflow_amd import ops

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


def _pad_w(w):
    N, K = w.shape
    out = torch.zeros((N + 15) // 16 * 16, (K + 31) // 32 * 32, dtype=torch.bfloat16, device=dev)
    out[:N, :K] = w.to(torch.bfloat16)
    return out


@pytest.mark.parametrize("B,K,N,p", [(64, 256, 128, 0.5), (1024, 9216, 128, 0.5), (96, 64, 40, 0.25)])
def test_dense_epilogue_dropout_is_the_standalone_mask(B, K, N, p):
    x = torch.randn(B, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev) / K ** 0.5
    b = torch.randn(N, device=dev) * 0.1
    step = torch.tensor(7, dtype=torch.int64, device=dev)
    plain = torch.empty(B, N, dtype=torch.bfloat16, device=dev)
    ops.dense_fwd(x, _pad_w(w), b, plain, relu=True)
    ref = torch.empty_like(plain)
    ops.dropout(plain, ref, p, 1234, step=step)
    out = torch.empty_like(ref)
    ops.dense_fwd(x, _pad_w(w), b, out, relu=True, drop=(p, 1234, step))
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    kept = (out > 0)[plain > 0].float().mean().item()
    assert abs(kept - (1 - p)) < 0.06


@pytest.mark.parametrize("p", [0.25, 0.5])
def test_maxpool_dropout_is_the_standalone_mask(p):
    x = torch.relu(torch.randn(8, 24, 24, 64, device=dev)).to(torch.bfloat16)
    step = torch.tensor(3, dtype=torch.int64, device=dev)
    ref = torch.empty(8, 12, 12, 64, dtype=torch.bfloat16, device=dev)
    ops.maxpool_fwd(x, ref, 2)
    ops.dropout(ref, ref, p, 99, step=step)
    out = torch.empty_like(ref)
    ops.maxpool_fwd(x, out, 2, drop=(p, 99, step))
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("B,H,C,N,pad,drop", [(4, 26, 32, 64, 0, None), (3, 14, 16, 32, 1, 0.25),
                                               (2, 12, 8, 16, 0, 0.5)])
def test_pooled_conv_epilogue_equals_conv_then_pool(B, H, C, N, pad, drop):
    """igemm64 POOL: the pooled map equals conv (bf16 out) -> max-pool [-> dropout], bitwise; the unpooled
    gradient from its codes equals maxpool_bwd over the unpooled conv output (relu fused)."""
    x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
    w = torch.randn(N, 9 * C, device=dev) / (9 * C) ** 0.5
    b = torch.randn(N, device=dev) * 0.1
    OH = H + 2 * pad - 2
    assert ops.conv_pool_supported(H, H, C, 3, 3, 1, pad, N)
    y = torch.empty(B, OH, OH, N, dtype=torch.bfloat16, device=dev)
    ops.conv_fwd(x, _pad_w(w), b, y, 3, 3, 1, pad, relu=True)
    step = torch.tensor(5, dtype=torch.int64, device=dev)
    dspec = None if drop is None else (drop, 77, step)
    ref = torch.empty(B, OH // 2, OH // 2, N, dtype=torch.bfloat16, device=dev)
    ops.maxpool_fwd(y, ref, 2, drop=dspec)
    out = torch.empty_like(ref)
    code = torch.empty(ref.shape, dtype=torch.uint8, device=dev)
    ops.conv_pool_fwd(x, _pad_w(w), b, out, code, 3, 3, 1, pad, relu=True, drop=dspec)
    dyp = torch.randn(ref.shape, device=dev).to(torch.bfloat16)
    d_ref = torch.empty_like(y)
    ops.maxpool_bwd(y, dyp, d_ref, 2, relu_fused=True)
    d_out = torch.empty_like(y)
    ops.unpool2(dyp, code, d_out)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert torch.equal(d_out, d_ref)


def test_keras_cnn_plan_has_no_dropout_launch():
    from distriflow_amd.models.layers import ConvPoolGemm, Dense, Dropout, KerasConvBlock, MaxPooling2D
    from distriflow_amd.models.zoo import build_model

    net = build_model("keras_cnn", device=dev, seed=0)
    kinds = [type(l) for l in net.exec_layers]
    assert Dropout not in kinds and MaxPooling2D not in kinds
    pool = next(l for l in net.exec_layers if isinstance(l, (ConvPoolGemm, KerasConvBlock)))
    assert pool.drop is not None and pool.drop.rate == 0.25
    dense = [l for l in net.exec_layers if isinstance(l, Dense)]
    assert dense[0].drop is not None and dense[0].in_relu and abs(dense[0].dx_scale - 1 / 0.75) < 1e-12
    # the reference CNN's two dense layers form the split-K head (csrc/khead.hip); otherwise the logits
    # layer alone is the fused head
    assert net.khead and net.head_start == len(net.exec_layers) - 2
    assert dense[1].in_relu and dense[1].dx_scale == 2.0


def test_gather_advances_the_dropout_step():
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model

    net = build_model("keras_cnn", device=dev, seed=0)
    data, labels = synthetic_mnist(512, seed=1, device=dev)
    idx = torch.arange(64, device=dev)
    x, y = ops.GatherRef(data, idx, 1 / 255.0, (28, 28, 1)), ops.LabelRef(labels, idx)
    s0 = int(net.step_dev.item())
    g1 = net.compute_gradients(x, y).clone()
    gr1 = net.store.grad.clone()
    net.compute_gradients(x, y)
    gr2 = net.store.grad.clone()
    torch.cuda.synchronize()
    assert int(net.step_dev.item()) == s0 + 2
    assert torch.isfinite(g1).all()
    assert not torch.equal(gr1, gr2)  # a fresh dropout mask per step
