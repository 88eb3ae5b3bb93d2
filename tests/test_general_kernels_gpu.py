"""csrc/act.hip against fp32 PyTorch references of the same ops (bf16-rounded inputs): standalone
activations forward / backward, sigmoid cross-entropy, general max / average pooling; plus a general
Keras model (tanh, same-padded pools, sigmoid output) trained on the GPU engine against the CPU fp32
engine, layer for layer.  Reference: tf.LayersModel generality (/root/reference/src/common/utils.ts:236-244)."""
import pytest
import torch
import torch.nn.functional as F

from distriflow_amd import ops

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)

ACTS = ["relu", "relu6", "sigmoid", "tanh", "elu", "selu", "softplus", "softsign", "hard_sigmoid", "swish",
        "exponential", "linear"]


@pytest.mark.parametrize("act", ACTS)
@pytest.mark.parametrize("n", [8 * 1001, 999])
def test_act_fwd_bwd(act, n):
    g = torch.Generator().manual_seed(1)
    x = (torch.randn(n, generator=g) * 3).to(torch.bfloat16)
    dy = torch.randn(n, generator=g).to(torch.bfloat16)
    xd, dyd = x.to(dev), dy.to(dev)
    y = torch.empty_like(xd)
    ops.act_fwd(xd, y, act)
    ref = ops._act_ref(ops.ACT_KINDS[act], x.float())
    torch.testing.assert_close(y.float().cpu(), ref, rtol=2e-2, atol=2e-2)
    for in_relu in (False, True):
        dx = torch.empty_like(xd)
        ops.act_bwd(xd, dyd, dx, act, in_relu=in_relu)
        xv = x.float().requires_grad_(True)
        (gr,) = torch.autograd.grad(ops._act_ref(ops.ACT_KINDS[act], xv), xv, dy.float())
        if in_relu:
            gr = gr * (x.float() > 0)
        torch.testing.assert_close(dx.float().cpu(), gr, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("B,C", [(1, 1), (300, 10), (257, 37)])
def test_sigmoid_ce(B, C):
    g = torch.Generator().manual_seed(2)
    z = torch.randn(B, C, generator=g) * 4
    y = torch.randint(0, C, (B,), generator=g, dtype=torch.int32)
    dl = torch.empty(B, C, dtype=torch.bfloat16, device=dev)
    st = torch.zeros(2, device=dev)
    ops.sigmoid_ce(z.to(dev), y.to(dev), dl, st, grad_scale=1.0 / B)
    t = F.one_hot(y.long(), C).float()
    loss = F.binary_cross_entropy_with_logits(z, t, reduction="sum")
    assert abs(float(st[0]) - loss.item()) <= 1e-4 * abs(loss.item()) + 1e-3
    assert float(st[1]) == float((z.argmax(1) == y.long()).sum())
    torch.testing.assert_close(dl.float().cpu(), (torch.sigmoid(z) - t) / B, rtol=1e-2, atol=1e-4)


@pytest.mark.parametrize("H,C,pool,stride,pad,avg", [
    (28, 32, (2, 2), (2, 2), "same", False),
    (13, 8, (3, 3), (2, 2), "same", False),
    (13, 8, (3, 3), (2, 2), "same", True),
    (12, 5, (3, 3), (1, 1), "valid", True),
    (7, 3, (2, 3), (2, 1), "valid", False),
    (9, 16, (9, 9), (9, 9), "valid", False),  # a global max pool
])
def test_pool2d(H, C, pool, stride, pad, avg):
    g = torch.Generator().manual_seed(3)
    B = 3
    x = torch.randn(B, H, H, C, generator=g).relu().to(torch.bfloat16)
    geom = ops.pool_geometry(B, H, H, C, pool, stride, pad)
    OH, OW = geom[4], geom[5]
    y = torch.empty(B, OH, OW, C, dtype=torch.bfloat16, device=dev)
    ops.pool2d_fwd(x.to(dev), y, geom, avg=avg)
    ref = ops._pool_ref(x.float(), geom, avg)
    torch.testing.assert_close(y.float().cpu(), ref, rtol=1e-2, atol=1e-2)
    dy = torch.randn(B, OH, OW, C, generator=g).to(torch.bfloat16)
    for in_relu in (False, True):
        dx = torch.empty(B, H, H, C, dtype=torch.bfloat16, device=dev)
        ops.pool2d_bwd(x.to(dev), dy.to(dev), dx, geom, avg=avg, in_relu=in_relu)
        xv = x.float().requires_grad_(True)
        (gr,) = torch.autograd.grad(ops._pool_ref(xv, geom, avg), xv, dy.float())
        if in_relu:
            if avg:
                gr = gr * (x.float() > 0)
            else:  # a window whose max is not positive passes nothing
                mx = ops._pool_ref(x.float(), geom, False)
                gr = torch.autograd.grad(ops._pool_ref(xv, geom, False), xv, dy.float() * (mx > 0))[0]
        torch.testing.assert_close(dx.float().cpu(), gr, rtol=2e-2, atol=2e-2)


def test_general_keras_model_gpu_matches_cpu_engine():
    from distriflow_amd.models.keras import layers_from_keras
    from distriflow_amd.models.net import Net

    topo = {"class_name": "Sequential", "config": {"name": "g", "layers": [
        {"class_name": "Conv2D", "config": {"name": "c1", "filters": 8, "kernel_size": [3, 3], "activation": "tanh",
                                            "padding": "same", "batch_input_shape": [None, 14, 14, 1]}},
        {"class_name": "MaxPooling2D", "config": {"name": "p1", "pool_size": [3, 3], "strides": [2, 2],
                                                  "padding": "same"}},
        {"class_name": "Conv2D", "config": {"name": "c2", "filters": 16, "kernel_size": [3, 3], "activation": "relu"}},
        {"class_name": "AveragePooling2D", "config": {"name": "p2", "pool_size": [2, 2], "padding": "same"}},
        {"class_name": "Flatten", "config": {"name": "f"}},
        {"class_name": "Dense", "config": {"name": "d1", "units": 32, "activation": "elu"}},
        {"class_name": "Dense", "config": {"name": "d2", "units": 6, "activation": "sigmoid"}}]}}
    g = torch.Generator().manual_seed(4)
    x = torch.rand(64, 14, 14, 1, generator=g)
    y = torch.randint(0, 6, (64,), generator=g)
    nets = {}
    for d in ("cpu", "cuda"):
        layers, shape = layers_from_keras(topo)
        nets[d] = Net(layers, shape, device=d, seed=9)
    nets["cuda"].store.master.copy_(nets["cpu"].store.master.to(dev))
    nets["cuda"].store.refresh_compute()
    xb = x.to(torch.bfloat16).float()  # the GPU engine computes on bf16 inputs
    st_c = nets["cpu"].compute_gradients(xb, y)
    st_g = nets["cuda"].compute_gradients(xb.to(dev), y.to(dev))
    torch.cuda.synchronize()
    assert nets["cuda"].final_act == "sigmoid"
    assert abs(float(st_g[0]) - float(st_c[0])) <= 0.02 * abs(float(st_c[0]))
    for s in nets["cpu"].store.specs:
        a = nets["cpu"].store.gradient(s.name).flatten()
        b = nets["cuda"].store.gradient(s.name).flatten().cpu()
        cos = float(F.cosine_similarity(a, b, dim=0))
        assert cos > 0.99, (s.name, cos)
