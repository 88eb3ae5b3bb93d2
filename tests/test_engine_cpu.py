"""The explicit-backward engine (CPU fp32 path) against torch autograd on an equivalent nn.Module."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from distriflow_amd.models.layers import Conv2D, ConvPoolGemm, Dense, FusedConvPool, MaxPooling2D, ResidualBlock, \
    BatchNorm, GlobalAveragePooling2D
from distriflow_amd.models.net import Net
from distriflow_amd.models.zoo import MODELS, build_model


def torch_forward(net: Net, x: torch.Tensor, params: dict):
    """Re-implement the engine model with autograd ops (NHWC in, logits out)."""
    h = x.permute(0, 3, 1, 2)
    for l in net.exec_layers:
        if isinstance(l, (Conv2D, FusedConvPool, ConvPoolGemm)):
            c = l.conv if isinstance(l, (FusedConvPool, ConvPoolGemm)) else l
            w = params[f"{l.name}/kernel"].permute(0, 3, 1, 2)
            b = params.get(f"{l.name}/bias")
            h = F.conv2d(h, w, b, stride=c.stride, padding=c.pad)
            if c.relu:
                h = F.relu(h)
            if isinstance(l, (FusedConvPool, ConvPoolGemm)):
                h = F.max_pool2d(h, 2)
        elif isinstance(l, MaxPooling2D):
            h = F.max_pool2d(h, l.p)
        elif hasattr(l, "rate"):  # Dropout with rate 0 in these tests
            pass
        elif isinstance(l, Dense):
            if h.dim() == 4:
                h = h.permute(0, 2, 3, 1).reshape(h.shape[0], -1)  # Keras channels_last flatten order
            h = F.linear(h, params[f"{l.name}/kernel"], params.get(f"{l.name}/bias"))
            if l.relu:
                h = F.relu(h)
        else:
            raise NotImplementedError(type(l))
    return h


@pytest.mark.parametrize("name", ["mlp_mnist", "lenet5", "keras_cnn"])
@pytest.mark.parametrize("fuse", [True, False])
def test_grads_match_autograd(name, fuse):
    layers, shape = MODELS[name]()
    net = Net(layers, shape, device="cpu", seed=1, fuse=fuse)
    for l in net.exec_layers:  # dropout off for the comparison
        if hasattr(l, "rate"):
            l.rate = 0.0
    torch.manual_seed(0)
    x = torch.rand(6, *shape)
    y = torch.randint(0, net.num_classes, (6,))
    st = net.compute_gradients(x, y)
    params = {s.name: net.store[s.name].detach().clone().requires_grad_(True) for s in net.store.specs}
    logits = torch_forward(net, x, params)
    loss = F.cross_entropy(logits, y, reduction="mean")
    loss.backward()
    assert abs(float(st[0]) / 6 - loss.item()) < 1e-4
    for s in net.store.specs:
        torch.testing.assert_close(net.store.gradient(s.name), params[s.name].grad, rtol=1e-4, atol=1e-5)


def test_resnet_block_grads_match_autograd():
    layers = [Conv2D(8, 3, 1, 1, use_bias=False, name="stem"), BatchNorm(relu=True, name="bn"),
              ResidualBlock(8, 1, name="b1"), ResidualBlock(16, 2, name="b2"), GlobalAveragePooling2D(name="gap"),
              Dense(10, name="fc")]
    net = Net(layers, (8, 8, 3), device="cpu", seed=2)
    x = torch.rand(4, 8, 8, 3)
    y = torch.randint(0, 10, (4,))
    net.compute_gradients(x, y)
    P = {s.name: net.store[s.name].detach().clone().requires_grad_(True) for s in net.store.specs}

    def conv(h, n, s, p):
        return F.conv2d(h, P[f"{n}/kernel"].permute(0, 3, 1, 2), None, stride=s, padding=p)

    def bn(h, n):
        return F.batch_norm(h, None, None, P[f"{n}/gamma"], P[f"{n}/beta"], training=True, eps=1e-5)

    def block(h, n, s, proj):
        o = F.relu(bn(conv(h, f"{n}/conv1", s, 1), f"{n}/bn1"))
        o = bn(conv(o, f"{n}/conv2", 1, 1), f"{n}/bn2")
        sc = bn(conv(h, f"{n}/proj", s, 0), f"{n}/proj_bn") if proj else h
        return F.relu(o + sc)

    h = x.permute(0, 3, 1, 2)
    h = F.relu(bn(conv(h, "stem", 1, 1), "bn"))
    h = block(h, "b1", 1, False)
    h = block(h, "b2", 2, True)
    h = h.mean(dim=(2, 3))
    logits = F.linear(h, P["fc/kernel"], P["fc/bias"])
    F.cross_entropy(logits, y).backward()
    for s in net.store.specs:
        torch.testing.assert_close(net.store.gradient(s.name), P[s.name].grad, rtol=1e-3, atol=1e-5)


def test_fusion_plan_and_param_counts():
    assert build_model("mlp_mnist", "cpu").num_params() == 7960
    assert build_model("keras_cnn", "cpu").num_params() == 600165
    assert build_model("lenet5", "cpu").num_params() == 61706
    net = build_model("lenet5", "cpu")
    kinds = [type(l).__name__ for l in net.exec_layers]
    assert kinds == ["FusedConvPool", "FusedConvPool", "Dense", "Dense", "Dense"]
    assert net.exec_layers[0].need_dx is False


def test_sgd_cpu_matches_formula():
    net = build_model("mlp_mnist", "cpu")
    st = net.store
    st.grad.normal_()
    w0 = st.master.clone()
    st.set_hyper(0.1, momentum=0.9, grad_scale=0.5)
    st.sgd_step()
    for sp in st.specs:
        o = st.offsets[sp.name]
        sl = slice(o, o + sp.numel)
        torch.testing.assert_close(st.master[sl], w0[sl] - 0.1 * (0.5 * st.grad[sl]))


def test_training_converges_on_synthetic_mnist():
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer, epoch_permutations

    net = build_model("mlp_mnist", "cpu", seed=0)
    x, y = synthetic_mnist(2048)
    tr = DataParallelTrainer(net, lr=0.1, graph="none")
    tr.bind_dataset(x, y, 64, scale=1 / 255)
    perm = epoch_permutations(2048, 64, 60, "cpu")
    first = float(tr.step_indices(perm[0])[0]) / 64
    for i in range(1, 60):
        st = tr.step_indices(perm[i])
    assert float(st[0]) / 64 < 0.5 * first


def test_index_stream_cpu_eager():
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer, epoch_permutations

    data, labels = synthetic_mnist(512, seed=2)
    perm = epoch_permutations(512, 32, 3, "cpu", seed=4)
    outs = []
    for mode in ("explicit", "stream"):
        net = build_model("mlp_mnist", device="cpu", seed=0)
        tr = DataParallelTrainer(net, lr=0.1, graph="none")
        tr.bind_dataset(data, labels, 32, scale=1 / 255)
        if mode == "explicit":
            for i in range(3):
                tr.step_indices(perm[i])
        else:
            tr.bind_index_stream(perm)
            for _ in range(3):
                tr.step()
        outs.append(net.store.master.clone())
    assert torch.equal(outs[0], outs[1])
