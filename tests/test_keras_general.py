"""General tf.js LayersModel support (VERDICT r2 Missing 4): any Keras activation, max / average pooling
with any window / stride / 'same' padding, global pooling, sigmoid outputs trained with sigmoid
cross-entropy, and single-chain functional models.

Reference: ``fetchModel`` wraps any tf.LayersModel (/root/reference/src/common/utils.ts:236-244) and the
loss registry includes sigmoidCrossEntropy (utils.ts:19-30).  The CPU fp32 engine is checked against
torch autograd on the same graph; the GPU kernels against fp32 references in tests/test_kernels_gpu.py.
"""
import json

import pytest
import torch
import torch.nn.functional as F

from distriflow_amd.models.keras import keras_config_from_layers, layers_from_keras
from distriflow_amd.models.net import Net


def _seq(layers, input_shape):
    out = []
    for i, (cls, cfg) in enumerate(layers):
        c = dict(cfg, name=cfg.get("name", f"l{i}"))
        if i == 0:
            c["batch_input_shape"] = [None, *input_shape]
        out.append({"class_name": cls, "config": c})
    return {"class_name": "Sequential", "config": {"name": "m", "layers": out}}


ACTS = ["tanh", "sigmoid", "elu", "selu", "softplus", "softsign", "hard_sigmoid", "swish", "relu6"]


def _torch_act(name, h):
    return {"tanh": torch.tanh, "sigmoid": torch.sigmoid, "elu": F.elu, "selu": F.selu, "softplus": F.softplus,
            "softsign": F.softsign, "hard_sigmoid": lambda v: _clip(0.2 * v + 0.5, 0, 1), "swish": F.silu,
            "relu6": lambda v: _clip(v, 0, 6), "relu": F.relu, "linear": lambda v: v}[name](h)


def _clip(v, lo, hi):  # TensorFlow's gradient of relu6 / hard_sigmoid is zero at the corners
    return torch.where((v > lo) & (v < hi), v, v.clamp(lo, hi).detach())


@pytest.mark.parametrize("act", ACTS)
def test_dense_activation_grads_match_autograd(act):
    topo = _seq([("Dense", {"units": 12, "activation": act}), ("Dense", {"units": 5, "activation": "softmax"})],
                (7,))
    layers, shape = layers_from_keras(topo)
    net = Net(layers, shape, device="cpu", seed=3)
    x = torch.randn(6, 7)
    y = torch.randint(0, 5, (6,))
    st = net.compute_gradients(x, y)
    P = {s.name: net.store[s.name].detach().clone().requires_grad_(True) for s in net.store.specs}
    h = _torch_act(act, F.linear(x, P["l0/kernel"], P["l0/bias"]))
    z = F.linear(h, P["l1/kernel"], P["l1/bias"])
    loss = F.cross_entropy(z, y)
    loss.backward()
    assert abs(float(st[0]) / 6 - loss.item()) < 1e-4
    for s in net.store.specs:
        torch.testing.assert_close(net.store.gradient(s.name), P[s.name].grad, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("pool,strides,padding,cls", [
    ((2, 2), None, "same", "MaxPooling2D"),
    ((3, 3), (2, 2), "valid", "MaxPooling2D"),
    ((3, 3), (1, 1), "same", "MaxPooling2D"),
    ((2, 2), None, "valid", "AveragePooling2D"),
    ((3, 3), (2, 2), "same", "AveragePooling2D"),
])
def test_pooling_grads_match_autograd(pool, strides, padding, cls):
    topo = _seq([("Conv2D", {"filters": 4, "kernel_size": [3, 3], "activation": "relu", "padding": "same"}),
                 (cls, {"pool_size": list(pool), "strides": strides, "padding": padding}),
                 ("Flatten", {}), ("Dense", {"units": 3})], (7, 7, 2))
    layers, shape = layers_from_keras(topo)
    net = Net(layers, shape, device="cpu", seed=4)
    x = torch.rand(5, 7, 7, 2)
    y = torch.randint(0, 3, (5,))
    st = net.compute_gradients(x, y)
    P = {s.name: net.store[s.name].detach().clone().requires_grad_(True) for s in net.store.specs}
    h = F.relu(F.conv2d(x.permute(0, 3, 1, 2), P["l0/kernel"].permute(0, 3, 1, 2), P["l0/bias"], padding=1))
    s = strides or pool
    H = 7
    if padding == "same":
        OH = -(-H // s[0])
        tot = max((OH - 1) * s[0] + pool[0] - H, 0)
        pt, pb = tot // 2, tot - tot // 2
    else:
        pt = pb = 0
    if cls == "MaxPooling2D":
        h = F.max_pool2d(F.pad(h, (pt, pb, pt, pb), value=float("-inf")), pool, s)
    else:  # TF averages over the in-image pixels only
        num = F.avg_pool2d(F.pad(h, (pt, pb, pt, pb)), pool, s, divisor_override=1)
        cnt = F.avg_pool2d(F.pad(torch.ones(1, 1, H, H), (pt, pb, pt, pb)), pool, s, divisor_override=1)
        h = num / cnt
    z = F.linear(h.permute(0, 2, 3, 1).reshape(5, -1), P["l3/kernel"], P["l3/bias"])
    loss = F.cross_entropy(z, y)
    loss.backward()
    assert net.exec_layers[1].out_shape == tuple(h.shape[2:]) + (4,)
    assert abs(float(st[0]) / 5 - loss.item()) < 1e-4
    for sp in net.store.specs:
        torch.testing.assert_close(net.store.gradient(sp.name), P[sp.name].grad, rtol=1e-4, atol=1e-5)


def test_sigmoid_output_trains_sigmoid_ce_and_evaluates():
    """A model.json ending in sigmoid trains sigmoid cross-entropy on its logits and evaluates with the
    reference's sigmoidCrossEntropy loss."""
    from distriflow_amd.models.distri_model import EngineModel

    topo = _seq([("Dense", {"units": 16, "activation": "tanh"}), ("Dense", {"units": 4}),
                 ("Activation", {"activation": "sigmoid"})], (6,))
    layers, shape = layers_from_keras(topo)
    net = Net(layers, shape, device="cpu", seed=5)
    assert net.final_act == "sigmoid"
    x = torch.randn(8, 6)
    y = torch.randint(0, 4, (8,))
    st = net.compute_gradients(x, y)
    P = {s.name: net.store[s.name].detach().clone().requires_grad_(True) for s in net.store.specs}
    z = F.linear(torch.tanh(F.linear(x, P["l0/kernel"], P["l0/bias"])), P["l1/kernel"], P["l1/bias"])
    t = F.one_hot(y, 4).float()
    loss = F.binary_cross_entropy_with_logits(z, t, reduction="sum") / 8
    loss.backward()
    assert abs(float(st[0]) / 8 - loss.item()) < 1e-4
    for s in net.store.specs:
        torch.testing.assert_close(net.store.gradient(s.name), P[s.name].grad, rtol=1e-4, atol=1e-5)
    # training through the DistriModel contract lowers the loss; predict() returns sigmoid probabilities
    m = EngineModel(net, {"loss": "sigmoidCrossEntropy", "learningRate": 0.5, "metrics": ["accuracy"]})
    X = torch.randn(64, 6)
    Y = (X[:, :4].argmax(1))
    l0 = m.evaluate(X, Y)[0]
    for _ in range(60):
        g = m.fit(X, Y)
        m.update(g)
    l1, acc = m.evaluate(X, Y)
    assert l1 < l0 and acc > 0.5
    p = m.predict(X[:3])
    assert float(p.min()) >= 0.0 and float(p.max()) <= 1.0
    assert not torch.allclose(p.sum(1), torch.ones(3))  # not a softmax


def test_functional_chain_model_loads_like_sequential():
    seq = _seq([("Conv2D", {"filters": 3, "kernel_size": [3, 3], "activation": "elu"}),
                ("MaxPooling2D", {"pool_size": [2, 2], "padding": "same"}), ("Flatten", {}),
                ("Dense", {"units": 4, "activation": "softmax"})], (6, 6, 1))
    lcs = seq["config"]["layers"]
    fl = [{"class_name": "InputLayer", "name": "inp",
           "config": {"name": "inp", "batch_input_shape": [None, 6, 6, 1]}, "inbound_nodes": []}]
    prev = "inp"
    for lc in lcs:
        c = dict(lc["config"])
        c.pop("batch_input_shape", None)
        fl.append({"class_name": lc["class_name"], "name": c["name"], "config": c,
                   "inbound_nodes": [[[prev, 0, 0, {}]]]})
        prev = c["name"]
    fl = [fl[0], fl[3], fl[1], fl[4], fl[2]]  # layer order in the JSON is not execution order
    func = {"class_name": "Model", "config": {"name": "f", "layers": fl, "input_layers": [["inp", 0, 0]],
                                              "output_layers": [[prev, 0, 0]]}}
    la, sa = layers_from_keras(seq)
    lb, sb = layers_from_keras(json.loads(json.dumps(func)))
    assert sa == sb and [type(l) for l in la] == [type(l) for l in lb] and [l.name for l in la] == [l.name for l in lb]
    na, nb = Net(la, sa, device="cpu", seed=7), Net(lb, sb, device="cpu", seed=7)
    x = torch.rand(3, 6, 6, 1)
    torch.testing.assert_close(na.predict(x), nb.predict(x))
    # a non-merge layer with two inputs is refused with a clear error (joins go through merge layers,
    # tests/test_keras_graph.py), and so is a cycle
    bad = json.loads(json.dumps(func))
    bad["config"]["layers"][-1]["inbound_nodes"] = [[["l0", 0, 0, {}], ["inp", 0, 0, {}]]]
    with pytest.raises(NotImplementedError):
        layers_from_keras(bad)
    bad["config"]["layers"][-1]["inbound_nodes"] = [[["l1", 0, 0, {}]]]
    with pytest.raises(ValueError):
        layers_from_keras(bad)


def test_export_roundtrip_keeps_general_layers():
    topo = _seq([("Conv2D", {"filters": 2, "kernel_size": [3, 3], "activation": "tanh", "padding": "same"}),
                 ("AveragePooling2D", {"pool_size": [3, 3], "strides": [2, 2], "padding": "same"}),
                 ("GlobalMaxPooling2D", {}), ("Dense", {"units": 3, "activation": "sigmoid"})], (5, 5, 1))
    layers, shape = layers_from_keras(topo)
    net = Net(layers, shape, device="cpu", seed=1)
    again, shape2 = layers_from_keras(keras_config_from_layers(net.layers_all, net.input_shape))
    assert shape2 == shape
    assert [type(l).__name__ for l in again] == [type(l).__name__ for l in layers]
    assert [getattr(l, "activation", None) for l in again] == [getattr(l, "activation", None) for l in layers]
    net2 = Net(again, shape2, device="cpu", seed=1)
    x = torch.rand(2, 5, 5, 1)
    torch.testing.assert_close(net.predict(x), net2.predict(x))
