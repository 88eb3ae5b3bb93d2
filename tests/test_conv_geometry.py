"""Conv2D with any kernel / stride / padding geometry: non-square kernels, per-axis
strides and Keras 'same' padding whose odd total puts the extra row / column at the bottom / right.

Reference: ``fetchModel`` wraps any tf.LayersModel (/root/reference/src/common/utils.ts:236-244), whose
Conv2D takes any ``kernel_size`` / ``strides`` pair.  The fp32 reference ops (ops/reference.py) are checked
against a direct loop over the definition and by the adjoint identities of their gradients; the CPU engine
against torch autograd of the same model.  GPU kernels: tests/test_conv_geometry_gpu.py.
"""
import pytest
import torch
import torch.nn.functional as F

from distriflow_amd import ops
from distriflow_amd.models.keras import keras_config_from_layers, layers_from_keras
from distriflow_amd.models.layers import Conv2D
from distriflow_amd.models.net import Net
from distriflow_amd.ops import reference as ref

# (H, W, C, N, kernel, strides, padding)
GEOMS = [
    (9, 8, 3, 4, (3, 5), (2, 1), "same"),
    (8, 8, 2, 3, (3, 3), (2, 2), "same"),   # odd total: pad 0 top/left, 1 bottom/right
    (7, 10, 2, 5, (2, 4), (1, 2), "same"),  # even kernels
    (9, 11, 3, 2, (1, 3), (3, 2), "valid"),
    (6, 6, 4, 3, (5, 1), (1, 1), "same"),
]


def _direct_conv(x, w4, b, sh, sw, pt, pl, OH, OW):
    """out[b, oh, ow, n] = sum x[b, oh*sh - pt + kh, ow*sw - pl + kw, c] * w[n, c, kh, kw] (zero outside)."""
    B, H, W, C = x.shape
    N, _, KH, KW = w4.shape
    out = torch.zeros(B, OH, OW, N, dtype=torch.float64)
    for oh in range(OH):
        for ow in range(OW):
            for kh in range(KH):
                for kw in range(KW):
                    ih, iw = oh * sh - pt + kh, ow * sw - pl + kw
                    if 0 <= ih < H and 0 <= iw < W:
                        out[:, oh, ow] += x[:, ih, iw].double() @ w4[:, :, kh, kw].double().t()
    return out + (b.double() if b is not None else 0)


def _layer(H, W, C, N, k, s, p):
    conv = Conv2D(N, k, s, p, name="c")
    conv.build((H, W, C))
    return conv


@pytest.mark.parametrize("H,W,C,N,k,s,p", GEOMS)
def test_layer_geometry_matches_keras_same(H, W, C, N, k, s, p):
    conv = _layer(H, W, C, N, k, s, p)
    OH, OW, _ = conv.out_shape
    if p == "same":
        assert (OH, OW) == (-(-H // s[0]), -(-W // s[1]))
        th = max((OH - 1) * s[0] + k[0] - H, 0)
        assert conv.pads == (th // 2, max((OW - 1) * s[1] + k[1] - W, 0) // 2)
    else:
        assert (OH, OW) == ((H - k[0]) // s[0] + 1, (W - k[1]) // s[1] + 1)
    assert not conv.regular
    assert conv.config()["kernel_size"] == list(k) and conv.config()["strides"] == list(s)


def test_regular_geometry_keeps_scalar_fields():
    conv = _layer(8, 8, 3, 4, 3, 1, "same")
    assert conv.regular and (conv.k, conv.stride, conv.pad) == (3, 1, 1)
    assert conv.geom == (3, 3, 1, 1)
    conv = _layer(9, 9, 3, 4, (3, 3), (2, 2), "same")  # total 2: symmetric
    assert conv.regular and conv.pad == 1


@pytest.mark.parametrize("H,W,C,N,k,s,p", GEOMS)
def test_reference_ops_match_definition_and_adjoints(H, W, C, N, k, s, p):
    conv = _layer(H, W, C, N, k, s, p)
    KH, KW, st, pd = conv.geom
    OH, OW, _ = conv.out_shape
    g = torch.Generator().manual_seed(H * 31 + W)
    x = torch.randn(2, H, W, C, generator=g)
    w4 = torch.randn(N, C, KH, KW, generator=g)
    b = torch.randn(N, generator=g)
    w2d = w4.permute(0, 2, 3, 1).reshape(N, KH * KW * C)
    y = ref.conv_fwd(x, w2d, b, KH, KW, st, pd, False, out_hw=(OH, OW))
    exp = _direct_conv(x, w4, b, conv.sh, conv.sw, conv.pads[0], conv.pads[1], OH, OW)
    torch.testing.assert_close(y.double(), exp, rtol=1e-4, atol=1e-4)
    dy = torch.randn(2, OH, OW, N, generator=g)
    # <conv(x), dy> = <x, dgrad(dy)> and = <w, wgrad(x, dy)> (the conv is bilinear)
    lin = (ref.conv_fwd(x, w2d, None, KH, KW, st, pd, False, out_hw=(OH, OW)).double() * dy.double()).sum()
    dx = ref.conv_dgrad(dy, w2d, x.shape, KH, KW, st, pd)
    gw, gb = ref.conv_wgrad(dy, x, KH, KW, st, pd)
    assert abs(float((x.double() * dx.double()).sum() - lin)) <= 1e-4 * max(1.0, abs(float(lin)))
    assert abs(float((w2d.double() * gw.double()).sum() - lin)) <= 1e-4 * max(1.0, abs(float(lin)))
    torch.testing.assert_close(gb, dy.sum(dim=(0, 1, 2)))


def _topo(H, W, C, k, s, p):
    return {"class_name": "Sequential", "config": {"name": "m", "layers": [
        {"class_name": "Conv2D", "config": {"name": "c1", "filters": 6, "kernel_size": list(k), "strides": list(s),
                                            "padding": p, "activation": "relu", "batch_input_shape": [None, H, W, C]}},
        {"class_name": "Conv2D", "config": {"name": "c2", "filters": 8, "kernel_size": [1, 3], "strides": [1, 2],
                                            "padding": "same", "activation": "tanh"}},
        {"class_name": "Flatten", "config": {"name": "f"}},
        {"class_name": "Dense", "config": {"name": "d", "units": 4, "activation": "softmax"}}]}}


@pytest.mark.parametrize("H,W,C,N,k,s,p", GEOMS[:3])
def test_engine_grads_match_autograd(H, W, C, N, k, s, p):
    topo = _topo(H, W, C, k, s, p)
    layers, shape = layers_from_keras(topo)
    net = Net(layers, shape, device="cpu", seed=5)
    x = torch.rand(5, H, W, C)
    y = torch.randint(0, 4, (5,))
    st = net.compute_gradients(x, y)
    P = {sp.name: net.store[sp.name].detach().clone().requires_grad_(True) for sp in net.store.specs}

    def tconv(h, name, kk, ss, pads_out):
        (ph, pw), (OH, OW) = pads_out
        H_, W_ = h.shape[2], h.shape[3]
        pb = (OH - 1) * ss[0] + kk[0] - H_ - ph
        pr = (OW - 1) * ss[1] + kk[1] - W_ - pw
        return F.conv2d(F.pad(h, (pw, pr, ph, pb)), P[f"{name}/kernel"].permute(0, 3, 1, 2), P[f"{name}/bias"],
                        stride=ss)

    c1, c2 = layers[0], layers[1]
    h = F.relu(tconv(x.permute(0, 3, 1, 2), "c1", k, s, (c1.pads, c1.out_shape[:2])))
    h = torch.tanh(tconv(h, "c2", (1, 3), (1, 2), (c2.pads, c2.out_shape[:2])))
    z = F.linear(h.permute(0, 2, 3, 1).reshape(5, -1), P["d/kernel"], P["d/bias"])
    loss = F.cross_entropy(z, y)
    loss.backward()
    assert abs(float(st[0]) / 5 - loss.item()) < 1e-4
    for sp in net.store.specs:
        torch.testing.assert_close(net.store.gradient(sp.name), P[sp.name].grad, rtol=1e-4, atol=1e-5)


def test_keras_round_trip_keeps_geometry():
    topo = _topo(9, 8, 3, (3, 5), (2, 1), "same")
    layers, _ = layers_from_keras(topo)
    back = keras_config_from_layers(layers, (9, 8, 3))
    convs = [l["config"] for l in back["config"]["layers"] if l["class_name"] == "Conv2D"]
    assert convs[0]["kernel_size"] == [3, 5] and convs[0]["strides"] == [2, 1] and convs[0]["padding"] == "same"
    assert convs[1]["kernel_size"] == [1, 3] and convs[1]["strides"] == [1, 2]


def test_native_geometry_encoding():
    assert ops._geom(8, 8, 3, 4, 4, 3, 3, 2, 1) == [8, 8, 3, 4, 4, 3, 3, 2, 1]
    assert ops._geom(9, 8, 3, 5, 8, 3, 5, (2, 1), (1, 2)) == [9, 8, 3, 5, 8, 3, 5, 2, 1, 1, 2]


def test_tfjs_checkpoint_round_trip_keeps_non_square_kernels(tmp_path):
    """A (3, 5) / stride (2, 1) Conv2D saves as Keras HWIO [3][5][C][N] and reloads into a fresh model that
    computes the same function (rebuilt from the saved model.json's topology)."""
    import json as _json

    from distriflow_amd.checkpoint import load_layers_model_weights, save_layers_model

    topo = _topo(9, 8, 3, (3, 5), (2, 1), "same")
    layers, shape = layers_from_keras(topo)
    a = Net(layers, shape, device="cpu", seed=1)
    save_layers_model(a, str(tmp_path / "m"))
    doc = _json.load(open(tmp_path / "m" / "model.json"))
    shapes = {w["name"]: w["shape"] for w in doc["weightsManifest"][0]["weights"]}
    assert shapes["c1/kernel"] == [3, 5, 3, 6] and shapes["c2/kernel"] == [1, 3, 6, 8]
    layers_b, shape_b = layers_from_keras(doc["modelTopology"])
    b = Net(layers_b, shape_b, device="cpu", seed=2)
    load_layers_model_weights(b, str(tmp_path / "m" / "model.json"))
    assert torch.equal(a.store.master, b.store.master)
    x = torch.rand(3, 9, 8, 3)
    torch.testing.assert_close(a.predict(x), b.predict(x))
