"""GPU conv kernels on irregular geometry (non-square kernels, per-axis strides, asymmetric Keras 'same'):
the generic implicit-GEMM kernels (csrc/igemm.hip) against the fp32 reference ops, and a Keras model with
such convs trained on the GPU engine against the CPU engine.  CPU side: tests/test_conv_geometry.py."""
import pytest
import torch
import torch.nn.functional as F

from distriflow_amd import ops
from distriflow_amd.models.layers import Conv2D
from distriflow_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
dev = "cuda"

# (B, H, W, C, N, kernel, strides, padding); C % 8 == 0 takes the vectorised gathers, the rest the LUT ones
GEOMS = [
    (4, 9, 8, 8, 16, (3, 5), (2, 1), "same"),
    (4, 16, 16, 16, 32, (3, 3), (2, 2), "same"),  # odd total: the extra row / column at the bottom / right
    (3, 7, 10, 3, 8, (2, 4), (1, 2), "same"),
    (2, 9, 11, 8, 24, (1, 3), (3, 2), "valid"),
    (2, 12, 6, 5, 40, (5, 1), (1, 1), "same"),
]


def _close(got, exp, tol=3e-2):
    err = (got.float().cpu() - exp.float().cpu()).abs().max().item()
    scale = exp.float().abs().max().item() + 1e-6
    assert err <= tol * scale, (err, scale)


@pytest.mark.parametrize("B,H,W,C,N,k,s,p", GEOMS)
def test_irregular_conv_kernels_match_reference(B, H, W, C, N, k, s, p):
    conv = Conv2D(N, k, s, p, name="c")
    conv.build((H, W, C))
    assert not conv.regular
    KH, KW, st, pd = conv.geom
    OH, OW, _ = conv.out_shape
    g = torch.Generator().manual_seed(B * 7 + H)
    K = KH * KW * C
    x = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.2).to(torch.bfloat16)
    b = torch.randn(N, generator=g)
    Npad, Kpad = -(-N // 16) * 16, -(-K // 32) * 32
    wp = torch.zeros(Npad, Kpad, dtype=torch.bfloat16)
    wp[:N, :K] = w
    out = torch.empty(B, OH, OW, N, dtype=torch.bfloat16, device=dev)
    ops.conv_fwd(x.to(dev), wp.to(dev), b.to(dev), out, KH, KW, st, pd, relu=True)
    _close(out, ref.conv_fwd(x.float(), w.float(), b, KH, KW, st, pd, True, out_hw=(OH, OW)))

    dy = torch.randn(B, OH, OW, N, generator=g).to(torch.bfloat16)
    # dgrad weight copy as the store builds it: [Cpad16][K2pad32] with (ci, t, n) <- w[n, t, ci]
    wt = w.float().reshape(N, KH * KW, C).permute(2, 1, 0).reshape(C, KH * KW * N)
    Cpad, K2pad = -(-C // 16) * 16, -(-(KH * KW * N) // 32) * 32
    wtp = torch.zeros(Cpad, K2pad, dtype=torch.bfloat16)
    wtp[:C, :KH * KW * N] = wt.to(torch.bfloat16)
    dx = torch.empty(B, H, W, C, dtype=torch.bfloat16, device=dev)
    ops.conv_dgrad(dy.to(dev), wp.to(dev), wtp.to(dev), dx, KH, KW, st, pd)
    _close(dx, ref.conv_dgrad(dy.float(), w.float(), (B, H, W, C), KH, KW, st, pd))

    gw = torch.empty(N, K, device=dev)
    gb = torch.empty(N, device=dev)
    ws = torch.empty(1 << 22, device=dev)
    ops.conv_wgrad(dy.to(dev), x.to(dev), gw, gb, ws, KH, KW, st, pd)
    torch.cuda.synchronize()
    ew, eb = ref.conv_wgrad(dy.float(), x.float(), KH, KW, st, pd)
    _close(gw, ew)
    _close(gb, eb)


def test_irregular_keras_model_gpu_matches_cpu_engine():
    from distriflow_amd.models.keras import layers_from_keras
    from distriflow_amd.models.net import Net

    topo = {"class_name": "Sequential", "config": {"name": "g", "layers": [
        {"class_name": "Conv2D", "config": {"name": "c1", "filters": 16, "kernel_size": [3, 5], "strides": [2, 1],
                                            "activation": "relu", "padding": "same",
                                            "batch_input_shape": [None, 15, 12, 1]}},
        {"class_name": "Conv2D", "config": {"name": "c2", "filters": 16, "kernel_size": [4, 4], "strides": [2, 2],
                                            "activation": "relu", "padding": "same"}},
        {"class_name": "MaxPooling2D", "config": {"name": "p", "pool_size": [2, 2]}},
        {"class_name": "Flatten", "config": {"name": "f"}},
        {"class_name": "Dense", "config": {"name": "d", "units": 10, "activation": "softmax"}}]}}
    g = torch.Generator().manual_seed(6)
    x = torch.rand(64, 15, 12, 1, generator=g)
    y = torch.randint(0, 10, (64,), generator=g)
    nets = {}
    for d in ("cpu", "cuda"):
        layers, shape = layers_from_keras(topo)
        nets[d] = Net(layers, shape, device=d, seed=9)
    nets["cuda"].store.master.copy_(nets["cpu"].store.master.to(dev))
    nets["cuda"].store.refresh_compute()
    xb = x.to(torch.bfloat16).float()
    st_c = nets["cpu"].compute_gradients(xb, y)
    st_g = nets["cuda"].compute_gradients(xb.to(dev), y.to(dev))
    torch.cuda.synchronize()
    assert abs(float(st_g[0]) - float(st_c[0])) <= 0.02 * abs(float(st_c[0]))
    for s in nets["cpu"].store.specs:
        a = nets["cpu"].store.gradient(s.name).flatten()
        b = nets["cuda"].store.gradient(s.name).flatten().cpu()
        cos = float(F.cosine_similarity(a, b, dim=0))
        assert cos > 0.99, (s.name, cos)
