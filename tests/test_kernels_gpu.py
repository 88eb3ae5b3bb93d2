"""Numerics of every gfx950 HIP kernel against a plain-PyTorch fp32 reference of the same op.

Inputs are rounded to bf16 first (the kernels consume bf16), the reference computes in fp32 on the
same rounded values; tolerances cover the bf16 rounding of outputs only.
"""
import pytest
import torch

from distriflow_amd import ops
from distriflow_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

dev = "cuda"


def _r(a, b):
    return (a + b - 1) // b * b


def _pad_w(w2d):
    """fp32 [N][K] -> zero padded bf16 [Npad16][Kpad32] (the engine's compute layout)."""
    N, K = w2d.shape
    out = torch.zeros(_r(N, 16), _r(K, 32), dtype=torch.bfloat16, device=dev)
    out[:N, :K] = w2d.to(torch.bfloat16)
    return out


def _rowpad_w(w2d, KH, KW, C, H, W, pad):
    """fp32 [N][KH*KW*C] -> fused conv+pool forward layout bf16 [Npad16][Kpad2]: column
    ky*RLp + kx*Cp + c with the kernel's channel stride Cp; pair layout (N <= 8) additionally holds
    in rows 8+n the kernel of channel n shifted right by one column (RLp = round8((KW+1)*Cp))."""
    from distriflow_amd import ops as O
    N = w2d.shape[0]
    Cp, kp, pair = O.convpool_fwd_layout(H, W, C, KH, KW, pad, N)
    RLp = _r((KW + (1 if pair else 0)) * Cp, 8)
    out = torch.zeros(_r(N, 16), kp, dtype=torch.bfloat16, device=dev)
    w4 = w2d.view(N, KH, KW, C).to(torch.bfloat16)
    for ky in range(KH):
        for kx in range(KW):
            out[:N, ky * RLp + kx * Cp: ky * RLp + kx * Cp + C] = w4[:, ky, kx]
            if pair:
                out[8:8 + N, ky * RLp + (kx + 1) * Cp: ky * RLp + (kx + 1) * Cp + C] = w4[:, ky, kx]
    return out


def _pad_wt(w2d, N, T, Ci):
    """fp32 [N][T*Ci] -> dgrad layout bf16 [Ci_pad16][pad32(T*N)] with (ci, t, n) <- w[n, t, ci]."""
    w3 = w2d.view(N, T, Ci).permute(2, 1, 0).reshape(Ci, T * N)
    out = torch.zeros(_r(Ci, 16), _r(T * N, 32), dtype=torch.bfloat16, device=dev)
    out[:Ci, :T * N] = w3.to(torch.bfloat16)
    return out


def _cp_wt(w2d, KH, KW, C, H, W, pad):
    """fp32 [N][KH*KW*C] -> fused conv+pool dgrad layout: the plain [Cpad16][K2pad] layout, or the pair
    layout [16][round32(KH*(KW+1)*N)] (row c: tap (a, b) = W[n][KH-1-a][KW-1-b][c]; row 8+c: the
    same shifted by one column, W[n][KH-1-a][KW-b][c])."""
    from distriflow_amd import ops as O
    N = w2d.shape[0]
    pair, k2p = O.convpool_dgrad_layout(H, W, C, KH, KW, pad, N)
    if not pair:
        return _pad_wt(w2d, N, KH * KW, C)
    out = torch.zeros(16, k2p, dtype=torch.bfloat16, device=dev)
    w4 = w2d.view(N, KH, KW, C).to(torch.bfloat16)
    for a in range(KH):
        for b in range(KW + 1):
            col = (a * (KW + 1) + b) * N
            if b < KW:
                out[:C, col:col + N] = w4[:, KH - 1 - a, KW - 1 - b, :].t()
            if b >= 1:
                out[8:8 + C, col:col + N] = w4[:, KH - 1 - a, KW - b, :].t()
    return out


def _close(a, b, rtol=2e-2, atol=2e-2):
    a = a.float()
    b = b.float()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= atol + rtol * scale, f"max err {err:.4g} vs scale {scale:.4g}"


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)


DENSE = [(64, 10, 784), (4096, 120, 400), (333, 84, 120), (1000, 10, 84), (7, 3, 5), (300, 200, 64), (50, 512, 1024)]


@pytest.mark.parametrize("M,N,K", DENSE)
@pytest.mark.parametrize("relu", [False, True])
def test_dense_fwd(M, N, K, relu):
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev) / K ** 0.5
    b = torch.randn(N, device=dev)
    out = torch.empty(M, N, device=dev, dtype=torch.float32)
    ops.dense_fwd(x, _pad_w(w), b, out, relu)
    exp = ref.dense_fwd(x.float(), w.to(torch.bfloat16).float(), b, relu)
    _close(out, exp, 1e-3, 1e-3)
    out16 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.dense_fwd(x, _pad_w(w), b, out16, relu)
    _close(out16, exp)


@pytest.mark.parametrize("M,N,K", DENSE)
def test_dense_dgrad_masked(M, N, K):
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev) / N ** 0.5
    mask = torch.randn(M, K, device=dev).to(torch.bfloat16)
    out = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    ops.dense_dgrad(dy, None, _pad_wt(w, N, 1, K), out, mask=mask)
    exp = ref.dense_dgrad(dy.float(), w.to(torch.bfloat16).float(), K, mask)
    _close(out, exp)


@pytest.mark.parametrize("M,N,K", DENSE)
def test_dense_wgrad(M, N, K):
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    gw = torch.empty(N, K, device=dev)
    gb = torch.empty(N, device=dev)
    ws = torch.empty(1 << 22, device=dev)
    ops.dense_wgrad(dy, x, gw, gb, ws)
    ew, eb = ref.dense_wgrad(dy.float(), x.float())
    _close(gw, ew, 1e-3, 1e-3)
    _close(gb, eb, 1e-3, 1e-3)


CONVS = [  # B, H, W, C, N, k, stride, pad
    (4, 28, 28, 1, 6, 5, 1, 2),
    (8, 14, 14, 6, 16, 5, 1, 0),
    (4, 28, 28, 1, 32, 3, 1, 0),
    (5, 28, 28, 1, 32, 3, 1, 1),
    (3, 30, 17, 1, 32, 3, 1, 0),
    (4, 26, 26, 32, 32, 3, 1, 0),
    (2, 32, 32, 3, 64, 3, 1, 1),
    (2, 16, 16, 64, 128, 3, 2, 1),
    (2, 8, 8, 64, 128, 1, 2, 0),
    (3, 9, 7, 16, 24, 3, 2, 1),
    # 64-channel multiples at stride 1: the igemm64 FAST gather (buffer loads, per-row tap masks) in
    # both the forward and the data gradient
    (2, 8, 8, 128, 64, 3, 1, 1),
    (3, 10, 6, 64, 64, 3, 1, 1),
    (2, 5, 7, 64, 128, 1, 1, 0),
    # stride-2 data gradients over parity classes (igemm64 PAR): odd sizes, zero-tap classes of a 1x1
    (3, 9, 7, 64, 64, 3, 2, 1),
    (2, 7, 9, 128, 64, 1, 2, 0),
]


@pytest.mark.parametrize("B,H,W,C,N,k,s,p", CONVS)
@pytest.mark.parametrize("relu", [False, True])
def test_conv_fwd(B, H, W, C, N, k, s, p, relu):
    x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    w = torch.randn(N, k * k * C, device=dev) / (k * k * C) ** 0.5
    b = torch.randn(N, device=dev)
    OH, OW = ops.conv_out_hw(H, W, k, k, s, p)
    out = torch.empty(B, OH, OW, N, device=dev, dtype=torch.bfloat16)
    ops.conv_fwd(x, _pad_w(w), b, out, k, k, s, p, relu)
    exp = ref.conv_fwd(x.float(), w.to(torch.bfloat16).float(), b, k, k, s, p, relu)
    _close(out, exp)


@pytest.mark.parametrize("B,H,W,C,N,k,s,p", CONVS)
@pytest.mark.parametrize("masked", [False, True])
def test_conv_dgrad(B, H, W, C, N, k, s, p, masked):
    OH, OW = ops.conv_out_hw(H, W, k, k, s, p)
    dy = torch.randn(B, OH, OW, N, device=dev).to(torch.bfloat16)
    w = torch.randn(N, k * k * C, device=dev) / (k * k * N) ** 0.5
    mask = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16) if masked else None
    out = torch.empty(B, H, W, C, device=dev, dtype=torch.bfloat16)
    ops.conv_dgrad(dy, None, _pad_wt(w, N, k * k, C), out, k, k, s, p, mask=mask)
    exp = ref.conv_dgrad(dy.float(), w.to(torch.bfloat16).float(), (B, H, W, C), k, k, s, p, mask)
    _close(out, exp)


@pytest.mark.parametrize("B,H,W,C,N,k,s,p", CONVS)
def test_conv_wgrad(B, H, W, C, N, k, s, p):
    OH, OW = ops.conv_out_hw(H, W, k, k, s, p)
    dy = torch.randn(B, OH, OW, N, device=dev).to(torch.bfloat16)
    x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    gw = torch.empty(N, k * k * C, device=dev)
    gb = torch.empty(N, device=dev)
    ws = torch.empty(1 << 22, device=dev)
    ops.conv_wgrad(dy, x, gw, gb, ws, k, k, s, p)
    ew, eb = ref.conv_wgrad(dy.float(), x.float(), k, k, s, p)
    _close(gw, ew, 1e-3, 1e-3)
    _close(gb, eb, 1e-3, 1e-3)


WGRAD_TR = [  # B, H, W, C, N, k, stride, pad: ResNet-18 CIFAR shapes on the transposed-read kernel
    (8, 32, 32, 64, 64, 3, 1, 1),
    (8, 32, 32, 64, 128, 3, 2, 1),
    (8, 16, 16, 128, 128, 3, 1, 1),
    (8, 16, 16, 64, 128, 1, 2, 0),
    (16, 4, 4, 512, 512, 3, 1, 1),
    (3, 9, 7, 16, 24, 3, 2, 1),       # odd sizes: m / n / k tails
]


@pytest.mark.parametrize("B,H,W,C,N,k,s,p", WGRAD_TR)
def test_conv_wgrad_transposed_reads(B, H, W, C, N, k, s, p):
    OH, OW = ops.conv_out_hw(H, W, k, k, s, p)
    dy = torch.randn(B, OH, OW, N, device=dev).to(torch.bfloat16)
    x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    gw = torch.full((N, k * k * C), float("nan"), device=dev)
    ws = torch.empty(1 << 24, device=dev)
    ops.conv_wgrad(dy, x, gw, None, ws, k, k, s, p, scale=0.5)
    ew, _ = ref.conv_wgrad(dy.float(), x.float(), k, k, s, p, with_bias=False)
    _close(gw, 0.5 * ew, 1e-3, 1e-3)


WGRAD_HALO = [  # B, H, W, C, N, ws floats: 3x3 stride-1 shapes on the halo-tiled kernel (csrc/wgrad_halo.hip)
    (8, 32, 32, 64, 64, 1 << 24),     # ResNet layer 1: 2 rows x 32 per tile
    (4, 16, 16, 128, 128, 1 << 24),   # layer 2: 4 rows x 16
    (2, 8, 8, 256, 256, 1 << 24),     # layer 3: one whole image per tile
    (16, 4, 4, 512, 512, 1 << 24),    # layer 4: four images per tile
    (8, 8, 8, 64, 192, 1 << 24),      # three co blocks
    (4, 32, 32, 128, 64, 1 << 24),    # C != N
    (4, 16, 16, 64, 64, 1),           # no slab room: one split writes the gradient directly
]


@pytest.mark.parametrize("B,H,W,C,N,wsf", WGRAD_HALO)
def test_conv_wgrad_halo(B, H, W, C, N, wsf):
    dy = torch.randn(B, H, W, N, device=dev).to(torch.bfloat16)
    x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    gw = torch.full((N, 9 * C), float("nan"), device=dev)
    ws = torch.empty(wsf, device=dev)
    ops.conv_wgrad(dy, x, gw, None, ws, 3, 3, 1, 1, scale=0.5)
    ew, _ = ref.conv_wgrad(dy.float(), x.float(), 3, 3, 1, 1, with_bias=False)
    _close(gw, 0.5 * ew, 1e-3, 1e-3)


@pytest.mark.parametrize("B,H,W,C,N,k,s,p", [(64, 26, 26, 32, 32, 3, 1, 0), (8, 16, 16, 64, 128, 3, 2, 1),
                                              (3, 9, 7, 16, 24, 3, 2, 1)])
def test_conv_wgrad_transposed_reads_with_bias(B, H, W, C, N, k, s, p):
    """Conv bias gradient on the transposed-read kernel: an extra k chunk of ones (column K), split-m
    slabs included (the Keras CNN conv2 shape)."""
    OH, OW = ops.conv_out_hw(H, W, k, k, s, p)
    dy = torch.randn(B, OH, OW, N, device=dev).to(torch.bfloat16)
    x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    gw = torch.full((N, k * k * C), float("nan"), device=dev)
    gb = torch.full((N,), float("nan"), device=dev)
    ws = torch.empty(1 << 24, device=dev)
    ops.conv_wgrad(dy, x, gw, gb, ws, k, k, s, p, scale=0.5)
    ew, eb = ref.conv_wgrad(dy.float(), x.float(), k, k, s, p)
    _close(gw, 0.5 * ew, 1e-3, 1e-3)
    _close(gb, 0.5 * eb, 1e-3, 1e-3)


def test_conv_wgrad_large_m_split():
    """Tall-skinny reduction (K = B*OH*OW = 1.3M) exercising many split-m slabs + the reduce kernel."""
    B, H, W, C, N, k = 512, 28, 28, 1, 6, 5
    dy = torch.randn(B, H, W, N, device=dev).to(torch.bfloat16)
    x = torch.rand(B, H, W, C, device=dev).to(torch.bfloat16)
    gw = torch.empty(N, k * k * C, device=dev)
    gb = torch.empty(N, device=dev)
    ws = torch.empty(1 << 22, device=dev)
    ops.conv_wgrad(dy, x, gw, gb, ws, k, k, 1, 2)
    ew, eb = ref.conv_wgrad(dy.float(), x.float(), k, k, 1, 2)
    _close(gw, ew, 1e-3, 1e-2)
    _close(gb, eb, 1e-3, 1e-2)


POOLS = [(4, 28, 28, 6, 2), (4, 24, 24, 32, 2), (2, 10, 10, 16, 2), (2, 5, 5, 3, 2), (2, 9, 9, 8, 3)]


@pytest.mark.parametrize("B,H,W,C,P", POOLS)
def test_maxpool(B, H, W, C, P):
    # distinct values so the arg-max is unique (tie-breaking is implementation defined)
    x = (torch.randperm(B * H * W * C, device=dev).float() / (B * H * W * C) - 0.3).view(B, H, W, C)
    x = x.to(torch.bfloat16)
    # bf16 rounding can create ties; re-draw until unique within windows is overkill: use few values
    y = torch.empty(B, H // P, W // P, C, device=dev, dtype=torch.bfloat16)
    ops.maxpool_fwd(x, y, P)
    _close(y, ref.maxpool_fwd(x.float(), P), 0, 0)
    dy = torch.randn(B, H // P, W // P, C, device=dev).to(torch.bfloat16)
    for relu in (False, True):
        dx = torch.empty(B, H, W, C, device=dev, dtype=torch.bfloat16)
        ops.maxpool_bwd(x, dy, dx, P, relu)
        exp = ref.maxpool_bwd(x.float(), dy.float(), P, relu)
        # compare sums per window (robust to ties created by bf16 rounding)
        _close(dx.float().sum(), exp.sum(), 1e-2, 1e-2)
        assert ((dx.float() != 0).sum() <= (exp != 0).sum() + 8)


@pytest.mark.parametrize("B,C", [(4096, 10), (100, 5), (64, 100), (3, 1000)])
def test_softmax_ce(B, C):
    z = torch.randn(B, C, device=dev) * 3
    y = torch.randint(0, C, (B,), device=dev, dtype=torch.int32)
    dl = torch.empty(B, C, device=dev, dtype=torch.bfloat16)
    st = torch.zeros(2, device=dev)
    ops.softmax_ce(z, y, dl, st, 1.0 / B)
    el, ec, ed = ref.softmax_ce(z, y, 1.0 / B)
    _close(dl, ed, 1e-2, 1e-4)
    assert abs(st[0].item() - el.item()) <= 1e-3 * abs(el.item()) + 1e-3
    assert st[1].item() == ec.item()


def test_dropout_matches_cpu_hash():
    x = torch.randn(3, 1001, device=dev).to(torch.bfloat16)
    y = torch.empty_like(x)
    step = torch.tensor(5, dtype=torch.int64, device=dev)
    ops.dropout(x, y, 0.25, 12345, step=step)
    seed = 12345 ^ (5 * 0x9E3779B1)
    exp = ref.dropout(x.cpu().float(), 0.25, seed)
    _close(y.cpu(), exp, 1e-2, 1e-2)
    keep = (y != 0).float().mean().item()
    assert 0.7 < keep < 0.8


def test_gather_batch_u8():
    data = torch.randint(0, 256, (1000, 28, 28, 1), dtype=torch.uint8, device=dev)
    labels = torch.randint(0, 10, (1000,), dtype=torch.int32, device=dev)
    idx = torch.randperm(1000, device=dev)[:257]
    out = torch.empty(257, 28, 28, 1, dtype=torch.bfloat16, device=dev)
    ol = torch.empty(257, dtype=torch.int32, device=dev)
    ops.gather_batch(data, labels, idx, out, ol, 1.0 / 255)
    _close(out, data[idx].float() / 255, 1e-2, 1e-3)
    assert torch.equal(ol, labels[idx])


@pytest.mark.parametrize("M,C,relu", [(4096, 64, True), (1000, 128, False), (512, 6, True), (65536, 512, False),
                                      (262144, 64, True), (300, 1024, False)])
def test_batchnorm(M, C, relu):
    x = (torch.randn(M, C, device=dev) * 2 + 0.5).to(torch.bfloat16)
    g = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev)
    y = torch.empty_like(x)
    mean = torch.empty(C, device=dev)
    inv = torch.empty(C, device=dev)
    rm = torch.zeros(C, device=dev)
    rv = torch.ones(C, device=dev)
    ws = torch.empty(ops.bn_workspace_floats(C), device=dev)
    cnt = torch.zeros(2, ops.BN_COUNTERS, dtype=torch.int32, device=dev)
    coef = torch.empty(3 * C, device=dev)
    for _ in range(2):  # the last workgroups re-arm the ticket counters: a second launch must agree
        ops.bn_stats_fwd(x, mean, inv, rm, rv, ws, cnt[0], 0.1, 1e-5)
    ops.bn_apply(x, y, g, b, mean, inv, relu=relu)
    ey, emu, evar, einv = ref.batchnorm_train(x.float(), g, b, 1e-5)
    if relu:
        ey = torch.relu(ey)
    _close(y, ey)
    _close(mean, emu, 1e-4, 1e-4)
    _close(inv, einv, 1e-3, 1e-3)
    unb = evar * M / (M - 1)
    _close(rm, 0.19 * emu, 1e-4, 1e-4)          # two momentum-0.1 updates from 0
    _close(rv, 0.81 + 0.19 * unb, 1e-3, 1e-3)   # ... and from 1
    assert int(cnt[0].abs().sum()) == 0
    dy = torch.randn(M, C, device=dev).to(torch.bfloat16)
    dx = torch.empty_like(x)
    dg = torch.empty(C, device=dev)
    db = torch.empty(C, device=dev)
    ops.bn_bwd(x, y if relu else None, dy, dx, g, mean, inv, dg, db, ws, coef, cnt[1])
    assert int(cnt[1][:64].abs().sum()) == 0  # word 64: the fused launch's generation (only increments)
    gin = dy.float() * (y.float() > 0) if relu else dy.float()
    edx, esg, esb = ref.batchnorm_bwd(x.float(), gin, g, emu, einv)
    _close(dx, edx, 3e-2, 3e-2)
    _close(dg, esg, 1e-2, 1e-2)
    _close(db, esb, 1e-3, 1e-3)
    # eval mode normalizes with the running statistics
    ops.bn_apply(x, y, g, b, rm, rv, relu=relu, eval_mode=True)
    ee = (x.float() - rm) * torch.rsqrt(rv + 1e-5) * g + b
    _close(y, torch.relu(ee) if relu else ee)


@pytest.mark.parametrize("M,C", [(32768, 64), (8192, 128), (4096, 512), (40, 64)])
@pytest.mark.parametrize("res", [0, 1, 2])
def test_bn_fused_forward_matches_two_launches(M, C, res):
    """Statistics + apply in one launch (csrc/bn.hip bn_fused_kernel, in-launch hand-off) == the
    statistics launch + the apply launch: mean / invstd / running statistics to fp32 summation order (the
    fused launch has its own, larger grid), output to one bf16 ulp; three launches in a row (the
    generation word keeps counting, tickets re-arm)."""
    torch.manual_seed(C + res)
    x = torch.randn(M, C, device=dev).to(torch.bfloat16)
    r = torch.randn(M, C, device=dev).to(torch.bfloat16) if res else None
    g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    rbn = (torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev), torch.randn(C, device=dev),
           torch.rand(C, device=dev) + 0.5) if res == 2 else None
    ws = torch.empty(ops.bn_workspace_floats(C), device=dev)
    outs = []
    for fused in (False, True):
        cnt = torch.zeros(2, ops.BN_COUNTERS, dtype=torch.int32, device=dev)
        mean, inv = torch.empty(C, device=dev), torch.empty(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        y = torch.empty_like(x)
        for _ in range(3):
            if fused:
                ops.bn_fwd_fused(x, y, g, b, mean, inv, rm, rv, ws, cnt[0], relu=True, residual=r, residual_bn=rbn)
            else:
                ops.bn_stats_fwd(x, mean, inv, rm, rv, ws, cnt[0], 0.1, 1e-5)
                ops.bn_apply(x, y, g, b, mean, inv, relu=True, residual=r, residual_bn=rbn)
        torch.cuda.synchronize()
        assert int(cnt[0][:64].abs().sum()) == 0
        outs.append((y.float(), mean.clone(), inv.clone(), rm.clone(), rv.clone()))
    (y0, m0, i0, rm0, rv0), (y1, m1, i1, rm1, rv1) = outs
    for u, v in ((m0, m1), (i0, i1), (rm0, rm1), (rv0, rv1)):
        torch.testing.assert_close(v, u, rtol=1e-5, atol=1e-6)
    assert ((y1 - y0).abs() <= y0.abs() * 2 ** -7 + 1e-5).all()


@pytest.mark.parametrize("M,C", [(32768, 64), (4096, 512)])
def test_bn_fused_backward_matches_two_launches(M, C, monkeypatch):
    """Backward statistics + dx in one launch == the statistics launch + the dx launch."""
    torch.manual_seed(C)
    x = torch.randn(M, C, device=dev).to(torch.bfloat16)
    mask = torch.randn(M, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(M, C, device=dev).to(torch.bfloat16)
    g = torch.rand(C, device=dev) + 0.5
    mean, inv = x.float().mean(0), torch.rsqrt(x.float().var(0, unbiased=False) + 1e-5)
    ws = torch.empty(ops.bn_workspace_floats(C), device=dev)
    outs = []
    for fused in ("0", "1"):
        monkeypatch.setenv("DISTRIFLOW_DIAG", f"bn_fused={fused}")
        cnt = torch.zeros(2, ops.BN_COUNTERS, dtype=torch.int32, device=dev)
        dx, dg, db, coef = torch.empty_like(x), torch.empty(C, device=dev), torch.empty(C, device=dev), torch.empty(3 * C, device=dev)
        for _ in range(2):
            ops.bn_bwd(x, mask, dy, dx, g, mean, inv, dg, db, ws, coef, cnt[1])
        torch.cuda.synchronize()
        outs.append((dx.float(), dg.clone(), db.clone(), coef.clone()))
    for a, b in zip(outs[0][1:], outs[1][1:]):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5)
    assert ((outs[1][0] - outs[0][0]).abs() <= outs[0][0].abs() * 2 ** -6 + 1e-4).all()


@pytest.mark.parametrize("proj", [False, True])
def test_bn_apply_residual_join(proj):
    M, C = 2048, 128
    x = torch.randn(M, C, device=dev).to(torch.bfloat16)
    r = torch.randn(M, C, device=dev).to(torch.bfloat16)
    g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    m, inv = torch.randn(C, device=dev), torch.rand(C, device=dev) + 0.5
    rbn = (torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev), torch.randn(C, device=dev),
           torch.rand(C, device=dev) + 0.5) if proj else None
    y = torch.empty_like(x)
    ops.bn_apply(x, y, g, b, m, inv, relu=True, residual=r, residual_bn=rbn)
    e = (x.float() - m) * inv * g + b
    e = e + (((r.float() - rbn[2]) * rbn[3] * rbn[0] + rbn[1]) if proj else r.float())
    _close(y, torch.relu(e))


@pytest.mark.parametrize("s", [1, 2])
def test_conv_dgrad_residual_epilogue(s):
    """ResNet block join in the dgrad epilogue: dx = (conv^T dy + res * [resmask > 0]) * [mask > 0]
    (stride 2: the parity-class data gradient, whose epilogue remaps rows to pixels)."""
    B, H, W, C, N, k = 4, 16, 16, 64, 64, 3
    OH, OW = ops.conv_out_hw(H, W, k, k, s, 1)
    dy = torch.randn(B, OH, OW, N, device=dev).to(torch.bfloat16)
    w = torch.randn(N, k * k * C, device=dev) / (k * k * N) ** 0.5
    res = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    rmask = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    mask = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    out = torch.empty(B, H, W, C, device=dev, dtype=torch.bfloat16)
    ops.conv_dgrad(dy, None, _pad_wt(w, N, k * k, C), out, k, k, s, 1, mask=mask, residual=res, residual_mask=rmask)
    exp = ref.conv_dgrad(dy.float(), w.to(torch.bfloat16).float(), (B, H, W, C), k, k, s, 1, None)
    exp = (exp + res.float() * (rmask.float() > 0)) * (mask.float() > 0)
    _close(out, exp)


CONV_HALO = [  # B, H, W, C, N: 3x3 stride-1 shapes on the halo-tiled kernel (csrc/conv3_halo.hip)
    (4, 32, 32, 64, 64),      # ResNet layer 1: 4 rows x 32 per 128-pixel tile
    (4, 16, 16, 128, 128),    # layer 2: 8 rows x 16, two input channel blocks
    (4, 8, 8, 256, 256),      # layer 3: two images per tile
    (16, 4, 4, 512, 512),     # layer 4: eight images per tile, 288 halo rows
    (8, 16, 16, 64, 128),     # C != N
    (4, 16, 16, 128, 64),
    (256, 16, 16, 128, 128),  # >= 512 tiles of 128 channels: the 128-wide variant
    (64, 32, 32, 64, 64),     # >= 512 tiles of 64 -> 64: the weights-resident persistent kernel
    (260, 16, 16, 64, 64),    # same, 16x16 images, a partial last workgroup
]


@pytest.mark.parametrize("B,H,W,C,N", CONV_HALO)
@pytest.mark.parametrize("relu", [False, True])
def test_conv_halo_fwd(B, H, W, C, N, relu):
    x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    w = torch.randn(N, 9 * C, device=dev) / (9 * C) ** 0.5
    out = torch.full((B, H, W, N), float("nan"), device=dev, dtype=torch.bfloat16)
    ops.conv_fwd(x, _pad_w(w), None, out, 3, 3, 1, 1, relu)
    _close(out, ref.conv_fwd(x.float(), w.to(torch.bfloat16).float(), None, 3, 3, 1, 1, relu))


@pytest.mark.parametrize("B,H,W,C,N", CONV_HALO)
@pytest.mark.parametrize("join", [False, True])
def test_conv_halo_dgrad(B, H, W, C, N, join):
    """Flipped-tap data gradient; ``join``: the ResNet block join dx = (conv^T dy + res * [resmask > 0]) *
    [mask > 0] in the epilogue."""
    dy = torch.randn(B, H, W, N, device=dev).to(torch.bfloat16)
    w = torch.randn(N, 9 * C, device=dev) / (9 * N) ** 0.5
    res = rmask = mask = None
    if join:
        res, rmask, mask = (torch.randn(B, H, W, C, device=dev).to(torch.bfloat16) for _ in range(3))
    out = torch.full((B, H, W, C), float("nan"), device=dev, dtype=torch.bfloat16)
    ops.conv_dgrad(dy, None, _pad_wt(w, N, 9, C), out, 3, 3, 1, 1, mask=mask, residual=res, residual_mask=rmask)
    exp = ref.conv_dgrad(dy.float(), w.to(torch.bfloat16).float(), (B, H, W, C), 3, 3, 1, 1, None)
    if join:
        exp = (exp + res.float() * (rmask.float() > 0)) * (mask.float() > 0)
    _close(out, exp)


@pytest.mark.parametrize("B,H,W,C,N", [(16, 4, 4, 512, 512), (8, 8, 8, 256, 256), (3, 4, 4, 256, 512)])
def test_conv_splitk_fwd_and_dgrad(B, H, W, C, N):
    """ResNet-18 layer 3/4 shapes: small M, K up to 4608 -> igemm64 split-K (fp32 partials + a fixed-order
    combine that applies the epilogue), forward with bias + ReLU and data gradient with the full join."""
    k = 3
    x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    w = torch.randn(N, k * k * C, device=dev) / (k * k * C) ** 0.5
    b = torch.randn(N, device=dev)
    out = torch.empty(B, H, W, N, device=dev, dtype=torch.bfloat16)
    ops.conv_fwd(x, _pad_w(w), b, out, k, k, 1, 1, True)
    _close(out, ref.conv_fwd(x.float(), w.to(torch.bfloat16).float(), b, k, k, 1, 1, True))
    dy = torch.randn(B, H, W, N, device=dev).to(torch.bfloat16)
    res = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    rmask = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    mask = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    dx = torch.empty(B, H, W, C, device=dev, dtype=torch.bfloat16)
    ops.conv_dgrad(dy, None, _pad_wt(w, N, k * k, C), dx, k, k, 1, 1, mask=mask, residual=res, residual_mask=rmask)
    exp = ref.conv_dgrad(dy.float(), w.to(torch.bfloat16).float(), (B, H, W, C), k, k, 1, 1, None)
    exp = (exp + res.float() * (rmask.float() > 0)) * (mask.float() > 0)
    _close(dx, exp)


CONVPOOL = [  # B, H, W, C, N, k, pad
    (16, 28, 28, 1, 6, 5, 2),    # LeNet conv1 ('same')
    (16, 14, 14, 6, 16, 5, 0),   # LeNet conv2
    (5, 12, 12, 3, 20, 3, 1),    # odd batch, N > 16, partial window tiles
    (3, 10, 10, 16, 8, 3, 0),
    (7, 12, 12, 4, 8, 3, 0),     # dgrad pair mode with N = 8 (odd 16-byte pixel stride), partial tiles
    (6, 10, 10, 8, 16, 5, 2),    # dgrad pair mode, C = 8 fills both column halves
]


@pytest.mark.parametrize("B,H,W,C,N,k,p", CONVPOOL)
def test_convpool_fwd_wgrad_dgrad(B, H, W, C, N, k, p):
    from distriflow_amd import ops as O

    x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, k * k * C, device=dev) / (k * k * C) ** 0.5).to(torch.bfloat16).float()
    b = torch.randn(N, device=dev) * 0.1
    OH, OW = H + 2 * p - k + 1, W + 2 * p - k + 1
    out = torch.empty(B, OH // 2, OW // 2, N, device=dev, dtype=torch.bfloat16)
    code = torch.empty(B, OH // 2, OW // 2, N, device=dev, dtype=torch.uint8)
    O.convpool_fwd(x, _rowpad_w(w, k, k, C, H, W, p), b, out, code, k, k, p)
    ep, ec = ref.convpool_fwd(x.float().cpu(), w.cpu(), b.cpu(), k, k, p)
    _close(out.cpu(), ep)
    agree = (code.cpu() == ec).float().mean().item()
    assert agree > 0.97, agree  # near-ties may resolve differently under bf16 vs fp32 accumulation order
    # backward uses the kernel's own codes so both sides see the same routing
    dp = torch.randn(B, OH // 2, OW // 2, N, device=dev).to(torch.bfloat16)
    gw = torch.empty(N, k * k * C, device=dev)
    gb = torch.empty(N, device=dev)
    ws = torch.empty(1 << 22, device=dev)
    O.convpool_wgrad(x, dp, code, gw, gb, ws, k, k, p)
    ew, eb = ref.convpool_wgrad(x.float().cpu(), dp.float().cpu(), code.cpu(), k, k, p)
    _close(gw.cpu(), ew, 1e-3, 1e-3)
    _close(gb.cpu(), eb, 1e-3, 1e-3)
    if C <= 16:
        dx = torch.empty(B, H, W, C, device=dev, dtype=torch.bfloat16)
        O.convpool_dgrad(dp, code, None, _cp_wt(w, k, k, C, H, W, p), dx, k, k, p)
        edx = ref.convpool_dgrad(dp.float().cpu(), code.cpu(), w.cpu(), (B, H, W, C), k, k, p)
        _close(dx.cpu(), edx)


def test_convpool_fused_gather_u8():
    from distriflow_amd import ops as O

    data = torch.randint(0, 256, (300, 28, 28, 1), dtype=torch.uint8, device=dev)
    idx = torch.randperm(300, device=dev)[:64]
    w = (torch.randn(6, 25, device=dev) / 5).to(torch.bfloat16).float()
    b = torch.zeros(6, device=dev)
    out = torch.empty(64, 14, 14, 6, device=dev, dtype=torch.bfloat16)
    code = torch.empty(64, 14, 14, 6, device=dev, dtype=torch.uint8)
    O.convpool_fwd(O.GatherRef(data, idx, 1 / 255, (28, 28, 1)), _rowpad_w(w, 5, 5, 1, 28, 28, 2), b, out, code, 5, 5, 2)
    xb = (data[idx].float() / 255).to(torch.bfloat16)
    out2 = torch.empty_like(out)
    O.convpool_fwd(xb, _rowpad_w(w, 5, 5, 1, 28, 28, 2), b, out2, None, 5, 5, 2)
    assert torch.equal(out, out2)


@pytest.mark.parametrize("B,dims,with_idx,x_relu", [
    (50, (64, 48, 32, 10), False, False),    # odd batch: partial row block + zero tail columns
    (256, (400, 120, 84, 10), True, True),   # LeNet-5 head, labels through an index vector, relu' on X
    (96, (784, 10), False, False),           # single-layer (softmax regression) head
])
def test_fused_head_matches_autograd(B, dims, with_idx, x_relu):
    from distriflow_amd import ops as O

    torch.manual_seed(0)
    nl = len(dims) - 1
    x = torch.randn(B, dims[0], device=dev)
    if x_relu:
        x = x.clamp_min(0)
    x = x.to(torch.bfloat16)
    ws = [(torch.randn(dims[i + 1], dims[i], device=dev) / dims[i] ** 0.5).to(torch.bfloat16).float()
          for i in range(nl)]
    bs = [torch.randn(dims[i + 1], device=dev) * 0.1 for i in range(nl)]
    nrows = 3 * B
    all_labels = torch.randint(0, dims[-1], (nrows,), device=dev, dtype=torch.int32)
    idx = torch.randperm(nrows, device=dev)[:B] if with_idx else None
    y = all_labels[idx] if with_idx else all_labels[:B]
    ldt = (B + 31) // 32 * 32
    gw = [torch.empty(dims[i + 1], dims[i], device=dev) for i in range(nl)]
    gb = [torch.empty(dims[i + 1], device=dev) for i in range(nl)]
    hT = [torch.zeros(dims[i + 1], ldt, device=dev, dtype=torch.bfloat16) for i in range(nl - 1)] + [None]
    dzT = [torch.zeros(dims[i + 1], ldt, device=dev, dtype=torch.bfloat16) for i in range(nl)]
    xT = torch.zeros(dims[0], ldt, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(B, dims[0], device=dev, dtype=torch.bfloat16)
    logits = torch.empty(B, dims[-1], device=dev)
    loss_part = torch.zeros(2 * ((B + 15) // 16), device=dev)
    stats = torch.zeros(2, device=dev)
    O.head_train([_pad_w(w) for w in ws], [_pad_wt(w, w.shape[0], 1, w.shape[1]) for w in ws], bs, gw, gb, hT, dzT,
                 list(dims[:-1]), list(dims[1:]), x, x_relu, xT, dx, logits,
                 all_labels if with_idx else y, idx, 1.0 / B, loss_part, stats, phases=3)
    # fp32 reference
    xr = x.float().requires_grad_(True)
    wr = [w.clone().requires_grad_(True) for w in ws]
    br = [b.clone().requires_grad_(True) for b in bs]
    h = xr
    for i in range(nl):
        h = h @ wr[i].t() + br[i]
        if i < nl - 1:
            h = torch.relu(h)
    loss = torch.nn.functional.cross_entropy(h, y.long(), reduction="sum")
    (loss / B).backward()
    _close(logits, h.detach(), 3e-2, 3e-2)
    for i in range(nl):
        _close(gw[i], wr[i].grad, 3e-2, 3e-2)
        _close(gb[i], br[i].grad, 3e-2, 3e-2)
    edx = xr.grad * (x.float() > 0) if x_relu else xr.grad
    _close(dx, edx, 3e-2, 3e-2)
    torch.testing.assert_close(stats[0], loss.detach(), rtol=2e-2, atol=2e-2 * B)
    assert abs(stats[1].item() - (h.argmax(1) == y.long()).sum().item()) <= 2
