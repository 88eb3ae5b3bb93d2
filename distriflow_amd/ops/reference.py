"""Plain-PyTorch fp32 reference implementations of every distriflow_amd op.

Two uses: (1) the CPU execution path (gloo multi-process tests, CPU plumbing config of
BASELINE.json configs[0]); (2) the numerics oracle the HIP kernels are tested against.
Layouts match the kernels exactly: activations NHWC, weights [N][KH*KW*Cin] (OHWI).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _nchw(x):
    return x.permute(0, 3, 1, 2)


def _nhwc(x):
    return x.permute(0, 2, 3, 1)


def conv_weight_4d(w2d, N, KH, KW, C):
    """[N][KH*KW*C] (OHWI) -> [N][C][KH][KW] (torch OIHW)."""
    return w2d[:N, : KH * KW * C].reshape(N, KH, KW, C).permute(0, 3, 1, 2)


def _conv_pad(x, KH, KW, stride, pad, OH, OW):
    """NCHW input padded for a padding-free conv of output OH x OW: ``pad`` = (top, left); the bottom /
    right padding (possibly negative = cropped rows that no output reads) follows from the output size."""
    (sh, sw), (pt, pl) = _pair(stride), _pair(pad)
    H, W = x.shape[2], x.shape[3]
    pb = (OH - 1) * sh + KH - H - pt
    pr = (OW - 1) * sw + KW - W - pl
    return F.pad(x, (pl, pr, pt, pb))


def _pair(v):
    return (int(v[0]), int(v[1])) if isinstance(v, (tuple, list)) else (int(v), int(v))


def _out_hw(H, W, KH, KW, stride, pad):
    (sh, sw), (ph, pw) = _pair(stride), _pair(pad)
    return (H + 2 * ph - KH) // sh + 1, (W + 2 * pw - KW) // sw + 1


def _conv(xc, w4, bias, KH, KW, stride, pad, OH, OW):
    return F.conv2d(_conv_pad(xc, KH, KW, stride, pad, OH, OW), w4, bias, stride=_pair(stride))


def conv_fwd(x, w2d, bias, KH, KW, stride, pad, relu, out_hw=None):
    """fp32 NHWC conv.  ``stride`` = s or (sh, sw); ``pad`` = p or (top, left); ``out_hw`` = (OH, OW)
    (default: symmetric padding)."""
    B, H, W, C = x.shape
    N = bias.shape[0] if bias is not None else w2d.shape[0]
    w4 = conv_weight_4d(w2d.float(), N, KH, KW, C)
    OH, OW = out_hw or _out_hw(H, W, KH, KW, stride, pad)
    y = _conv(_nchw(x.float()), w4, bias.float() if bias is not None else None, KH, KW, stride, pad, OH, OW)
    if relu:
        y = torch.relu(y)
    return _nhwc(y)


def conv_dgrad(dy, w2d, in_shape, KH, KW, stride, pad, mask=None):
    B, H, W, C = in_shape
    _, OH, OW, N = dy.shape
    w4 = conv_weight_4d(w2d.float(), N, KH, KW, C)
    xz = torch.zeros((B, C, H, W), dtype=torch.float32, device=dy.device, requires_grad=True)
    with torch.enable_grad():
        y = _conv(xz, w4, None, KH, KW, stride, pad, OH, OW)
        dx, = torch.autograd.grad(y, xz, _nchw(dy.float()))
    dx = _nhwc(dx)
    if mask is not None:
        dx = dx * (mask.float() > 0)
    return dx


def conv_wgrad(dy, x, KH, KW, stride, pad, with_bias=True):
    B, H, W, C = x.shape
    _, OH, OW, N = dy.shape
    w4 = torch.zeros((N, C, KH, KW), dtype=torch.float32, device=dy.device, requires_grad=True)
    with torch.enable_grad():
        y = _conv(_nchw(x.float()), w4, None, KH, KW, stride, pad, OH, OW)
        gw, = torch.autograd.grad(y, w4, _nchw(dy.float()))
    gw = gw.permute(0, 2, 3, 1).reshape(N, KH * KW * C)
    gb = dy.float().sum(dim=(0, 1, 2)) if with_bias else None
    return gw, gb


def dense_fwd(x, w2d, bias, relu):
    N = bias.shape[0] if bias is not None else w2d.shape[0]
    K = x.shape[-1]
    y = x.float() @ w2d[:N, :K].float().t()
    if bias is not None:
        y = y + bias.float()
    if relu:
        y = torch.relu(y)
    return y


def dense_dgrad(dy, w2d, K, mask=None):
    N = dy.shape[-1]
    dx = dy.float() @ w2d[:N, :K].float()
    if mask is not None:
        dx = dx * (mask.float() > 0)
    return dx


def dense_wgrad(dy, x, with_bias=True):
    gw = dy.float().t() @ x.float()
    gb = dy.float().sum(0) if with_bias else None
    return gw, gb


def maxpool_fwd(x, P):
    return _nhwc(F.max_pool2d(_nchw(x.float()), P, P))


def maxpool_bwd(x, dy, P, relu_fused):
    xf = _nchw(x.float()).detach().requires_grad_(True)
    y = F.max_pool2d(xf, P, P)
    B, H, W, C = x.shape
    g = _nchw(dy.float().reshape(B, H // P, W // P, C))
    if relu_fused:
        g = g * (y.detach() > 0)
    (dx,) = torch.autograd.grad(y, xf, g)
    return _nhwc(dx)


def softmax_ce(logits, labels, grad_scale):
    z = logits.float()
    lse = torch.logsumexp(z, dim=1)
    loss = lse - z.gather(1, labels.long().view(-1, 1)).squeeze(1)
    p = torch.softmax(z, dim=1)
    onehot = F.one_hot(labels.long(), z.shape[1]).float()
    dlogits = (p - onehot) * grad_scale
    correct = (z.argmax(1) == labels.long()).float().sum()
    return loss.sum(), correct, dlogits


def _hash_u32(seed: int, idx: torch.Tensor) -> torch.Tensor:
    """Bit-exact CPU twin of dfa::hash_u32 (splitmix64 finaliser) on int64 tensors."""
    M64 = (1 << 64) - 1

    def u64(v):
        return torch.tensor(v - (1 << 64) if v >= (1 << 63) else v, dtype=torch.int64)

    def lsr(v, s):  # logical shift right on int64 tensors holding uint64 bits
        return (v >> s) & ((1 << (64 - s)) - 1)

    x = idx.to(torch.int64) * u64(0x9E3779B97F4A7C15 & M64) + u64(seed & M64)
    x = x ^ lsr(x, 30)
    x = x * u64(0xBF58476D1CE4E5B9)
    x = x ^ lsr(x, 27)
    x = x * u64(0x94D049BB133111EB)
    x = x ^ lsr(x, 31)
    return x & 0xFFFFFFFF


def dropout_mask(n: int, p: float, seed: int) -> torch.Tensor:
    thresh = int(p * 4294967296.0)
    h = _hash_u32(seed, torch.arange(n, dtype=torch.int64))
    return (h >= thresh).float()


def dropout(x, p, seed, mask=None):
    keep = dropout_mask(x.numel(), p, seed).view_as(x)
    y = x.float() * keep / (1.0 - p)
    if mask is not None:
        y = y * (mask.float() > 0)
    return y


def batchnorm_train(x2d, gamma, beta, eps):
    mean = x2d.float().mean(0)
    var = x2d.float().var(0, unbiased=False)
    invstd = torch.rsqrt(var + eps)
    y = (x2d.float() - mean) * invstd * gamma + beta
    return y, mean, var, invstd


def batchnorm_bwd(x2d, dy2d, gamma, mean, invstd):
    M = x2d.shape[0]
    xh = (x2d.float() - mean) * invstd
    g = dy2d.float()
    sb = g.sum(0)
    sg = (g * xh).sum(0)
    dx = gamma * invstd * (g - sb / M - xh * sg / M)
    return dx, sg, sb


# ---------------------------------------------------------------- fused conv + relu + maxpool2x2
def convpool_fwd(x, w2d, bias, KH, KW, pad):
    """-> (pooled relu output [B,PH,PW,N], code uint8 = argmax(dy*2+dx) | 4*(max>0))."""
    y = conv_fwd(x, w2d, bias, KH, KW, 1, pad, relu=False)  # [B,OH,OW,N] pre-activation
    B, OH, OW, N = y.shape
    win = y.reshape(B, OH // 2, 2, OW // 2, 2, N).permute(0, 1, 3, 5, 2, 4).reshape(B, OH // 2, OW // 2, N, 4)
    m, am = win.max(dim=-1)  # first maximal index on ties
    code = (am | ((m > 0).to(am.dtype) << 2)).to(torch.uint8)
    return torch.relu(m), code


def convpool_unpool(dp, code, OH, OW):
    """Regenerate the full-resolution conv gradient from the pooled gradient and the codes."""
    B, PH, PW, N = code.shape
    dp = dp.float().reshape(B, PH, PW, N)
    c = code.long()
    sel = torch.nn.functional.one_hot(c & 3, 4).float() * ((c & 4) > 0).float().unsqueeze(-1)  # [B,PH,PW,N,4]
    full = (sel * dp.unsqueeze(-1)).reshape(B, PH, PW, N, 2, 2).permute(0, 1, 4, 2, 5, 3).reshape(B, 2 * PH, 2 * PW, N)
    out = torch.zeros(B, OH, OW, N, dtype=full.dtype)
    out[:, : 2 * PH, : 2 * PW] = full
    return out


def convpool_wgrad(x, dp, code, KH, KW, pad):
    B, H, W, C = x.shape
    OH, OW = H + 2 * pad - KH + 1, W + 2 * pad - KW + 1
    dconv = convpool_unpool(dp, code, OH, OW)
    return conv_wgrad(dconv, x, KH, KW, 1, pad, True)


def convpool_dgrad(dp, code, w2d, in_shape, KH, KW, pad):
    B, H, W, C = in_shape
    OH, OW = H + 2 * pad - KH + 1, W + 2 * pad - KW + 1
    dconv = convpool_unpool(dp, code, OH, OW)
    return conv_dgrad(dconv, w2d, in_shape, KH, KW, 1, pad, None)
