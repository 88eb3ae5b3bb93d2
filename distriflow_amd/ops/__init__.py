"""Functional ops of the training engine.

GPU tensors run the hand-written gfx950 kernels of ``distriflow_amd._C`` (no fallback: a missing
extension raises); CPU tensors run the fp32 reference in :mod:`.reference` (CPU plumbing config
and numerics oracle).  All ops write into caller-provided output buffers so that the engine can
preallocate everything once and capture the whole training step into a hipGraph.

Weight arguments:
  * ``w``  — compute weights [Npad][Kpad] (GPU: zero-padded bf16 copy; CPU: fp32 master view [N][K])
  * ``wt`` — dgrad weights [Cin_pad][pad(KH*KW*N)] (GPU only; the CPU path derives it from ``w``)
"""
from __future__ import annotations

import torch

from .. import native
from ..diagnostics import on as _diag_on
from . import reference as ref

MODE_DIRECT, MODE_FWD, MODE_DGRAD = 0, 1, 2


class _DebugSync:
    """``DISTRIFLOW_DEBUG_SYNC=1``: every kernel entry point is followed by a device
    synchronize outside graph capture, so an asynchronous fault or a race between streams is reported
    at the op that caused it (combine with ``AMD_SERIALIZE_KERNEL=3`` set before the first HIP call)."""

    def __init__(self, mod):
        self._mod = mod

    def __getattr__(self, name):
        fn = getattr(self._mod, name)
        if not callable(fn) or isinstance(fn, type):
            return fn

        def wrapped(*args, **kw):
            out = fn(*args, **kw)
            if torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
                try:
                    torch.cuda.synchronize()
                except RuntimeError as e:
                    raise RuntimeError(f"distriflow_amd kernel '{name}' failed: {e}") from e
            return out

        return wrapped


_DEBUG = None


def _C():
    global _DEBUG
    mod = native.require()
    if _DEBUG is None:
        import os

        _DEBUG = os.environ.get("DISTRIFLOW_DEBUG_SYNC", "0") == "1"
    return _DebugSync(mod) if _DEBUG else mod


def graph_upload(g) -> bool:
    """hipGraphUpload of a captured ``torch.cuda.CUDAGraph`` on the current stream: the graph's launch
    resources are staged on the device at capture time, so its first replay (often the first one inside a
    timed region) costs what every later one does.  An optimisation only: a graph the runtime will not
    upload (returns False) is replayed as it is."""
    try:
        _C().graph_upload(int(g.raw_cuda_graph_exec()))
        return True
    except (RuntimeError, AttributeError):
        return False


def _pair(v):
    return (int(v[0]), int(v[1])) if isinstance(v, (tuple, list)) else (int(v), int(v))


def _geom(SH=1, SW=1, SC=1, OH=1, OW=1, KH=1, KW=1, stride=1, pad=0):
    """Native conv geometry.  ``stride`` = s or (row, column); ``pad`` = p or (top, left) -- the bottom /
    right padding is whatever the output size implies (asymmetric Keras 'same')."""
    (sh, sw), (ph, pw) = _pair(stride), _pair(pad)
    g = [int(SH), int(SW), int(SC), int(OH), int(OW), int(KH), int(KW), sh, ph]
    return g if (sh, ph) == (sw, pw) else g + [sw, pw]


def conv_out_hw(H, W, KH, KW, stride, pad):
    """Output size of a conv with symmetric padding ``pad`` = p or (ph, pw) and ``stride`` = s or (sh, sw)."""
    (sh, sw), (ph, pw) = _pair(stride), _pair(pad)
    return (H + 2 * ph - KH) // sh + 1, (W + 2 * pw - KW) // sw + 1


def same_padding(H, W, KH, KW, stride):
    """Keras / TF 'same': output ceil(in / stride); total padding max((out - 1) * s + k - in, 0) split with
    the odd element at the bottom / right.  Returns ((OH, OW), (top, left))."""
    sh, sw = _pair(stride)
    OH, OW = -(-H // sh), -(-W // sw)
    th = max((OH - 1) * sh + KH - H, 0)
    tw = max((OW - 1) * sw + KW - W, 0)
    return (OH, OW), (th // 2, tw // 2)


# ----------------------------------------------------------------------------------- dense
def _drop_kw(drop) -> dict:
    """Keyword arguments of a folded dropout ``(p, seed, step[, step_add])`` for the native launchers."""
    if drop is None:
        return {}
    return {"drop_p": float(drop[0]), "drop_seed": int(drop[1]), "drop_step": drop[2],
            "drop_step_add": int(drop[3]) if len(drop) > 3 else 0}


def dense_fwd(x, w, bias, out, relu=False, drop=None):
    """out[B][N] = act(x[B][K] @ W^T + b); out may be bf16 or fp32 (logits).  ``drop = (p, seed, step)``:
    a Dropout that follows, folded into the epilogue (the mask of :func:`dropout` on ``out``)."""
    B, K = x.shape[0], x.shape[-1]
    N = out.shape[-1]
    if x.is_cuda:
        dkw = _drop_kw(drop)
        _C().igemm_fwd(x, w, bias, None, out, B, N, K, w.shape[1], K, N, _geom(), MODE_DIRECT, relu, 1.0, **dkw)
    else:
        out.copy_(ref.dense_fwd(x, w, bias, relu))
        if drop is not None:
            dropout(out, out, drop[0], drop[1], step=drop[2], step_add=drop[3] if len(drop) > 3 else 0)
    return out


def dense_dgrad(dy, w, wt, out, mask=None, alpha=1.0):
    """out[B][K] = alpha * (dy[B][N] @ W) * relu'(mask)."""
    B, N = dy.shape[0], dy.shape[-1]
    K = out.shape[-1]
    if dy.is_cuda:
        _C().igemm_fwd(dy, wt, None, mask, out, B, K, N, wt.shape[1], N, K, _geom(), MODE_DIRECT, False,
                       float(alpha))
    else:
        out.copy_(ref.dense_dgrad(dy, w, K, mask) * alpha)
    return out


def dense_wgrad(dy, x, gw, gb, workspace=None, scale=1.0):
    """gw[N][K] = dy^T x * scale ; gb[N] = sum_b dy * scale."""
    B, N = dy.shape[0], dy.shape[-1]
    K = x.shape[-1]
    if dy.is_cuda:
        _C().igemm_wgrad(dy, x, gw, gb, workspace, B, N, K, N, K, _geom(), MODE_DIRECT, scale)
    else:
        g, b = ref.dense_wgrad(dy, x, gb is not None)
        gw.copy_(g.reshape(gw.shape) * scale)
        if gb is not None:
            gb.copy_(b * scale)


# ----------------------------------------------------------------------------------- conv2d
def _bn_kwargs(bn):
    """igemm launch arguments of an in-launch BatchNorm statistics spec (kernels.h BnEpi):
    ``bn`` = dict(ws, ticket, mode=0, vecs=[mean, invstd, run_mean, run_var], momentum, eps) or
    dict(ws, ticket, mode=1, x=bn_input, vecs=[mean, invstd, gamma, dgamma, dbeta, coef], gscale)."""
    if bn is None:
        return {}
    return dict(bn_ws=bn["ws"], bn_ticket=bn["ticket"], bn_mode=int(bn.get("mode", 0)), bn_vecs=list(bn["vecs"]),
                bn_x=bn.get("x"), bn_momentum=float(bn.get("momentum", 0.1)), bn_eps=float(bn.get("eps", 1e-5)),
                bn_gscale=float(bn.get("gscale", 1.0)))


def _bacc_kwargs(bacc):
    """igemm launch arguments of epilogue-accumulated BatchNorm sums (kernels.h BnAcc, csrc/bn_acc.h):
    ``bacc`` = dict(acc=[nrep][2][N] float64, mode=0) or dict(acc, mode=1, x, mean, invstd[, acc2, x2, mean2,
    invstd2]) -- mode 1 with the BatchNorm input(s) at the output's positions."""
    if bacc is None:
        return {}
    kw = dict(bacc=bacc["acc"], bacc_mode=int(bacc.get("mode", 0)))
    if kw["bacc_mode"] == 1:
        kw["bacc_in"] = [bacc["x"], bacc["mean"], bacc["invstd"]]
        if bacc.get("acc2") is not None:
            kw.update(bacc2=bacc["acc2"], bacc2_in=[bacc["x2"], bacc["mean2"], bacc["invstd2"]])
    return kw


def conv_bacc_ok(B, H, W, C, OH, OW, N, KH, KW, stride, pad, Kpad, dgrad=False, mode=0, two=False,
                 has_res=False, has_mask=False) -> bool:
    """Can the conv launch (forward, or the data gradient with output [B][H][W][C]) accumulate BatchNorm
    sums of its output in its epilogue (igemm_bacc_ok on the dispatch the launch will take)?"""
    m = native.get(build_if_missing=False)
    if m is None or not hasattr(m, "igemm_bacc_supported"):
        return False
    if dgrad:
        return bool(m.igemm_bacc_supported(B * H * W, C, KH * KW * N, Kpad, _geom(OH, OW, N, H, W, KH, KW, stride, pad),
                                           MODE_DGRAD, int(mode), bool(two), bool(has_res), bool(has_mask)))
    return bool(m.igemm_bacc_supported(B * OH * OW, N, KH * KW * C, Kpad, _geom(H, W, C, OH, OW, KH, KW, stride, pad),
                                       MODE_FWD, int(mode), bool(two), bool(has_res), bool(has_mask)))


def conv_fwd(x, w, bias, out, KH, KW, stride=1, pad=0, relu=False, bn=None, bacc=None):
    """NHWC conv: out[B][OH][OW][N]; w = [Npad][Kpad] with K = KH*KW*C.  ``bn``: the consuming
    BatchNorm's statistics are finalised inside this launch (:func:`_bn_kwargs`, :func:`conv_bn_layout`).
    ``bacc``: the consuming BatchNorm's sums are accumulated by the epilogue (:func:`_bacc_kwargs`)."""
    B, H, W, C = x.shape
    _, OH, OW, N = out.shape
    if x.is_cuda:
        K = KH * KW * C
        _C().igemm_fwd(x, w, bias, None, out, B * OH * OW, N, K, w.shape[1], 0, N,
                       _geom(H, W, C, OH, OW, KH, KW, stride, pad), MODE_FWD, relu, 1.0, **_bn_kwargs(bn),
                       **_bacc_kwargs(bacc))
    else:
        out.copy_(ref.conv_fwd(x, w, bias, KH, KW, stride, pad, relu, out_hw=(OH, OW)))
    return out


def conv_bn_layout(B, H, W, C, OH, OW, N, KH, KW, stride, pad, Kpad, dgrad=False):
    """(row tiles, column ranges) of the conv launch (forward, or the data gradient whose output is
    [B][H][W][C] from an output gradient [B][OH][OW][N]) when it can finalise BatchNorm statistics of
    its output inside the launch; (0, 0) when it cannot.  Sizes: ws (ntm + ceil(ntm / 16)) * 2 * channels
    floats, tickets ntn * (1 + ceil(ntm / 16)) int32 (zero-initialised)."""
    m = native.get(build_if_missing=False)
    if m is None or not hasattr(m, "igemm64_bn_tiles"):
        return 0, 0
    if dgrad:
        r = m.igemm64_bn_tiles(B * H * W, C, KH * KW * N, Kpad, _geom(OH, OW, N, H, W, KH, KW, stride, pad), MODE_DGRAD)
    else:
        r = m.igemm64_bn_tiles(B * OH * OW, N, KH * KW * C, Kpad, _geom(H, W, C, OH, OW, KH, KW, stride, pad), MODE_FWD)
    return int(r[0]), int(r[1])


def bn_finalize_partials(part, ntm, C, M, mean, invstd, run_mean, run_var, momentum, eps):
    """mean / invstd (+ running statistics) from a conv epilogue's partial sums (csrc/bn.hip)."""
    _C().bn_finalize_partials(part, int(ntm), int(C), int(M), mean, invstd, run_mean, run_var, float(momentum),
                              float(eps))


def conv_pool_supported(H, W, C, KH, KW, stride, pad, N) -> bool:
    """Conv + 2x2 max-pool in the igemm64 epilogue (pooled map + argmax codes only)."""
    m = native.get(build_if_missing=False)
    if m is None or not hasattr(m, "igemm64_pool_supported") or stride != 1:
        return False
    OH, OW = conv_out_hw(H, W, KH, KW, stride, pad)
    return bool(m.igemm64_pool_supported(H, W, C, OH, OW, KH * KW * C, N))


def conv_pool_fwd(x, w, bias, out, code, KH, KW, stride=1, pad=0, relu=True, drop=None):
    """conv(+bias, ReLU) then 2x2 max-pool [then a folded dropout]: ``out`` = pooled [B][OH/2][OW/2][N],
    ``code`` = argmax position 0..3 per pooled element (4 = no gradient)."""
    B, H, W, C = x.shape
    _, PH, PW, N = out.shape
    OH, OW = 2 * PH, 2 * PW
    if x.is_cuda:
        K = KH * KW * C
        dkw = _drop_kw(drop)
        _C().igemm_fwd(x, w, bias, None, out, B * OH * OW, N, K, w.shape[1], 0, N,
                       _geom(H, W, C, OH, OW, KH, KW, stride, pad), MODE_FWD, relu, 1.0, pool_code=code, **dkw)
    else:
        y = ref.conv_fwd(x, w, bias, KH, KW, stride, pad, relu).to(out.dtype).float()
        win = y.reshape(B, PH, 2, PW, 2, N).permute(0, 1, 3, 5, 2, 4).reshape(B, PH, PW, N, 4)
        mx, am = win.max(dim=-1)  # first max
        if relu:
            am = torch.where(mx > 0, am, torch.full_like(am, 4))
        out.copy_(mx)
        code.copy_(am.to(torch.uint8))
        if drop is not None:
            dropout(out, out, drop[0], drop[1], step=drop[2], step_add=drop[3] if len(drop) > 3 else 0)
    return out


def unpool2(dyp, code, dy):
    """dy [B][OH][OW][N]: each pooled gradient at the window position its code names."""
    if dy.is_cuda:
        _C().unpool2(dyp.contiguous(), code, dy)
    else:
        B, OH, OW, N = dy.shape
        g = dyp.float().reshape(B, OH // 2, OW // 2, N, 1)
        sel = (code.long().reshape(B, OH // 2, OW // 2, N, 1) == torch.arange(4).reshape(1, 1, 1, 1, 4)).float()
        full = (g * sel).reshape(B, OH // 2, OW // 2, N, 2, 2).permute(0, 1, 4, 2, 5, 3).reshape(B, OH, OW, N)
        dy.copy_(full)
    return dy


def kcnn_supported() -> bool:
    m = native.get(build_if_missing=False)
    return m is not None and hasattr(m, "kcnn_fwd")


def _kc_in(x):
    if isinstance(x, GatherRef):
        return x.data, x.idx, x.scale
    return x, None, 1.0


def kcnn_fwd(x, w1, b1, w2, b2, out, code, drop=None):
    """The reference CNN's conv block forward on GPU (csrc/kcnn_fused.hip): conv1 + ReLU, conv2 + ReLU,
    2x2 max-pool [+ folded dropout] -> pooled ``out`` [B][12][12][32] and argmax ``code``.  ``x``: a
    :class:`GatherRef` (uint8 dataset rows, read in-kernel) or a bf16 batch [B][28][28][1]."""
    src, idx, scale = _kc_in(x)
    dkw = _drop_kw(drop)
    _C().kcnn_fwd(src, idx, float(scale), int(out.shape[0]), w1, b1, int(w1.shape[1]), w2, b2, out, code, **dkw)
    return out


def kcnn_slab_floats(B: int) -> int:
    return int(_C().kcnn_slab_floats(int(B)))


def kcnn_bwd(x, w1, b1, w2t, dyp, code, slabs, g_w1, g_b1, g_w2, g_b2, step_inc=None):
    """Both conv weight gradients of the block from the pooled gradient ``dyp`` (one backward launch +
    one deterministic slab reduction, which also advances ``step_inc``)."""
    src, idx, scale = _kc_in(x)
    _C().kcnn_bwd(src, idx, float(scale), int(dyp.shape[0]), w1, b1, int(w1.shape[1]), w2t, dyp.contiguous(), code,
                  slabs, g_w1, g_b1, g_w2, g_b2, step_inc=step_inc)


def conv_dgrad(dy, w, wt, out, KH, KW, stride=1, pad=0, mask=None, residual=None, residual_mask=None, bn=None,
               bacc=None):
    """dX (NHWC [B][H][W][C]) of a conv whose output gradient is dy [B][OH][OW][N].

    Epilogue (ResNet block join): dX = (conv^T dy + residual * [residual_mask > 0]) * [mask > 0].
    ``bn`` (mode 1): dX is the output gradient of a BatchNorm; its backward statistics are finalised
    inside this launch (:func:`_bn_kwargs`).  ``bacc`` (mode 1): its backward sums are accumulated by
    the epilogue instead (:func:`_bacc_kwargs`)."""
    B, OH, OW, N = dy.shape
    _, H, W, C = out.shape
    if dy.is_cuda:
        K = KH * KW * N
        _C().igemm_fwd(dy, wt, None, mask, out, B * H * W, C, K, wt.shape[1], 0, C,
                       _geom(OH, OW, N, H, W, KH, KW, stride, pad), MODE_DGRAD, False, 1.0, residual, residual_mask,
                       **_bn_kwargs(bn), **_bacc_kwargs(bacc))
    else:
        dx = ref.conv_dgrad(dy, w, out.shape, KH, KW, stride, pad, None)
        if residual is not None:
            r = residual.float().reshape(dx.shape)
            if residual_mask is not None:
                r = r * (residual_mask.float().reshape(dx.shape) > 0)
            dx = dx + r
        if mask is not None:
            dx = dx * (mask.float().reshape(dx.shape) > 0)
        out.copy_(dx)
    return out


def conv_wgrad(dy, x, gw, gb, workspace, KH, KW, stride=1, pad=0, scale=1.0):
    B, H, W, C = x.shape
    _, OH, OW, N = dy.shape
    if dy.is_cuda:
        K = KH * KW * C
        _C().igemm_wgrad(dy, x, gw, gb, workspace, B * OH * OW, N, K, N, 0,
                         _geom(H, W, C, OH, OW, KH, KW, stride, pad), MODE_FWD, scale)
    else:
        g, b = ref.conv_wgrad(dy, x, KH, KW, stride, pad, gb is not None)
        gw.copy_(g.reshape(gw.shape) * scale)
        if gb is not None:
            gb.copy_(b * scale)


# ----------------------------------------------------------------------------------- pooling etc.
def maxpool_fwd(x, out, P, drop=None):
    """``drop = (p, seed, step)``: a Dropout that follows, folded in (same mask as :func:`dropout`)."""
    B, H, W, C = x.shape
    if x.is_cuda:
        dkw = _drop_kw(drop)
        _C().maxpool_fwd(x, out, B, H, W, C, P, **dkw)
    else:
        out.copy_(ref.maxpool_fwd(x, P))
        if drop is not None:
            dropout(out, out, drop[0], drop[1], step=drop[2], step_add=drop[3] if len(drop) > 3 else 0)
    return out


def maxpool_bwd(x, dy, dx, P, relu_fused=False):
    B, H, W, C = x.shape
    if x.is_cuda:
        _C().maxpool_bwd(x, dy, dx, B, H, W, C, P, relu_fused)
    else:
        dx.copy_(ref.maxpool_bwd(x, dy, P, relu_fused))
    return dx


def softmax_ce(logits, labels, dlogits=None, stats=None, grad_scale=1.0):
    """Fused softmax-cross-entropy: dlogits = (softmax - onehot) * grad_scale; stats += [loss_sum, #correct]."""
    B, C = logits.shape
    if logits.is_cuda:
        ldg = dlogits.shape[-1] if dlogits is not None else C
        _C().softmax_ce(logits, labels, dlogits, stats, B, C, C, ldg, grad_scale)
    else:
        loss, corr, dl = ref.softmax_ce(logits, labels, grad_scale)
        if dlogits is not None:
            dlogits.copy_(dl)
        if stats is not None:
            stats[0] += loss
            stats[1] += corr


def dropout(x, out, p, seed, mask=None, step=None, step_add=0):
    """out = x * keep(seed ^ step, i) / (1 - p) [* relu'(mask)]; ``step`` is a device int64 scalar."""
    if x.is_cuda:
        if step_add:
            raise ValueError("step_add is for folded dropouts only")
        _C().dropout(x, out, p, seed, mask, step)
    else:
        s = seed ^ ((int(step.item()) + step_add) * 0x9E3779B1 if step is not None else 0)
        out.copy_(ref.dropout(x, p, s, mask).reshape(out.shape))
    return out


def gather_batch(data, labels, idx, out, out_labels, scale=1.0, step_inc=None):
    """out[b] = data[idx[b]] (uint8 -> bf16 * scale on the fly); out_labels[b] = labels[idx[b]].
    ``step_inc``: a device int64 counter the launch advances by one (the engine's dropout step)."""
    B = idx.shape[0]
    row = out[0].numel()
    if out.is_cuda:
        _C().gather_batch(data, labels, idx, out, out_labels, B, row, scale, step_inc=step_inc)
    else:
        if step_inc is not None:
            step_inc.add_(1)
        out.copy_((data.index_select(0, idx).float() * scale).reshape(out.shape))
        if labels is not None:
            out_labels.copy_(labels.index_select(0, idx))
    return out


def add_act(a, b, out, relu=False):
    if a.is_cuda:
        _C().add_act(a, b, out, relu)
    else:
        r = a.float() + b.float()
        out.copy_(torch.relu(r) if relu else r)
    return out


# ---- Keras merge layers of branching graphs (csrc/merge.hip); codes match kernels.h kMerge*
MERGE_KINDS = {"Add": 0, "Subtract": 1, "Multiply": 2, "Average": 3, "Maximum": 4, "Minimum": 5, "Concatenate": 6}


def _merge_ref(kind: int, xs):
    xs = [x.float() for x in xs]
    if kind == 6:
        return torch.cat(xs, dim=-1)
    out = xs[0].clone()
    for x in xs[1:]:
        if kind in (0, 3):
            out = out + x
        elif kind == 1:
            out = out - x
        elif kind == 2:
            out = out * x
        elif kind == 4:
            out = torch.maximum(out, x)
        else:
            out = torch.minimum(out, x)
    return out / len(xs) if kind == 3 else out


def merge_fwd(inputs, out, kind: str):
    """out = merge(inputs) over the last axis layout [..., C] (one launch on GPU)."""
    k = MERGE_KINDS[kind]
    if out.is_cuda:
        _C().merge_fwd([x.contiguous() for x in inputs], out, k)
    else:
        out.copy_(_merge_ref(k, inputs).to(out.dtype))
    return out


def merge_bwd(inputs, dy, grads, kind: str):
    """grads[i] = d merge / d inputs[i] * dy (Maximum / Minimum: to the first input holding the extreme)."""
    k = MERGE_KINDS[kind]
    if dy.is_cuda:
        _C().merge_bwd([x.contiguous() for x in inputs], dy.contiguous(), list(grads), k)
        return grads
    if k == 6:
        off = 0
        for x, g in zip(inputs, grads):
            w = x.shape[-1]
            g.copy_(dy[..., off:off + w])
            off += w
        return grads
    if k in (4, 5):  # first extreme wins, as the kernel
        xs = [x.float() for x in inputs]
        ext = _merge_ref(k, inputs)
        taken = torch.zeros_like(ext, dtype=torch.bool)
        for x, g in zip(xs, grads):
            hit = (x == ext) & ~taken
            taken |= hit
            g.copy_(torch.where(hit, dy.float(), torch.zeros_like(ext)).to(g.dtype))
        return grads
    xs = [x.float().detach().requires_grad_(True) for x in inputs]
    y = _merge_ref(k, xs)
    gs = torch.autograd.grad(y, xs, dy.float())
    for g, v in zip(grads, gs):
        g.copy_(v.to(g.dtype))
    return grads


# ---- generic Keras layers (csrc/act.hip); codes match kernels.h ActKind
ACT_KINDS = {"linear": 0, None: 0, "relu": 1, "relu6": 2, "sigmoid": 3, "tanh": 4, "elu": 5, "selu": 6,
             "softplus": 7, "softsign": 8, "hard_sigmoid": 9, "hardSigmoid": 9, "swish": 10, "silu": 10,
             "exponential": 11}


def _act_ref(kind: int, x):
    import torch.nn.functional as F

    def clip(v, lo, hi):  # TensorFlow's gradient of a clipped activation: zero AT the corners too
        return torch.where((v > lo) & (v < hi), v, v.clamp(lo, hi).detach())

    f = {0: lambda v: v, 1: F.relu, 2: lambda v: clip(v, 0.0, 6.0), 3: torch.sigmoid, 4: torch.tanh, 5: F.elu,
         6: F.selu, 7: F.softplus, 8: F.softsign, 9: lambda v: clip(0.2 * v + 0.5, 0.0, 1.0), 10: F.silu,
         11: torch.exp}[kind]
    return f(x)


def act_fwd(x, out, activation):
    """out = act(x) for the Keras activations in ACT_KINDS (one streaming launch on GPU)."""
    kind = ACT_KINDS[activation]
    if x.is_cuda:
        _C().act_fwd(x.contiguous(), out, kind)
    else:
        out.copy_(_act_ref(kind, x.float()).to(out.dtype))
    return out


def act_bwd(x, dy, dx, activation, in_relu=False):
    """dx = dy * act'(x) [* relu'(x) when x is itself a fused-ReLU output]."""
    kind = ACT_KINDS[activation]
    if x.is_cuda:
        _C().act_bwd(x.contiguous(), dy.contiguous(), dx, kind, bool(in_relu))
    else:
        xv = x.float().detach().requires_grad_(True)
        y = _act_ref(kind, xv)
        (g,) = torch.autograd.grad(y, xv, dy.float())
        if in_relu:
            g = g * (x.float() > 0)
        dx.copy_(g.to(dx.dtype))
    return dx


def sigmoid_ce(logits, labels, dlogits=None, stats=None, grad_scale=1.0):
    """Sigmoid cross-entropy on logits vs one-hot(labels), summed over classes: dlogits = (sigmoid(z) -
    onehot) * grad_scale; stats += [loss_sum, #correct (argmax)]."""
    B, C = logits.shape
    if logits.is_cuda:
        ldg = dlogits.shape[-1] if dlogits is not None else C
        _C().sigmoid_ce(logits, labels.to(torch.int32), dlogits, stats, B, C, C, ldg, grad_scale)
    else:
        z = logits.float()
        t = torch.nn.functional.one_hot(labels.long().clamp(0, C - 1), C).float()
        loss = (z.clamp_min(0) - z * t + torch.log1p(torch.exp(-z.abs()))).sum()
        if dlogits is not None:
            dlogits.copy_(((torch.sigmoid(z) - t) * grad_scale).to(dlogits.dtype))
        if stats is not None:
            stats[0] += loss
            stats[1] += (z.argmax(1) == labels.long()).float().sum()
    return stats


def pool_geometry(B, H, W, C, pool, strides, padding):
    """[B, H, W, C, OH, OW, ph, pw, sh, sw, pt, pl] of a Keras/TF pooling layer ('valid' | 'same')."""
    ph, pw = pool
    sh, sw = strides
    if padding == "same":
        OH, OW = -(-H // sh), -(-W // sw)
        tot_h = max((OH - 1) * sh + ph - H, 0)
        tot_w = max((OW - 1) * sw + pw - W, 0)
        pt, pl = tot_h // 2, tot_w // 2  # TF: the odd pixel of padding goes bottom / right
    elif padding == "valid":
        OH, OW = (H - ph) // sh + 1, (W - pw) // sw + 1
        pt = pl = 0
    else:
        raise ValueError(f"pooling padding {padding!r}")
    if OH < 1 or OW < 1:
        raise ValueError(f"pool {pool} / {strides} does not fit a {H}x{W} input")
    return [B, H, W, C, OH, OW, ph, pw, sh, sw, pt, pl]


def _pool_ref(x, g, avg):
    B, H, W, C, OH, OW, ph, pw, sh, sw, pt, pl = g
    xf = x.float().permute(0, 3, 1, 2)
    pb, pr = max((OH - 1) * sh + ph - H - pt, 0), max((OW - 1) * sw + pw - W - pl, 0)
    if avg:
        ones = torch.ones(1, 1, H, W, dtype=xf.dtype, device=xf.device)
        num = torch.nn.functional.avg_pool2d(torch.nn.functional.pad(xf, (pl, pr, pt, pb)), (ph, pw), (sh, sw),
                                             divisor_override=1)
        cnt = torch.nn.functional.avg_pool2d(torch.nn.functional.pad(ones, (pl, pr, pt, pb)), (ph, pw), (sh, sw),
                                             divisor_override=1)
        y = num / cnt.clamp_min(1.0)
    else:
        y = torch.nn.functional.max_pool2d(torch.nn.functional.pad(xf, (pl, pr, pt, pb), value=float("-inf")),
                                           (ph, pw), (sh, sw))
    return y[:, :, :OH, :OW].permute(0, 2, 3, 1)


def pool2d_fwd(x, out, geom, avg=False):
    """General 2-D pooling (max / average; any window, stride and 'valid' / 'same' padding), NHWC."""
    if x.is_cuda:
        _C().pool2d_fwd(x.contiguous(), out, [int(v) for v in geom], bool(avg))
    else:
        out.copy_(_pool_ref(x, geom, avg).reshape(out.shape).to(out.dtype))
    return out


def pool2d_bwd(x, dy, dx, geom, avg=False, in_relu=False):
    if x.is_cuda:
        _C().pool2d_bwd(x.contiguous(), dy.contiguous(), dx, [int(v) for v in geom], bool(avg), bool(in_relu))
    else:
        xv = x.float().detach().requires_grad_(True)
        y = _pool_ref(xv, geom, avg)
        (g,) = torch.autograd.grad(y, xv, dy.float().reshape(y.shape))
        if in_relu:
            g = g * (x.float() > 0)
        dx.copy_(g.reshape(dx.shape).to(dx.dtype))
    return dx


def relu_bwd(y, dy, dx):
    if y.is_cuda:
        _C().relu_bwd(y, dy, dx)
    else:
        dx.copy_((dy.float().reshape(y.shape) * (y.float() > 0)).reshape(dx.shape))
    return dx


def gap_fwd(x, out):
    B, H, W, C = x.shape
    if x.is_cuda:
        _C().gap_fwd(x, out, B, H * W, C)
    else:
        out.copy_(x.float().mean(dim=(1, 2)))
    return out


def gap_bwd(dy, dx):
    B, H, W, C = dx.shape
    if dy.is_cuda:
        _C().gap_bwd(dy, dx, B, H * W, C)
    else:
        dx.copy_((dy.float() / (H * W)).view(B, 1, 1, C).expand(B, H, W, C))
    return dx


BN_COUNTERS = 65  # ticket counters of one BN statistics launch: 1 global + 1 per group of 16 (<= 1024) workgroups


def bn_workspace_floats(C: int) -> int:
    """fp32 workspace of a BN statistics launch of any M: <= 1024 partial slabs + <= 64 group slabs of [2][C]."""
    return (1024 + 64) * 2 * C


def bn_stats_fwd(x2d, mean, invstd, run_mean, run_var, ws, counter, momentum=0.1, eps=1e-5):
    """Training batch statistics of x2d [M][C] -> mean, invstd; running statistics updated in place.
    GPU: one launch (csrc/bn.hip; ``counter`` = int32 last-arriver ticket, zero between launches)."""
    M, C = x2d.shape
    if x2d.is_cuda:
        _C().bn_stats_fwd(x2d, mean, invstd, run_mean, run_var, ws, counter, M, C, momentum, eps)
    else:
        mu = x2d.float().mean(0)
        var = x2d.float().var(0, unbiased=False)
        mean.copy_(mu)
        invstd.copy_(torch.rsqrt(var + eps))
        if run_mean is not None:
            unb = var * M / max(M - 1, 1)
            run_mean.mul_(1 - momentum).add_(mu * momentum)
            run_var.mul_(1 - momentum).add_(unb * momentum)


def bn_apply(x2d, y2d, gamma, beta, mean, invstd, relu=False, residual=None, residual_bn=None, eval_mode=False,
             eps=1e-5):
    """y = act(bn(x) [+ r | + bn_r(r)]): ``residual_bn`` = (gamma, beta, mean, invstd) of the residual's BN
    (ResNet projection shortcut).  ``eval_mode``: mean / invstd are the running mean / variance."""
    M, C = x2d.shape
    if x2d.is_cuda:
        rg = rb = rm = ri = None
        if residual_bn is not None:
            rg, rb, rm, ri = residual_bn
        _C().bn_apply(x2d, y2d, gamma, beta, mean, invstd, residual, rg, rb, rm, ri, M, C, relu, eval_mode, eps)
    else:
        def aff(x, g, b, m, v):
            inv = torch.rsqrt(v + eps) if eval_mode else v
            return (x.float() - m) * inv * g + b

        y = aff(x2d, gamma, beta, mean, invstd)
        if residual is not None:
            r = residual.reshape(M, C)
            y = y + (aff(r, *residual_bn) if residual_bn is not None else r.float())
        y2d.copy_(torch.relu(y) if relu else y)
    return y2d


def bn_fused_ok(C: int, device) -> bool:
    """Statistics + streaming pass in one launch (csrc/bn.hip bn_fused_kernel): GPU, C % 8 == 0."""
    from ..diagnostics import on as diag_on

    return torch.device(device).type == "cuda" and C % 8 == 0 and C <= 1024 and diag_on("bn_fused")


def bn_fwd_fused(x2d, y2d, gamma, beta, mean, invstd, run_mean, run_var, ws, counter, relu=False, residual=None,
                 residual_bn=None, momentum=0.1, eps=1e-5):
    """Training forward in one launch: batch statistics (mean, invstd, running statistics) and
    y = act(bn(x) [+ r | + bn_r(r)]).  ``counter``: the layer's 65-word ticket row (word 64: generation)."""
    M, C = x2d.shape
    rg = rb = rm = ri = None
    if residual_bn is not None:
        rg, rb, rm, ri = residual_bn
    _C().bn_fwd_fused(x2d, y2d, gamma, beta, mean, invstd, run_mean, run_var, residual, rg, rb, rm, ri, ws, counter,
                      M, C, relu, momentum, eps)
    return y2d


def bn_apply_acc(x2d, y2d, gamma, beta, acc, zero, mean, invstd, run_mean, run_var, relu=False, residual=None,
                 rbn=None, momentum=0.1, eps=1e-5):
    """Training y = act(bn(x) [+ r | + bn_r(r)]) with the batch statistics finalised from the producing
    conv's accumulated sums ``acc`` (csrc/bn.hip bn_apply_acc): writes mean / invstd / running statistics
    and clears ``zero`` (the other direction's accumulator).  ``rbn``: the residual's BatchNorm as
    [gamma, beta, acc, zero, mean, invstd, run_mean, run_var] (its statistics finalised the same way)."""
    M, C = x2d.shape
    z = zero if zero is not None else None
    rb = list(rbn) if rbn is not None else []
    if rb and rb[3] is None:
        rb[3] = torch.empty(0, dtype=torch.float64, device=x2d.device)
    _C().bn_apply_acc(x2d, y2d, gamma, beta, acc, z, mean, invstd, run_mean, run_var, residual, rb, M, C, relu,
                      momentum, eps)
    return y2d


def bn_dx_acc(x2d, g2d, dx2d, acc, zero, gamma, mean, invstd, dgamma, dbeta, coef, gscale=1.0):
    """dx = k1 g + k2 x + k3 with the coefficients finalised from the producer's backward sums ``acc``
    (csrc/bn.hip bn_dx_acc); also writes dgamma, dbeta (x gscale) and coef, and clears ``zero``."""
    M, C = x2d.shape
    _C().bn_dx_acc(x2d, g2d, dx2d, acc, zero, gamma, mean, invstd, dgamma, dbeta, coef, M, C, gscale)
    return dx2d


def gap_bwd_bn(dy, mask, dx, acc, x, mean, invstd):
    """GAP backward with relu'(mask) and the BatchNorm backward sums of dx (``x`` = that BN's input)."""
    B, H, W, C = dx.shape
    _C().gap_bwd_bn(dy.contiguous(), mask, dx, B, H * W, C, acc, [x, mean, invstd])
    return dx


def bn_dx(x2d, g2d, dx2d, coef):
    """dx = k1 g + k2 x + k3 per channel (coef [3][C] from a finalised backward statistics pass)."""
    M, C = x2d.shape
    if x2d.is_cuda:
        _C().bn_dx(x2d, None, g2d, dx2d, coef, M, C)
    else:
        dx2d.copy_(coef[:C] * g2d.float() + coef[C:2 * C] * x2d.float() + coef[2 * C:3 * C])
    return dx2d


def bn_bwd(x2d, mask2d, dy2d, dx2d, gamma, mean, invstd, dgamma, dbeta, ws, coef, counter, gscale=1.0):
    """Backward of y = bn(x): dx, dgamma, dbeta (scaled by gscale) from dy; g = dy * (mask > 0) when a
    mask (relu' source) is given.  GPU: statistics launch (which also writes the dx coefficients) + dx pass."""
    M, C = x2d.shape
    if x2d.is_cuda and bn_fused_ok(C, x2d.device) and counter.numel() >= BN_COUNTERS:
        _C().bn_bwd_fused(x2d, mask2d, dy2d, dx2d, gamma, mean, invstd, dgamma, dbeta, coef, ws, counter, M, C, gscale)
    elif x2d.is_cuda:
        _C().bn_stats_bwd(x2d, mask2d, dy2d, gamma, mean, invstd, dgamma, dbeta, coef, ws, counter, M, C, gscale)
        _C().bn_dx(x2d, mask2d, dy2d, dx2d, coef, M, C)
    else:
        g = dy2d.float() * (mask2d.float() > 0) if mask2d is not None else dy2d.float()
        dx, sg, sb = ref.batchnorm_bwd(x2d, g, gamma, mean, invstd)
        dx2d.copy_(dx)
        dgamma.copy_(sg * gscale)
        dbeta.copy_(sb * gscale)
    return dx2d


# ----------------------------------------------------------------------------------- fused conv+pool
class GatherRef:
    """A batch that has not been materialised: rows ``idx`` of an HBM-resident uint8 dataset, scaled.
    The first layer reads it directly (fused gather + cast); other consumers call :meth:`materialise`."""

    def __init__(self, data, idx, scale, shape):
        self.data, self.idx, self.scale = data, idx, scale
        self.shape = (idx.shape[0],) + tuple(shape)
        self.device = data.device
        self.is_cuda = data.is_cuda

    def materialise(self, out, step_inc=None):
        return gather_batch(self.data, None, self.idx, out, None, self.scale, step_inc=step_inc)


class LabelRef:
    """Labels of a batch that has not been gathered: ``labels[idx]`` (consumers that can read through
    the index vector — the fused head — never materialise it)."""

    def __init__(self, labels, idx):
        self.labels, self.idx = labels, idx
        self.shape = (idx.shape[0],)

    def materialise(self, out):
        return gather_labels(self.labels, self.idx, out)


def head_supported() -> bool:
    m = native.get(build_if_missing=False)
    return m is not None and hasattr(m, "head_train")


def head_train(w, wt, b, gw, gb, hT, dzT, K, N, x, x_relu, xT, dx, logits, labels, idx, grad_scale, loss_part,
               stats, phases=3, dx_scale=1.0):
    """Fused dense head on GPU (csrc/mlphead.hip): forward + softmax-CE + backward of a Dense chain.
    phases bit 1: forward, loss, backward data chain (dx, logits, H^T/dZ^T); bit 2: weight/bias
    gradients gw/gb (batch-mean scaled via grad_scale) and stats.  Each phase is one launch on the
    current stream, so the two can be placed on different streams."""
    _C().head_train(list(w), list(wt), list(b), list(gw), list(gb), list(hT), list(dzT), list(K), list(N),
                    x.reshape(x.shape[0], -1) if x.is_contiguous() else x.contiguous().reshape(x.shape[0], -1),
                    bool(x_relu), xT, dx, logits, labels, idx, float(grad_scale), loss_part, stats, int(phases),
                    dx_scale=float(dx_scale))


def khead_supported(K: int, C: int) -> bool:
    m = native.get(build_if_missing=False)
    return m is not None and hasattr(m, "khead_train") and bool(m.khead_supported(int(K), int(C)))


def khead_ws_floats(B: int, K: int) -> int:
    return int(_C().khead_ws_floats(int(B), int(K)))


def khead_error(ws: torch.Tensor, B: int) -> int:
    """The dense-head launch's sticky error word (csrc/khead.hip): non-zero after a row tile's flag wait timed
    out (its results invalid).  ``ws``: the launch's workspace (ops.khead_ws_floats floats)."""
    nt = -(-int(B) // 32)
    off = nt * 8 * 32 * 128 + nt * 32 * 128 // 2 + 2 * nt + 2  # (after the tag and the done counter)
    return int(ws[off:off + 1].view(torch.int32).item())


def khead_train(p, pT, dp, w1, w1t, b1, w2, w2t, b2, h1T, dz1T, dz2T, logits, labels, idx, grad_scale, loss_part, ws,
                drop=None, dh_scale=1.0, dp_scale=1.0, dp_mask=False):
    """The reference CNN's dense head on GPU (csrc/khead.hip): dense1 (K -> 128, ReLU, folded ``drop``),
    dense2 (128 -> C) and softmax-CE, forward + loss + both data gradients in ONE launch (split-K over 8
    workgroups per 32 batch rows).  Writes logits, the loss partials, dP (``dp``) and the weight-gradient
    operands P^T / H1^T / dZ1^T / dZ2^T that :func:`head_train` (phases=2) turns into gw / gb / stats."""
    dk = _drop_kw(drop)
    _C().khead_train(p.reshape(p.shape[0], -1), pT, dp, w1, w1t, b1, w2, w2t, b2, dk.get("drop_p", 0.0),
                     dk.get("drop_seed", 0), dk.get("drop_step"), dk.get("drop_step_add", 0), float(dh_scale),
                     float(dp_scale), bool(dp_mask), h1T, dz1T, dz2T, logits, labels, idx, float(grad_scale),
                     loss_part, ws)


def khead_wgrad(pT, h1T, dz1T, dz2T, gw1, gb1, gw2, gb2, B, K, C, loss_part, stats):
    """Weight / bias gradients of the :func:`khead_train` head from its transposed operands, and the
    loss partials -> stats (one launch, csrc/khead.hip)."""
    _C().khead_wgrad(pT, h1T, dz1T, dz2T, gw1, gb1, gw2, gb2, int(B), int(K), int(C), loss_part, stats)


METRIC_KINDS = {"meanSquaredError": 0, "mse": 0, "absoluteDifference": 1, "hingeLoss": 2, "huberLoss": 3,
                "logLoss": 4, "sigmoidCrossEntropy": 5, "softmaxCrossEntropy": 6, "categorical_crossentropy": 7,
                "categoricalCrossentropy": 7}


def classifier_metrics(z, labels, loss: str, softmax, out):
    """[sum over the batch of the compiled loss, number correct] of fp32 model outputs ``z`` [B][C]
    against int labels (one launch on GPU, csrc/metrics.hip).  ``softmax``: the model output is
    softmax(z).  Returns ``out`` (device [2]); CPU uses the torch loss registry."""
    if z.is_cuda:
        # softmax: False / True (model ends in softmax) or the output activation name ("sigmoid")
        out_act = 2 if softmax == "sigmoid" else (1 if softmax in (True, "softmax") else 0)
        _C().classifier_metrics(z.contiguous(), labels.to(torch.int32).contiguous(), METRIC_KINDS[loss], out_act,
                                out)
        return out
    from ..losses import accuracy, get_loss

    if softmax == "sigmoid":
        p = torch.sigmoid(z.float())
    else:
        p = torch.softmax(z.float(), dim=1) if softmax in (True, "softmax") else z.float()
    onehot = torch.nn.functional.one_hot(labels.long(), z.shape[1]).float()
    out[0] = get_loss(loss)(onehot, p).sum()
    out[1] = accuracy(labels, p).sum()
    return out


def lenet_supported() -> bool:
    m = native.get(build_if_missing=False)
    return m is not None and hasattr(m, "lenet_train")


def lenet_frag_bytes() -> int:
    return int(_C().lenet_frag_bytes())


def lenet_blocks(B: int) -> int:
    return int(_C().lenet_blocks(int(B)))


_LENET_TABLES = {}


def lenet_tables(device):
    """Constant index tables of the fused LeNet-5 kernel (built once per device):
    ``ftab`` [98][2][16] u8 — conv2 data gradient: for pool1 pixel pair (y, X2), k-half and step s, the
    stored row swz(t) = t ^ ((t >> 3) & 7) of the window-major conv2 output row t it gathers, inside the
    image's 104-row block (outside the 10x10 map: swz(100) = 96, a zero padding row);
    ``pxtab`` [832] i16 — padded conv2 output row (image * 104 + window * 4 + position) -> pool1 pixel
    index (padding rows 100..103 of an image: its pixel 0, read against a zero gradient);
    ``frag`` — scratch for the per-step conv weight fragments (written by the kernel's prep launch)."""
    key = str(device)
    if key not in _LENET_TABLES:
        import numpy as np

        swz = lambda t: t ^ ((t >> 3) & 7)  # noqa: E731  (csrc/lenet_fused.hip dc2_swz)
        ft = np.full((98, 2, 16), swz(100), dtype=np.uint8)
        for yx in range(98):
            y, X2 = divmod(yx, 7)
            for hf in range(2):
                for s in range(16):
                    P = 2 * s + hf
                    if P >= 30:
                        continue
                    ky, u = divmod(P, 6)
                    oy, ox = y - ky, 2 * X2 + 1 - u
                    if 0 <= oy < 10 and 0 <= ox < 10:
                        ft[yx, hf, s] = swz((((oy >> 1) * 5 + (ox >> 1)) << 2) + ((oy & 1) << 1) + (ox & 1))
        px = np.zeros(832, dtype=np.int16)
        for m in range(832):
            img, q = divmod(m, 104)
            if q >= 100:
                px[m] = img * 196
                continue
            win, d = divmod(q, 4)
            py, pxx = divmod(win, 5)
            px[m] = img * 196 + (2 * py + (d >> 1)) * 14 + 2 * pxx + (d & 1)
        nbytes = int(_C().lenet_frag_bytes())
        _LENET_TABLES[key] = (torch.from_numpy(ft.reshape(-1)).to(device), torch.from_numpy(px).to(device),
                              torch.zeros(nbytes, dtype=torch.uint8, device=device))
    return _LENET_TABLES[key]


def lenet_dense_part_floats(B: int) -> int:
    return int(_C().lenet_dense_part_floats(int(B)))


def lenet_train(x, labels, conv, dense_w, dense_wt, dense_b, conv_grads, dense_gw, dense_gb, hT, dzT, conv_part,
                dense_part, loss_part, stats, grad_scale, frag=None, prep=True, snap=None, conv_mom=(), sgd=None):
    """Whole-network LeNet-5 training step on GPU (csrc/lenet_fused.hip, 2 launches): fills every
    gradient and ``stats`` = [loss sum, correct].  ``x``: bf16 batch [B,28,28,1] or a :class:`GatherRef`
    over a uint8 dataset; ``labels``: int32 [B] or a :class:`LabelRef` through the same indices."""
    if isinstance(x, GatherRef):
        src, idx, scale = x.data, x.idx, x.scale
    else:
        src, idx, scale = x.contiguous(), None, 1.0
    if isinstance(labels, LabelRef):
        lab, lidx = labels.labels, labels.idx
        if idx is None:
            idx = lidx
    else:
        lab = labels if labels.dtype == torch.int32 else labels.to(torch.int32)
    B = x.shape[0]
    ftab, pxtab, scratch = lenet_tables(stats.device)
    # ``frag``: the fragment buffer the optimizer rebuilds (ParamStore.lenet_frag), refreshed by the prep
    # launch only when ``prep``; None = prep into scratch.  ``snap`` [2][2550]: the reduce kernel stores the
    # conv kernels' weights and momentum (``conv_mom``) there for the optimizer's rebuild.
    _C().lenet_train(src, idx, float(scale), lab, list(conv), list(dense_w), list(dense_wt), list(dense_b),
                     list(conv_grads), list(dense_gw), list(dense_gb), list(hT), list(dzT), conv_part, dense_part,
                     loss_part, stats, scratch if frag is None else frag, ftab, pxtab, int(B), float(grad_scale),
                     prep=bool(prep) or frag is None, snap=snap, conv_mom=list(conv_mom),
                     red_succ=_diag_on("lenet_succ"), **(sgd or {}))


def lenet_red_error(dense_part) -> int:
    """Sticky error word of the LeNet-5 reduce launch's granule hand-off (non-zero: a wait timed out)."""
    o = int(_C().lenet_red_err_offset())  # (layout: csrc/lenet_fused.hip lenet_red_bind_scratch)
    return int(dense_part[o:o + 1].view(torch.int32)[0].item())


def convpool_supported(H, W, C, KH, KW, pad, N) -> bool:
    m = native.get(build_if_missing=False)
    if m is None:
        return False
    return bool(m.convpool_supported(H, W, C, KH, KW, pad, N))


def convpool_fwd_layout(H, W, C, KH, KW, pad, N):
    """(channel stride Cp, row length Kpad2, pair) of the fused conv+pool forward weight layout."""
    return tuple(_C().convpool_fwd_layout(H, W, C, KH, KW, pad, N))


def convpool_dgrad_layout(H, W, C, KH, KW, pad, N):
    """(pair, row length K2pad) of the fused conv+pool data-gradient weight layout."""
    return tuple(_C().convpool_dgrad_layout(H, W, C, KH, KW, pad, N))


def _cp_in(x):
    if isinstance(x, GatherRef):
        return x.data, x.idx, x.scale
    return x, None, 1.0


def convpool_fwd(x, w, bias, out, code, KH, KW, pad):
    """Fused conv(stride 1) + bias + ReLU + maxpool 2x2 -> pooled map ``out`` and argmax ``code``."""
    B, H, W, C = x.shape
    N = out.shape[-1]
    if x.is_cuda:
        src, idx, scale = _cp_in(x)
        _C().convpool_fwd(src, idx, scale, w, bias, out, code, [B, H, W, C, KH, KW, pad, N])
    else:
        if isinstance(x, GatherRef):
            x = (x.data.index_select(0, x.idx).float() * x.scale).reshape(x.shape)
        p, c = ref.convpool_fwd(x, w, bias, KH, KW, pad)
        out.copy_(p)
        if code is not None:
            code.copy_(c)
    return out


def convpool_wgrad(x, dp, code, gw, gb, workspace, KH, KW, pad, defer: list | None = None):
    """``defer``: a list to which the GPU path appends its split-m slab reduction instead of launching
    it; run them all with :func:`flush_slab_reductions` (one launch, bit-identical results)."""
    B, H, W, C = x.shape
    N = code.shape[-1]
    if code.is_cuda:
        src, idx, scale = _cp_in(x)
        S = _C().convpool_wgrad(src, idx, scale, dp, code, gw, gb, workspace, [B, H, W, C, KH, KW, pad, N],
                                defer is not None)
        if defer is not None and S > 0:
            K = KH * KW * C
            defer.append((workspace, gw.reshape(-1), gb, N, K, K + 1, int(S), 1.0))
    else:
        if isinstance(x, GatherRef):
            x = (x.data.index_select(0, x.idx).float() * x.scale).reshape(x.shape)
        g, b = ref.convpool_wgrad(x, dp, code, KH, KW, pad)
        gw.copy_(g.reshape(gw.shape))
        if gb is not None:
            gb.copy_(b)


def flush_slab_reductions(pending: list):
    """One launch for the deferred slab reductions in ``pending`` (emptied)."""
    for i in range(0, len(pending), 8):
        _C().slab_reduce_multi(pending[i:i + 8])
    pending.clear()


def convpool_dgrad(dp, code, w, wt, dx, KH, KW, pad):
    B, H, W, C = dx.shape
    N = code.shape[-1]
    if code.is_cuda:
        _C().convpool_dgrad(dp, code, wt, dx, [B, H, W, C, KH, KW, pad, N])
    else:
        dx.copy_(ref.convpool_dgrad(dp, code, w, dx.shape, KH, KW, pad))
    return dx


def gather_labels(labels, idx, out):
    if out.is_cuda:
        _C().gather_labels(labels, idx, out)
    else:
        out.copy_(labels.index_select(0, idx))
    return out
