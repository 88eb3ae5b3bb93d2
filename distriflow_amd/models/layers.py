"""Layers of the distriflow_amd training engine (explicit forward/backward, no autograd tape).

The layer set is what the reference's models use — Keras/tf.js ``Conv2D``, ``Dense``,
``Activation``, ``MaxPooling2D``, ``Dropout``, ``Flatten`` (/root/reference/experiment/mnist/model.json:1,
/root/reference/experiment/mnist/mnist_server.ts:16-22) — plus BatchNorm / residual / global-average
pooling for the CIFAR-10 ResNet-18 config of BASELINE.json.

Execution model (MI355X-first):
  * every buffer (activations, gradients, workspaces) is allocated once per batch size by
    :meth:`Layer.alloc`, so the full step can be replayed as one hipGraph;
  * ReLU never runs as its own pass: forward ReLU is fused into the producing GEMM / BN / add
    epilogue, and relu' is fused into the CONSUMER's backward (dgrad epilogue mask, pool backward,
    dropout backward), driven by ``in_relu`` = "my input is a ReLU output";
  * the first layer skips its data gradient.
"""
from __future__ import annotations

import copy
import math
import os
import zlib
from typing import Optional

import torch

from .. import ops
from ..diagnostics import on as diag_on
from .params import ParamSpec, dgrad_shape, primary_kpad


def primary_kpad_of(conv) -> int:
    """Row length of a conv's forward compute copy (the igemm launch's Kpad)."""
    return primary_kpad(conv.specs()[0])


def dgrad_kpad_of(conv) -> int:
    """Row length of a conv's data-gradient compute copy (the dgrad launch's Kpad)."""
    return dgrad_shape(conv.specs()[0])[1]


class Layer:
    has_params = False

    def __init__(self, name: Optional[str] = None):
        self.name = name or type(self).__name__.lower()
        self.in_shape: tuple = ()
        self.out_shape: tuple = ()
        self.relu = False          # output passed through a fused ReLU
        self.in_relu = False       # input is a ReLU output (apply relu' in backward)
        self.grad_premasked = False  # relu' of this layer's output already applied to dy by the consumer
        # a Dropout that follows this layer, folded into its forward epilogue (Net._fold_dropout); the
        # consumer then applies the dropout backward: relu'(its input) * dx_scale = keep / (1 - p)
        self.drop: Optional["Dropout"] = None
        self.dx_scale = 1.0
        self.need_dx = True
        self.store = None
        self.x: Optional[torch.Tensor] = None
        self.out: Optional[torch.Tensor] = None
        self.dx: Optional[torch.Tensor] = None

    # shapes exclude the batch dimension
    def build(self, in_shape: tuple) -> tuple:
        self.in_shape = tuple(in_shape)
        self.out_shape = self.in_shape
        return self.out_shape

    def specs(self) -> list[ParamSpec]:
        return []

    def can_fuse_relu(self) -> bool:
        return False

    def alloc(self, B: int, device, dtype, ws):
        self.out = torch.empty((B,) + self.out_shape, device=device, dtype=dtype)
        if self.need_dx:
            self.dx = torch.empty((B,) + self.in_shape, device=device, dtype=dtype)

    def forward(self, x, training: bool):
        raise NotImplementedError

    def backward(self, dy):
        raise NotImplementedError

    # Layers that can separate their weight gradient from their data gradient set split_backward;
    # the engine then runs backward_weights on a side stream, concurrently with the data-gradient
    # chain of the layers below (backward == backward_weights + backward_data).
    split_backward = False

    def backward_weights(self, dy):
        raise NotImplementedError

    def backward_data(self, dy):
        raise NotImplementedError

    def config(self) -> dict:
        return {}

    def drop_spec(self, training: bool):
        d = self.drop
        if d is None or not training or d.rate <= 0:
            return None
        return d.spec()


class Dense(Layer):
    """y = act(x W^T + b); W stored [units][in] (Keras kernel [in][units] is transposed at I/O)."""
    has_params = True

    def __init__(self, units: int, activation: str = "linear", use_bias: bool = True, name=None,
                 kernel_initializer="glorot_uniform"):
        super().__init__(name or "dense")
        self.units = int(units)
        self.activation = activation
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer
        self.out_f32 = False  # final logits layer writes fp32
        if activation == "relu":
            self.relu = True
        elif activation not in ops.ACT_KINDS and activation != "softmax":
            raise NotImplementedError(f"Dense activation {activation!r}")
        # any other activation runs as its own streaming launch after the GEMM (Net._plan inserts it), or
        # folds into the loss when it ends the model (sigmoid / softmax)

    def build(self, in_shape):
        self.in_shape = tuple(in_shape)
        self.in_features = int(math.prod(in_shape))
        self.out_shape = (self.units,)
        return self.out_shape

    def can_fuse_relu(self):
        return True

    def specs(self):
        K, N = self.in_features, self.units
        s = [ParamSpec(f"{self.name}/kernel", (N, K), "matrix", (N, 1, K), self.kernel_initializer, (K, N),
                       needs_dgrad=self.need_dx)]
        if self.use_bias:
            s.append(ParamSpec(f"{self.name}/bias", (N,), "vector", init="zeros"))
        return s

    def alloc(self, B, device, dtype, ws):
        odt = torch.float32 if self.out_f32 else dtype
        self.out = torch.empty((B, self.units), device=device, dtype=odt)
        if self.need_dx:
            self.dx = torch.empty((B,) + self.in_shape, device=device, dtype=dtype)
        self.ws = ws

    def forward(self, x, training):
        self.x = x
        xf = x.reshape(x.shape[0], self.in_features)
        st = self.store
        b = st[f"{self.name}/bias"] if self.use_bias else None
        ops.dense_fwd(xf, st.weight(f"{self.name}/kernel"), b, self.out, relu=self.relu,
                      drop=self.drop_spec(training))
        return self.out

    def backward(self, dy):
        st = self.store
        xf = self.x.reshape(self.x.shape[0], self.in_features)
        kn = f"{self.name}/kernel"
        gb = st.gradient(f"{self.name}/bias") if self.use_bias else None
        ops.dense_wgrad(dy, xf, st.grad_matrix(kn), gb, self.ws.wgrad)
        if not self.need_dx:
            return None
        dxf = self.dx.view(self.dx.shape[0], self.in_features)
        mask = self.x.reshape(dxf.shape) if self.in_relu else None
        ops.dense_dgrad(dy, st.weight(kn), st.weight_t(kn), dxf, mask=mask, alpha=self.dx_scale)
        return self.dx

    def config(self):
        return {"units": self.units, "activation": self.activation, "use_bias": self.use_bias}


class Conv2D(Layer):
    """NHWC conv, kernel stored OHWI [Cout][KH*KW*Cin] (Keras HWIO converted at I/O)."""
    has_params = True

    def __init__(self, filters: int, kernel_size=(3, 3), strides=(1, 1), padding="valid", activation="linear",
                 use_bias=True, name=None, kernel_initializer="glorot_uniform"):
        super().__init__(name or "conv2d")
        self.filters = int(filters)
        self.kh, self.kw = ops._pair(kernel_size)
        self.sh, self.sw = ops._pair(strides)
        # k / stride / pad: the square kernel, single stride and symmetric padding of a regular conv (what
        # the fused and specialised paths match on); None when the geometry is not regular, which then runs
        # on the generic implicit-GEMM kernels (csrc/igemm.hip) with per-axis strides and top/left padding
        self.k = self.kh if self.kh == self.kw else None
        self.stride = self.sh if self.sh == self.sw else None
        self.padding = padding
        self.activation = activation
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer
        if activation == "relu":
            self.relu = True
        elif activation not in ops.ACT_KINDS:
            raise NotImplementedError(f"Conv2D activation {activation!r}")

    def build(self, in_shape):
        H, W, C = in_shape
        self.in_shape = (H, W, C)
        if self.padding == "same":
            (OH, OW), self.pads = ops.same_padding(H, W, self.kh, self.kw, (self.sh, self.sw))
        else:
            self.pads = (0, 0) if self.padding == "valid" else ops._pair(self.padding)
            OH, OW = ops.conv_out_hw(H, W, self.kh, self.kw, (self.sh, self.sw), self.pads)
        if OH < 1 or OW < 1:
            raise ValueError(f"Conv2D {self.name}: input {H}x{W} too small for kernel {self.kh}x{self.kw}")
        sym = (OH, OW) == ops.conv_out_hw(H, W, self.kh, self.kw, (self.sh, self.sw), self.pads)
        self.pad = self.pads[0] if sym and self.pads[0] == self.pads[1] else None
        self.regular = self.k is not None and self.stride is not None and self.pad is not None
        self.out_shape = (OH, OW, self.filters)
        return self.out_shape

    @property
    def geom(self):
        """(KH, KW, stride, pad) as the conv ops take them: ints when regular, else per-axis tuples."""
        if self.regular:
            return self.k, self.k, self.stride, self.pad
        return self.kh, self.kw, (self.sh, self.sw), self.pads

    def can_fuse_relu(self):
        return True

    def specs(self):
        H, W, C = self.in_shape
        K = self.kh * self.kw * C
        fan_in, fan_out = K, self.kh * self.kw * self.filters
        s = [ParamSpec(f"{self.name}/kernel", (self.filters, self.kh, self.kw, C), "matrix",
                       (self.filters, self.kh * self.kw, C), self.kernel_initializer, (fan_in, fan_out),
                       needs_dgrad=self.need_dx)]
        if self.use_bias:
            s.append(ParamSpec(f"{self.name}/bias", (self.filters,), "vector", init="zeros"))
        return s

    fwd_bn = None  # the BatchNorm that consumes this conv's output in a layer chain (Net._plan)

    def bacc_ok(self, dgrad: bool, mode: int, two: bool = False, has_res: bool = False, has_mask: bool = False) -> bool:
        """Can this conv's forward (or data-gradient) launch accumulate the sums of a consuming BatchNorm in
        its epilogue (csrc/bn_acc.h)?  Shape / dispatch dependent; cached per variant."""
        if self.out is None or self.out.device.type != "cuda" or not diag_on("bn_acc") or not self.regular:
            return False
        key = (dgrad, mode, two, has_res, has_mask)
        if key not in self._bacc_cache:
            H, W, C = self.in_shape
            OH, OW, N = self.out_shape
            kp = dgrad_kpad_of(self) if dgrad else primary_kpad_of(self)
            self._bacc_cache[key] = ops.conv_bacc_ok(self._B, H, W, C, OH, OW, N, self.k, self.k, self.stride, self.pad,
                                                     kp, dgrad=dgrad, mode=mode, two=two, has_res=has_res,
                                                     has_mask=has_mask)
        return self._bacc_cache[key]

    def alloc(self, B, device, dtype, ws):
        super().alloc(B, device, dtype, ws)
        self.ws = ws
        self._B = B
        self._bacc_cache = {}
        # BatchNorm statistics finalised inside this conv's own launches (csrc/bn_epi.h): the forward's for
        # the BN that consumes the output, the data gradient's for the BN that produced the input
        self._bn_fwd = self._bn_bwd = None
        if torch.device(device).type == "cuda" and diag_on("bn_epilogue") and self.regular:
            H, W, C = self.in_shape
            OH, OW, N = self.out_shape
            kpad = primary_kpad_of(self)
            z = lambda n, dt: torch.zeros(n, dtype=dt, device=device)  # noqa: E731
            ntm, ntn = ops.conv_bn_layout(B, H, W, C, OH, OW, N, self.k, self.k, self.stride, self.pad, kpad)
            if ntm:
                ng = -(-ntm // 16)
                self._bn_fwd = (z((ntm + ng) * 2 * N, torch.float32), z(ntn * (1 + ng), torch.int32))
            if self.need_dx:
                ntm, ntn = ops.conv_bn_layout(B, H, W, C, OH, OW, N, self.k, self.k, self.stride, self.pad,
                                              dgrad_kpad_of(self), dgrad=True)
                if ntm:
                    ng = -(-ntm // 16)
                    self._bn_bwd = (z((ntm + ng) * 2 * C, torch.float32), z(ntn * (1 + ng), torch.int32))

    def forward(self, x, training, bn: Optional["BatchNorm"] = None):
        """``bn``: the BatchNorm that consumes this output (default: ``fwd_bn``); in training its batch
        statistics come from this launch when it can: the epilogue accumulates their sums (csrc/bn_acc.h,
        default) or finalises them (``bn_epilogue`` diagnostic) -- no statistics pass over the output."""
        self.x = x
        st = self.store
        b = st[f"{self.name}/bias"] if self.use_bias else None
        bn = bn if bn is not None else self.fwd_bn
        spec = bacc = None
        if bn is not None and training and self._bn_fwd is not None:
            ws, tk = self._bn_fwd
            spec = dict(ws=ws, ticket=tk, mode=0, vecs=[bn.mean, bn.invstd, bn.run_mean, bn.run_var],
                        momentum=bn.momentum, eps=bn.eps)
        elif bn is not None and training and bn.acc_on and self.bacc_ok(False, 0):
            bacc = dict(acc=bn.acc, mode=0)
        ops.conv_fwd(x, st.weight(f"{self.name}/kernel"), b, self.out, *self.geom, relu=self.relu, bn=spec,
                     bacc=bacc)
        if spec is not None:
            bn.x = self.out
            bn._stats_ready = True
        if bacc is not None:
            bn.x = self.out
            bn._fwd_acc_ready = True
            bn._acc_nz[0] = True
        return self.out

    def can_emit_bn_grad(self) -> bool:
        return self._bn_bwd is not None

    def backward(self, dy, residual=None, residual_mask=None, dx_mask=None):
        """``residual`` / ``residual_mask`` / ``dx_mask``: the ResNet block join fused into the dgrad
        epilogue, dx = (conv^T dy + residual * [residual_mask > 0]) * [dx_mask > 0]."""
        self.backward_weights(dy)
        return self.backward_data(dy, residual, residual_mask, dx_mask)

    def backward_weights(self, dy):
        st = self.store
        kn = f"{self.name}/kernel"
        gb = st.gradient(f"{self.name}/bias") if self.use_bias else None
        ops.conv_wgrad(dy, self.x, st.grad_matrix(kn), gb, self.ws.wgrad, *self.geom)

    def backward_data(self, dy, residual=None, residual_mask=None, dx_mask=None, bn: Optional["BatchNorm"] = None,
                      bn_acc: Optional[list] = None):
        """``bn``: the BatchNorm whose output this layer consumed; its backward statistics (dgamma, dbeta,
        dx coefficients) are finalised inside this launch over the stored (masked) gradient.  ``bn_acc``:
        the (one or two) BatchNorms whose output gradient this data gradient IS (relu' applied by the
        epilogue mask): the epilogue accumulates their backward sums (csrc/bn_acc.h) when it can."""
        if not self.need_dx:
            return None
        st = self.store
        kn = f"{self.name}/kernel"
        mask = dx_mask if dx_mask is not None else (self.x if self.in_relu else None)
        spec = bacc = None
        if bn is not None:
            ws, tk = self._bn_bwd
            spec = dict(ws=ws, ticket=tk, mode=1, x=bn.x,
                        vecs=[bn.mean, bn.invstd, st[f"{bn.name}/gamma"], st.gradient(f"{bn.name}/gamma"),
                              st.gradient(f"{bn.name}/beta"), bn.coef])
        elif bn_acc and mask is not None and all(b.acc_on and b.x is not None for b in bn_acc) and len(bn_acc) <= 2 \
                and self.bacc_ok(True, 1, two=len(bn_acc) == 2, has_res=residual is not None, has_mask=True):
            b0 = bn_acc[0]
            bacc = dict(acc=b0.acc_b, mode=1, x=b0.x, mean=b0.mean, invstd=b0.invstd)
            if len(bn_acc) == 2:
                b1 = bn_acc[1]
                bacc.update(acc2=b1.acc_b, x2=b1.x, mean2=b1.mean, invstd2=b1.invstd)
        ops.conv_dgrad(dy, st.weight(kn), st.weight_t(kn), self.dx, *self.geom, mask=mask, residual=residual,
                       residual_mask=residual_mask, bn=spec, bacc=bacc)
        if bacc is not None:
            for b in bn_acc:
                b._bwd_acc_ready = True
                b._acc_nz[1] = True
        return self.dx

    def config(self):
        return {"filters": self.filters, "kernel_size": [self.kh, self.kw], "strides": [self.sh, self.sw],
                "padding": self.padding if isinstance(self.padding, str) else "valid",
                "activation": self.activation, "use_bias": self.use_bias}


def _pair(v, default=None):
    if v is None:
        return default
    return (int(v[0]), int(v[1])) if isinstance(v, (list, tuple)) else (int(v), int(v))


class MaxPooling2D(Layer):
    """Keras MaxPooling2D: any pool_size / strides, 'valid' or 'same' padding.  Square pool == stride,
    'valid' (the MNIST CNNs) takes the vectorised max-pool kernels, which also fold a following Dropout
    and the fused conv+pool plans; everything else the general pooling kernels (csrc/act.hip)."""
    avg = False

    def __init__(self, pool_size=2, strides=None, padding="valid", name=None):
        super().__init__(name or ("average_pooling2d" if self.avg else "max_pooling2d"))
        self.pool = _pair(pool_size)
        self.strides = _pair(strides, self.pool)
        self.padding = padding
        if padding not in ("valid", "same"):
            raise NotImplementedError(f"pooling padding {padding!r}")
        # the fast square case keeps the historical attribute name
        self.p = self.pool[0] if (self.pool[0] == self.pool[1] == self.strides[0] == self.strides[1]
                                  and padding == "valid" and not self.avg) else 0

    @property
    def simple(self) -> bool:
        return self.p > 0

    def build(self, in_shape):
        H, W, C = in_shape
        self.in_shape = (H, W, C)
        if self.simple:
            self.out_shape = (H // self.p, W // self.p, C)
        else:
            g = ops.pool_geometry(1, H, W, C, self.pool, self.strides, self.padding)
            self.out_shape = (g[4], g[5], C)
        return self.out_shape

    def _geom(self, B):
        H, W, C = self.in_shape
        return ops.pool_geometry(B, H, W, C, self.pool, self.strides, self.padding)

    def forward(self, x, training):
        self.x = x
        if self.simple:
            ops.maxpool_fwd(x, self.out, self.p, drop=self.drop_spec(training))
            return self.out
        ops.pool2d_fwd(x, self.out, self._geom(x.shape[0]), avg=self.avg)
        d = self.drop_spec(training)
        if d is not None:
            ops.dropout(self.out, self.out, d[0], d[1], step=d[2], step_add=d[3] if len(d) > 3 else 0)
        return self.out

    def backward(self, dy):
        if not self.need_dx:
            return None
        if self.simple:
            ops.maxpool_bwd(self.x, dy, self.dx, self.p, relu_fused=self.in_relu)
        else:
            ops.pool2d_bwd(self.x, dy.reshape(self.out.shape), self.dx, self._geom(self.x.shape[0]), avg=self.avg,
                           in_relu=self.in_relu)
        return self.dx

    def config(self):
        return {"pool_size": list(self.pool), "strides": list(self.strides), "padding": self.padding}


class AveragePooling2D(MaxPooling2D):
    """Keras AveragePooling2D ('same' padding averages over the in-image pixels only, as TensorFlow)."""
    avg = True


class Dropout(Layer):
    """Inverted dropout with a counter-based mask (seed, step, element) regenerated in backward."""

    def __init__(self, rate: float, name=None, seed: int = 1234):
        super().__init__(name or "dropout")
        self.rate = float(rate)
        self.base_seed = seed
        self.step = 0
        self.step_add = 0  # 1 when the engine advances the step counter at the end of the step
        self.active = False

    def _seed(self):
        return (self.base_seed * 1000003 + zlib.crc32(self.name.encode()) % 100003) & 0x7FFFFFFFFFFF

    def spec(self):
        """(rate, seed, device step) of the mask, for a producer that folds this dropout in."""
        return (self.rate, self._seed(), self.step_dev, self.step_add)

    def forward(self, x, training):
        self.x = x
        self.active = training and self.rate > 0
        if not self.active:
            return x
        # the per-step part of the seed is read from device memory (self.step_dev, advanced by the
        # engine inside the captured step), so graph replays draw fresh masks
        ops.dropout(x, self.out, self.rate, self._seed(), step=self.step_dev)
        return self.out

    def backward(self, dy):
        if not self.need_dx:
            return None
        if not self.active:
            if self.in_relu:
                return ops.relu_bwd(self.x, dy, self.dx)
            return dy
        ops.dropout(dy, self.dx, self.rate, self._seed(), mask=self.x if self.in_relu else None, step=self.step_dev)
        return self.dx

    def config(self):
        return {"rate": self.rate}


class Flatten(Layer):
    """View only: consumers reshape their input; never executed in a chain (inside a branching graph,
    models/graph.py, forward / backward are reshapes of the same storage)."""

    def build(self, in_shape):
        self.in_shape = tuple(in_shape)
        self.out_shape = (int(math.prod(in_shape)),)
        return self.out_shape

    def alloc(self, B, device, dtype, ws):
        self.out = self.dx = None

    def forward(self, x, training):
        self.out = x.reshape((x.shape[0],) + self.out_shape)
        return self.out

    def backward(self, dy):
        if not self.need_dx:
            return None
        self.dx = dy.reshape((dy.shape[0],) + self.in_shape)
        return self.dx


class Activation(Layer):
    """Keras Activation.  The engine fuses relu into the producer's epilogue and a final softmax /
    sigmoid into the loss; any other placement executes here as one streaming launch forward
    (y = act(x)) and one backward (dx = dy * act'(x), csrc/act.hip)."""

    def __init__(self, activation: str, name=None, implicit: bool = False):
        super().__init__(name or "activation")
        if activation not in ops.ACT_KINDS and activation != "softmax":
            raise NotImplementedError(f"activation {activation!r}")
        self.activation = activation
        self.implicit = implicit  # split off a Dense / Conv2D activation (not a Keras layer of its own)

    def forward(self, x, training):
        self.x = x
        ops.act_fwd(x, self.out.view(x.shape), self.activation)
        return self.out

    def backward(self, dy):
        if not self.need_dx:
            return None
        ops.act_bwd(self.x, dy.reshape(self.x.shape), self.dx.view(self.x.shape), self.activation,
                    in_relu=self.in_relu)
        return self.dx

    def config(self):
        return {"activation": self.activation}


class BatchNorm(Layer):
    """BatchNorm over channels (NHWC / [B][F]) with fused ReLU; gamma/beta trainable, running stats buffers."""
    has_params = True

    def __init__(self, momentum=0.1, eps=1e-5, relu=False, name=None):
        super().__init__(name or "batch_normalization")
        self.momentum = momentum
        self.eps = eps
        self.relu = relu

    def build(self, in_shape):
        self.in_shape = self.out_shape = tuple(in_shape)
        self.C = in_shape[-1]
        return self.out_shape

    def specs(self):
        return [ParamSpec(f"{self.name}/gamma", (self.C,), "vector", init="ones"),
                ParamSpec(f"{self.name}/beta", (self.C,), "vector", init="zeros")]

    def alloc(self, B, device, dtype, ws):
        super().alloc(B, device, dtype, ws)
        self.ws = ws
        if not hasattr(self, "run_mean") or self.run_mean.device != torch.device(device):
            self.run_mean = torch.zeros(self.C, device=device)
            self.run_var = torch.ones(self.C, device=device)
        self.mean = torch.zeros(self.C, device=device)
        self.invstd = torch.ones(self.C, device=device)
        self.coef = torch.zeros(3 * self.C, device=device)               # dx = k1*g + k2*x + k3
        # last-arriver ticket counters of the statistics launches (forward row 0, backward row 1)
        self.counter = torch.zeros(2, ops.BN_COUNTERS, dtype=torch.int32, device=device)
        # sums accumulated by the producing kernels' epilogues (csrc/bn_acc.h): acc = forward [S, Q] of the
        # conv output, acc_b = backward [S, Q] of the output gradient; each consumer clears the other one
        C = self.C
        self.acc_on = (torch.device(device).type == "cuda" and diag_on("bn_acc") and C % 8 == 0 and C <= 1024
                       and 256 % (C // 8) == 0)
        self.acc = self.acc_b = None
        if self.acc_on:
            from ..diagnostics import diag

            nrep = max(1, min(16, diag("bn_acc_rep")))
            self.acc_all = torch.zeros(2, nrep, 2, C, dtype=torch.float64, device=device)
            self.acc, self.acc_b = self.acc_all[0], self.acc_all[1]
        self._fwd_acc_ready = self._bwd_acc_ready = False
        # "possibly non-zero" flags of acc / acc_b: set when a producer launch is given them, cleared by the
        # consumer that zeroes them (bn_dx_acc clears acc, bn_apply_acc clears acc_b); drop_acc clears only
        # what may hold sums (two memsets per BN per step for nothing)
        self._acc_nz = [False, False]

    def stats(self, x):
        """Training-mode batch statistics of ``x`` (and the running statistics); writes no output."""
        self.x = x
        ops.bn_stats_fwd(x.reshape(-1, self.C), self.mean, self.invstd, self.run_mean, self.run_var, self.ws.bn,
                         self.counter[0], self.momentum, self.eps)

    def affine(self, training):
        st = self.store
        g, b = st[f"{self.name}/gamma"], st[f"{self.name}/beta"]
        return (g, b, self.mean, self.invstd) if training else (g, b, self.run_mean, self.run_var)

    def apply(self, x, out, training, residual=None, residual_bn=None, relu=None):
        """out = act(bn(x) [+ residual | + residual_bn(residual)]) in one streaming pass."""
        g, b, m, v = self.affine(training)
        rbn = residual_bn.affine(training) if residual_bn is not None else None
        ops.bn_apply(x.reshape(-1, self.C), out.view(-1, self.C), g, b, m, v, self.relu if relu is None else relu,
                     residual.reshape(-1, self.C) if residual is not None else None, rbn, not training, self.eps)
        return out

    _stats_ready = False

    def fused_forward(self, x, out, residual=None, residual_bn=None, relu=None) -> bool:
        """Training statistics + apply in one launch when the fused kernel covers this shape (the
        statistics were not already produced by the conv epilogue); False: nothing launched."""
        if self._stats_ready or not ops.bn_fused_ok(self.C, x.device):
            return False
        self.x = x
        st = self.store
        rbn = residual_bn.affine(True) if residual_bn is not None else None
        ops.bn_fwd_fused(x.reshape(-1, self.C), out.view(-1, self.C), st[f"{self.name}/gamma"], st[f"{self.name}/beta"],
                         self.mean, self.invstd, self.run_mean, self.run_var, self.ws.bn, self.counter[0],
                         self.relu if relu is None else relu,
                         residual.reshape(-1, self.C) if residual is not None else None, rbn, self.momentum, self.eps)
        return True

    def apply_acc(self, x, out, residual=None, residual_bn=None, relu=None):
        """Training out = act(bn(x) [+ residual | + residual_bn(residual)]) with the statistics finalised from
        the producers' accumulated sums (this BN's and the residual BN's): one launch, no statistics pass."""
        st = self.store
        rb = None
        if residual_bn is not None:
            r = residual_bn
            rb = [st[f"{r.name}/gamma"], st[f"{r.name}/beta"], r.acc, r.acc_b, r.mean, r.invstd, r.run_mean, r.run_var]
            r._fwd_acc_ready = False
            r._acc_nz[1] = False
        self._fwd_acc_ready = False
        self._acc_nz[1] = False
        ops.bn_apply_acc(x.reshape(-1, self.C), out.view(-1, self.C), st[f"{self.name}/gamma"], st[f"{self.name}/beta"],
                         self.acc, self.acc_b, self.mean, self.invstd, self.run_mean, self.run_var,
                         self.relu if relu is None else relu,
                         residual.reshape(-1, self.C) if residual is not None else None, rb, self.momentum, self.eps)
        return out

    def drop_acc(self):
        """This step's statistics take the other path: clear the accumulators a producer may have added into
        (the producers only ever add into zeroed ones), so a later step can use the accumulated path again."""
        self._fwd_acc_ready = self._bwd_acc_ready = False
        if self.acc_on and (self._acc_nz[0] or self._acc_nz[1]):
            self.acc_all.zero_()
        self._acc_nz = [False, False]

    def forward(self, x, training):
        self.x = x
        if training and self._fwd_acc_ready:  # the producer accumulated this batch's sums
            return self.apply_acc(x, self.out)
        if training and self.acc_on:
            self.drop_acc()
        if training and self.fused_forward(x, self.out):
            return self.out
        if training and not self._stats_ready:
            self.stats(x)
        self._stats_ready = False
        return self.apply(x, self.out, training)

    def _dx_from_acc(self, g):
        """dx from a gradient g whose backward sums the producing kernel accumulated (relu' applied)."""
        st = self.store
        self._bwd_acc_ready = False
        self._acc_nz[0] = False
        ops.bn_dx_acc(self.x.reshape(-1, self.C), g.reshape(-1, self.C), self.dx.view(-1, self.C), self.acc_b, self.acc,
                      st[f"{self.name}/gamma"], self.mean, self.invstd, st.gradient(f"{self.name}/gamma"),
                      st.gradient(f"{self.name}/beta"), self.coef)
        return self.dx

    def backward_dx(self, g):
        """dx from a gradient ``g`` (relu' already applied) whose statistics the producing conv launch
        finalised (Conv2D.backward_data(bn=self)) or accumulated (bn_acc=[self]): the dx pass only."""
        if self._bwd_acc_ready:
            return self._dx_from_acc(g)
        ops.bn_dx(self.x.reshape(-1, self.C), g.reshape(-1, self.C), self.dx.view(-1, self.C), self.coef)
        return self.dx

    def backward(self, dy, mask=None):
        """``mask``: relu' source applied to dy (default: this layer's own output when it ends in ReLU)."""
        if self._bwd_acc_ready:  # dy is the premasked g whose sums its producer accumulated
            if self.in_relu:
                raise NotImplementedError("BatchNorm after a fused ReLU")
            return self._dx_from_acc(dy)
        if self.acc_on:
            self.drop_acc()
        st = self.store
        if mask is None and self.relu and not self.grad_premasked:
            mask = self.out
        ops.bn_bwd(self.x.reshape(-1, self.C), mask.reshape(-1, self.C) if mask is not None else None,
                   dy.reshape(-1, self.C), self.dx.view(-1, self.C), st[f"{self.name}/gamma"], self.mean, self.invstd,
                   st.gradient(f"{self.name}/gamma"), st.gradient(f"{self.name}/beta"), self.ws.bn, self.coef,
                   self.counter[1])
        if self.in_relu:
            raise NotImplementedError("BatchNorm after a fused ReLU")
        return self.dx


class GlobalMaxPooling2D(MaxPooling2D):
    """Keras GlobalMaxPooling2D: a max over the whole H x W map (general pooling kernel), output [C]."""

    def __init__(self, name=None):
        super().__init__(1, 1, "valid", name=name or "global_max_pooling2d")
        self.p = 0

    def build(self, in_shape):
        H, W, C = in_shape
        self.in_shape = (H, W, C)
        self.pool = self.strides = (H, W)
        self.out_shape = (C,)
        return self.out_shape

    def config(self):
        return {}


class GlobalAveragePooling2D(Layer):
    def build(self, in_shape):
        H, W, C = in_shape
        self.in_shape = (H, W, C)
        self.out_shape = (C,)
        return self.out_shape

    def forward(self, x, training):
        self.x = x
        ops.gap_fwd(x, self.out)
        return self.out

    def backward(self, dy):
        if not self.need_dx:
            return None
        sinks = getattr(self, "dx_bn_sinks", None) or []
        if (self.in_relu and len(sinks) == 1 and sinks[0].acc_on and sinks[0].x is not None and self.dx.is_cuda
                and self.dx.shape[-1] <= 1024 and 256 % (self.dx.shape[-1] // 4) == 0):
            # the relu' of the producing block's output and that block's last BatchNorm's backward sums in
            # the same launch (its gradient g IS this dx)
            b = sinks[0]
            ops.gap_bwd_bn(dy, self.x, self.dx, b.acc_b, b.x, b.mean, b.invstd)
            b._bwd_acc_ready = True
            b._acc_nz[1] = True
            return self.dx
        ops.gap_bwd(dy, self.dx)
        if self.in_relu:
            ops.relu_bwd(self.x, self.dx, self.dx)
        return self.dx


class ResidualBlock(Layer):
    """ResNet basic block: relu(bn2(conv2(relu(bn1(conv1(x))))) + shortcut(x)).

    shortcut = identity, or conv1x1(stride) + BN when the shape changes.  Sub-layers are engine
    layers, so every conv/BN runs on the same MFMA / BN kernels; the final add + ReLU is one fused
    kernel (``add_act``) and its relu' is applied once to the incoming gradient.
    """
    has_params = True

    side_stream = None  # set by the engine: stream for the weight gradients (None: in order on the main stream)
    proj_stream = None  # set by the engine: stream for the projection shortcut branch (None: in order)

    def __init__(self, filters: int, stride: int = 1, name=None):
        super().__init__(name or "block")
        self.filters = filters
        self.stride = stride
        self.relu = True

    def build(self, in_shape):
        H, W, C = in_shape
        self.in_shape = (H, W, C)
        n = self.name
        self.conv1 = Conv2D(self.filters, 3, self.stride, 1, use_bias=False, name=f"{n}/conv1",
                            kernel_initializer="he_normal")
        self.bn1 = BatchNorm(relu=True, name=f"{n}/bn1")
        self.conv2 = Conv2D(self.filters, 3, 1, 1, use_bias=False, name=f"{n}/conv2", kernel_initializer="he_normal")
        self.bn2 = BatchNorm(relu=False, name=f"{n}/bn2")
        s = self.conv1.build(self.in_shape)
        s = self.bn1.build(s)
        s = self.conv2.build(s)
        s = self.bn2.build(s)
        self.proj = None
        if self.stride != 1 or C != self.filters:
            self.proj = Conv2D(self.filters, 1, self.stride, 0, use_bias=False, name=f"{n}/proj",
                               kernel_initializer="he_normal")
            self.proj_bn = BatchNorm(relu=False, name=f"{n}/proj_bn")
            self.proj_bn.build(self.proj.build(self.in_shape))
        self.out_shape = s
        return s

    def sublayers(self):
        ls = [self.conv1, self.bn1, self.conv2, self.bn2]
        if self.proj is not None:
            ls += [self.proj, self.proj_bn]
        return ls

    def specs(self):
        out = []
        for l in self.sublayers():
            out += l.specs()
        return out

    def bind_store(self, store):
        self.store = store
        for l in self.sublayers():
            l.store = store

    def alloc(self, B, device, dtype, ws):
        self.conv1.need_dx = self.need_dx
        if self.proj is not None:
            self.proj.need_dx = self.need_dx
        for l in self.sublayers():
            l.alloc(B, device, dtype, ws)
        if self.proj is not None:
            # the projection branch may run on its own stream (proj_stream): its BatchNorm gets a private
            # statistics workspace so it never shares slabs with bn1 / bn2 on the main stream
            pws = copy.copy(ws)
            pws.bn = torch.empty_like(ws.bn)
            self.proj_bn.ws = pws
        self.out = torch.empty((B,) + self.out_shape, device=device, dtype=dtype)
        # conv1's data gradient IS the block's: its dgrad epilogue adds the shortcut gradient and relu'(x)
        self.dx = self.conv1.dx if self.need_dx else None

    def _proj_forward(self, x, training):
        p = self.proj.forward(x, training, bn=self.proj_bn)
        self.proj_bn.x = p
        if training and not self.proj_bn._stats_ready and not self.proj_bn._fwd_acc_ready:
            self.proj_bn.stats(p)
        self.proj_bn._stats_ready = False
        return p

    def forward(self, x, training):
        self.x = x
        ps = self.proj_stream if self.proj is not None else None
        pev = None
        if ps is not None:  # projection shortcut concurrently with conv1 -> bn1 -> conv2 -> bn2 statistics
            main = torch.cuda.current_stream(ps.device)
            ps.wait_event(main.record_event())
            with torch.cuda.stream(ps):
                p = self._proj_forward(x, training)
                pev = ps.record_event()
        h = self.conv1.forward(x, training, bn=self.bn1)
        h = self.bn1.forward(h, training)
        h = self.conv2.forward(h, training, bn=self.bn2)
        self.bn2.x = h
        r, rbn = x, None
        if self.proj is not None:
            if pev is not None:
                main.wait_event(pev)
            else:
                p = self._proj_forward(x, training)
            r, rbn = p, self.proj_bn
        # out = relu(bn2(h) + shortcut), shortcut = x or proj_bn(proj(x)): with the producers' accumulated
        # sums one streaming launch finalises both BatchNorms' statistics and joins; else bn2's statistics
        # and this streaming pass in one launch when the fused kernel covers the shape
        if training and self.bn2._fwd_acc_ready and (rbn is None or rbn._fwd_acc_ready):
            self.bn2.apply_acc(h, self.out, residual=r, residual_bn=rbn, relu=True)
            return self.out
        for b in (self.bn2, rbn):  # (only one of the two has accumulated sums: statistics passes instead)
            if training and b is not None and b._fwd_acc_ready:
                b.drop_acc()
                b.stats(b.x)
                if b is self.bn2:
                    b._stats_ready = True
        if training and self.bn2.fused_forward(h, self.out, residual=r, residual_bn=rbn, relu=True):
            return self.out
        if training and not self.bn2._stats_ready:
            self.bn2.stats(h)
        self.bn2._stats_ready = False
        self.bn2.apply(h, self.out, training, residual=r, residual_bn=rbn, relu=True)
        return self.out

    def backward(self, dy):
        # relu' of the block output is applied inside both BN backward passes (mask = block output),
        # unless the consumer already applied it to dy (grad_premasked: the next block's dgrad epilogue or
        # the pooling backward masks with this block's output)
        omask = None if self.grad_premasked else self.out
        side = self.side_stream
        ps = self.proj_stream if self.proj is not None else None

        def weights(conv, g):
            # weight gradients on the side stream (the engine joins it before the gradients are read):
            # they overlap the latency-bound BatchNorm passes and data gradients of the main chain
            if side is None:
                conv.backward_weights(g)
                return
            side.wait_event(torch.cuda.current_stream(side.device).record_event())
            with torch.cuda.stream(side):
                conv.backward_weights(g)

        def proj_branch():
            p = self.proj_bn.backward(dy, mask=omask)
            weights(self.proj, p)
            return self.proj.backward_data(p)

        ds = pev = None
        if ps is not None:  # the projection branch needs only dy: run it beside bn2 -> conv2 -> bn1
            main = torch.cuda.current_stream(ps.device)
            ps.wait_event(main.record_event())
            with torch.cuda.stream(ps):
                ds = proj_branch()
                pev = ps.record_event()
        d = self.bn2.backward(dy, mask=omask)
        weights(self.conv2, d)
        if (self.bn1.acc_on and not self.bn1.grad_premasked
                and self.conv2.bacc_ok(True, 1, two=False, has_res=False, has_mask=True)):
            # conv2's data gradient applies bn1's relu' and accumulates bn1's backward sums (csrc/bn_acc.h)
            d = self.conv2.backward_data(d, dx_mask=self.bn1.out, bn_acc=[self.bn1])
            d = self.bn1.backward_dx(d)
        elif self.conv2.can_emit_bn_grad() and not self.bn1.grad_premasked:
            # conv2's data gradient applies bn1's relu' and finalises bn1's backward statistics itself
            d = self.conv2.backward_data(d, dx_mask=self.bn1.out, bn=self.bn1)
            d = self.bn1.backward_dx(d)
        else:
            d = self.conv2.backward_data(d)
            d = self.bn1.backward(d)
        if self.proj is not None:
            if pev is not None:
                main.wait_event(pev)
            else:
                ds = proj_branch()
        weights(self.conv1, d)
        if not self.need_dx:
            return None
        # conv1's dgrad epilogue joins the branches: dx = (conv1^T d + shortcut grad) * relu'(x), where the
        # shortcut gradient is proj^T(...) or the identity path's dy * relu'(out)
        if self.proj is not None:
            res, res_mask = ds, None
        else:
            res, res_mask = dy, omask
        # and, when the previous layer's BatchNorms consume this gradient (Net._plan: dx_bn_sinks), their
        # backward sums accumulate in the same epilogue
        self.conv1.backward_data(d, residual=res, residual_mask=res_mask, dx_mask=self.x if self.in_relu else None,
                                 bn_acc=getattr(self, "dx_bn_sinks", None) if self.in_relu else None)
        return self.dx

    def config(self):
        return {"filters": self.filters, "stride": self.stride}


class FusedConvPool(Layer):
    """Conv2D(stride 1, +bias, ReLU) immediately followed by MaxPooling2D(2): one fused kernel each for
    forward, weight gradient and data gradient (csrc/convpool.hip).  Only the pooled map and a 1-byte
    argmax/relu' code are materialised; the parameters keep the Conv2D's names (checkpoint-compatible).
    relu' of this layer's output is applied inside its own backward (code bit 2), so consumers see
    ``relu = False``."""
    has_params = True

    def __init__(self, conv: "Conv2D", pool: "MaxPooling2D"):
        super().__init__(conv.name)
        self.conv, self.pool = conv, pool
        self.k, self.pad = conv.k, conv.pad
        self.use_bias = conv.use_bias
        self.in_shape = conv.in_shape
        self.out_shape = pool.out_shape
        self.relu = False

    def specs(self):
        self.conv.need_dx = self.need_dx
        sp = self.conv.specs()
        # the forward reads the row-segment weight layout chosen by the kernel (csrc/convpool.hip)
        H, W, C = self.in_shape
        cp, _, pair = ops.convpool_fwd_layout(H, W, C, self.k, self.k, self.pad, self.conv.filters)
        sp[0].row_pad, sp[0].row_cp, sp[0].row_pair = self.k, cp, bool(pair)
        if self.need_dx:
            sp[0].t_pair = bool(ops.convpool_dgrad_layout(H, W, C, self.k, self.k, self.pad, self.conv.filters)[0])
        return sp

    split_backward = True

    def alloc(self, B, device, dtype, ws):
        self.out = torch.empty((B,) + self.out_shape, device=device, dtype=dtype)
        self.code = torch.empty((B,) + self.out_shape, device=device, dtype=torch.uint8)
        if self.need_dx:
            self.dx = torch.empty((B,) + self.in_shape, device=device, dtype=dtype)
        # private split-m slab workspace: this layer's weight gradient may run concurrently with others
        self.ws_wgrad = torch.empty(1 << 22, dtype=torch.float32, device=device) if device.type == "cuda" else ws.wgrad

    def forward(self, x, training):
        self.x = x
        st = self.store
        b = st[f"{self.name}/bias"] if self.use_bias else None
        ops.convpool_fwd(x, st.weight(f"{self.name}/kernel"), b, self.out, self.code, self.k, self.k, self.pad)
        return self.out

    def backward_weights(self, dy, defer=None):
        st = self.store
        kn = f"{self.name}/kernel"
        gb = st.gradient(f"{self.name}/bias") if self.use_bias else None
        ops.convpool_wgrad(self.x, dy.reshape(self.out.shape), self.code, st.grad_matrix(kn), gb, self.ws_wgrad,
                           self.k, self.k, self.pad, defer=defer)

    def backward_data(self, dy):
        if not self.need_dx:
            return None
        st = self.store
        kn = f"{self.name}/kernel"
        ops.convpool_dgrad(dy.reshape(self.out.shape), self.code, st.weight(kn), st.weight_t(kn), self.dx, self.k,
                           self.k, self.pad)
        if self.in_relu:
            ops.relu_bwd(self.x, self.dx, self.dx)
        return self.dx

    def backward(self, dy, defer=None):
        self.backward_weights(dy, defer)
        return self.backward_data(dy)


class ConvPoolGemm(Layer):
    """Conv2D(stride 1, +bias, ReLU) followed by MaxPooling2D(2) for C % 8 == 0 (the Keras CNN's conv2,
    /root/reference/experiment/mnist/model.json: conv2d_2 -> max_pooling2d_1): the igemm64 forward
    reduces each 2x2 window in its epilogue (csrc/igemm64.hip POOL), so only the pooled map and a
    1-byte argmax code per pooled element reach HBM and no max-pool launch remains.  Backward: one
    unpool launch rebuilds the conv's output gradient from the codes, then the conv's own weight- and
    data-gradient kernels.  A following Dropout can fold in (Net._fold_dropout).  Parameter names are the
    Conv2D's (checkpoint-compatible)."""
    has_params = True

    def __init__(self, conv: "Conv2D", pool: "MaxPooling2D"):
        super().__init__(conv.name)
        self.conv, self.pool = conv, pool
        self.use_bias = conv.use_bias
        self.in_shape = conv.in_shape
        self.out_shape = pool.out_shape
        self.relu = False  # relu' is carried by the codes (4 = no gradient)

    def specs(self):
        self.conv.need_dx = self.need_dx
        return self.conv.specs()

    def alloc(self, B, device, dtype, ws):
        c = self.conv
        c.in_relu, c.need_dx, c.ws, c.store = self.in_relu, self.need_dx, ws, self.store
        c.dx = torch.empty((B,) + c.in_shape, device=device, dtype=dtype) if self.need_dx else None
        self.out = torch.empty((B,) + self.out_shape, device=device, dtype=dtype)
        self.code = torch.empty((B,) + self.out_shape, device=device, dtype=torch.uint8)
        self.dy_full = torch.empty((B,) + self.conv.out_shape, device=device, dtype=dtype)
        self.dx = self.conv.dx

    def forward(self, x, training):
        self.x = x
        c = self.conv
        c.x = x
        st = self.store
        b = st[f"{c.name}/bias"] if c.use_bias else None
        ops.conv_pool_fwd(x, st.weight(f"{c.name}/kernel"), b, self.out, self.code, c.k, c.k, c.stride, c.pad,
                          relu=c.relu, drop=self.drop_spec(training))
        return self.out

    def backward(self, dy):
        ops.unpool2(dy.reshape(self.out.shape), self.code, self.dy_full)
        self.conv.store = self.store
        return self.conv.backward(self.dy_full)

    def config(self):
        return self.conv.config()


class KerasConvBlock(Layer):
    """conv2d_1 (3x3x1 -> 32, ReLU) -> conv2d_2 (3x3x32 -> 32, ReLU) -> max_pooling2d_1 (2x2) of the
    reference CNN (/root/reference/experiment/mnist/model.json) on 28x28x1 inputs, as one layer of two
    launches forward / backward (csrc/kcnn_fused.hip): conv1's activation and gradient live only in LDS,
    conv2's output only as the pooled map plus argmax codes.  Reads dataset rows through the batch index
    (no gather launch).  A following Dropout folds in (Net._fold_dropout); the backward's reduce advances
    the dropout step.  Parameters keep both convs' names (checkpoint-compatible).  GPU only."""
    has_params = True

    def __init__(self, conv1: "Conv2D", conv2: "Conv2D", pool: "MaxPooling2D"):
        super().__init__(conv1.name)
        self.conv1, self.conv2, self.pool = conv1, conv2, pool
        self.in_shape = conv1.in_shape
        self.out_shape = pool.out_shape
        self.relu = False  # relu' rides in the codes
        self.step_inc = None

    @staticmethod
    def matches(c1, c2) -> bool:
        def conv_ok(c, shape, cin):
            return (isinstance(c, Conv2D) and c.k == 3 and c.stride == 1 and c.pad == 0 and c.relu and c.use_bias
                    and c.filters == 32 and tuple(c.in_shape) == shape and c.in_shape[2] == cin)
        return conv_ok(c1, (28, 28, 1), 1) and conv_ok(c2, (26, 26, 32), 32)

    def specs(self):
        self.conv1.need_dx = False
        self.conv2.need_dx = True  # the backward reads conv2's data-gradient weight copy
        return self.conv1.specs() + self.conv2.specs()

    def alloc(self, B, device, dtype, ws):
        self.out = torch.empty((B,) + self.out_shape, device=device, dtype=dtype)
        self.code = torch.empty((B,) + self.out_shape, device=device, dtype=torch.uint8)
        self.slabs = torch.empty(ops.kcnn_slab_floats(B), dtype=torch.float32, device=device)
        self.dx = None

    def _w(self):
        st, c1, c2 = self.store, self.conv1.name, self.conv2.name
        return st.weight(f"{c1}/kernel"), st[f"{c1}/bias"], st.weight(f"{c2}/kernel"), st[f"{c2}/bias"]

    def forward(self, x, training):
        self.x = x
        w1, b1, w2, b2 = self._w()
        ops.kcnn_fwd(x, w1, b1, w2, b2, self.out, self.code, drop=self.drop_spec(training))
        return self.out

    def backward(self, dy):
        st, c1, c2 = self.store, self.conv1.name, self.conv2.name
        w1, b1, _, _ = self._w()
        ops.kcnn_bwd(self.x, w1, b1, st.weight_t(f"{c2}/kernel"), dy.reshape(self.out.shape), self.code, self.slabs,
                     st.gradient(f"{c1}/kernel"), st.gradient(f"{c1}/bias"), st.gradient(f"{c2}/kernel"),
                     st.gradient(f"{c2}/bias"), step_inc=self.step_inc)
        return None

    def config(self):
        return self.conv1.config()

