"""Flat parameter storage for the training engine.

All trainable tensors of a model live in ONE contiguous fp32 master buffer (and one fp32 gradient
buffer with identical offsets), in model order — kernel then bias, exactly the order of a tf.js
LayersModel's ``trainableWeights`` / ``weightsManifest`` (the reference relies on
``Object.keys`` order; here the order is explicit).  Consequences:

  * the gradient all-reduce is a single RCCL call on one buffer (or a few contiguous buckets,
    since backward produces gradients in reverse layer order = a growing suffix of the buffer);
  * the SGD update is one fused multi-tensor launch (``sgd_multi``) that also re-emits the bf16
    compute copies of every weight matrix in the two MFMA layouts ([N][K] and the dgrad layout),
    zero padded to 16 x 32 tiles;
  * serialisation (protocol / checkpoints) is a view of one buffer.

Matrix parameters use the layout [N][T*Ci] (dense: [out][in]; conv: OHWI = [Cout][KH*KW*Cin]).
Keras/tf.js layouts ([in][out], HWIO) are converted at the checkpoint boundary only.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Optional

import torch

from .. import native

SGD_ELEMS_PER_BLOCK = 1024


def _r(a, b):
    return (a + b - 1) // b * b


def primary_kpad(spec: "ParamSpec") -> int:
    """Row length of the primary bf16 copy: round32(K), or for the row-segment layout
    (csrc/optim.hip, csrc/convpool.hip) round32(KH * round8(KW*Cp))."""
    N, T, Ci = spec.mat
    if spec.row_pad:
        cp = spec.row_cp or Ci
        return _r((T // spec.row_pad) * _r((spec.row_pad + (1 if spec.row_pair else 0)) * cp, 8), 32)
    return _r(T * Ci, 32)


def dgrad_shape(spec: "ParamSpec") -> tuple:
    """Shape of the bf16 dgrad copy: [round16(Ci)][round32(T*N)], or for the pair layout of the fused
    conv+pool data gradient (csrc/convpool.hip make_dgrad) [16][round32(KH*(KW+1)*N)]."""
    N, T, Ci = spec.mat
    if spec.t_pair:
        kw = spec.row_pad
        return 16, _r((T // kw) * (kw + 1) * N, 32)
    return _r(Ci, 16), _r(T * N, 32)


@dataclass
class ParamSpec:
    name: str
    shape: tuple                    # master (engine) layout
    kind: str = "vector"            # "matrix" | "vector"
    mat: tuple = (0, 0, 0)          # (N, T, Ci) for matrices
    init: str | Callable = "zeros"  # glorot_uniform | he_normal | zeros | ones | callable(tensor)
    fan: tuple = (1, 1)             # (fan_in, fan_out) for initialisers
    needs_dgrad: bool = True        # keep a bf16 dgrad-layout copy
    row_pad: int = 0                # KW > 0: primary bf16 copy in the fused conv+pool row-segment layout
    row_cp: int = 0                 #   ... with LDS channel stride Cp (>= Ci; 0 = Ci)
    row_pair: bool = False          #   ... pair layout: rows 8+n = row n shifted by one kernel column
    t_pair: bool = False            # dgrad copy in the conv+pool dgrad pair layout (needs row_pad, Ci <= 8)
    trainable: bool = True

    @property
    def numel(self) -> int:
        return int(math.prod(self.shape))


class ParamStore:
    def __init__(self, specs: list[ParamSpec], device, compute_bf16: bool, seed: int = 0):
        self.specs = list(specs)
        self.device = torch.device(device)
        self.compute_bf16 = compute_bf16 and self.device.type == "cuda"
        self.offsets: dict[str, int] = {}
        off = 0
        for s in self.specs:
            # 16-byte alignment of every tensor inside the flat buffers (vector loads)
            off = _r(off, 4)
            self.offsets[s.name] = off
            off += s.numel
        self.total = _r(off, 4)
        self.master = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        self.momentum: Optional[torch.Tensor] = None
        self._views = {s.name: self.master[self.offsets[s.name]: self.offsets[s.name] + s.numel].view(s.shape)
                       for s in self.specs}
        self._gviews = {s.name: self.grad[self.offsets[s.name]: self.offsets[s.name] + s.numel].view(s.shape)
                        for s in self.specs}
        self._spec = {s.name: s for s in self.specs}
        self.hyper = torch.zeros(5, dtype=torch.float32, device=self.device)
        self._hyper_host = None
        self._init_values(seed)
        if self.compute_bf16:
            self._build_compute_copies()
            self.refresh_compute()

    # ------------------------------------------------------------------ views
    def __getitem__(self, name) -> torch.Tensor:
        return self._views[name]

    def gradient(self, name) -> torch.Tensor:
        return self._gviews[name]

    def spec(self, name) -> ParamSpec:
        return self._spec[name]

    def names(self):
        return [s.name for s in self.specs]

    def weight(self, name) -> torch.Tensor:
        """Compute weights of a matrix param: GPU padded bf16 [Npad][Kpad]; CPU fp32 [N][K] view."""
        if self.compute_bf16:
            return self._wbf_views[name]
        s = self._spec[name]
        N, T, Ci = s.mat
        return self._views[name].view(N, T * Ci)

    def weight_t(self, name) -> Optional[torch.Tensor]:
        """dgrad-layout bf16 copy (GPU only): [Cipad][pad(T*N)] or the pair layout (dgrad_shape)."""
        if self.compute_bf16:
            return self._wbft_views.get(name)
        return None

    def grad_matrix(self, name) -> torch.Tensor:
        s = self._spec[name]
        N, T, Ci = s.mat
        return self._gviews[name].view(N, T * Ci)

    # ------------------------------------------------------------------ init
    def _init_values(self, seed):
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)
        for s in self.specs:
            v = torch.empty(s.shape, dtype=torch.float32)
            fan_in, fan_out = s.fan
            if callable(s.init):
                s.init(v)
            elif s.init == "zeros":
                v.zero_()
            elif s.init == "ones":
                v.fill_(1.0)
            elif s.init == "glorot_uniform":
                lim = math.sqrt(6.0 / (fan_in + fan_out))
                v.uniform_(-lim, lim, generator=g)
            elif s.init == "he_normal":
                v.normal_(0.0, math.sqrt(2.0 / fan_in), generator=g)
            elif s.init == "lecun_uniform":
                lim = math.sqrt(3.0 / fan_in)
                v.uniform_(-lim, lim, generator=g)
            else:
                raise ValueError(f"unknown initialiser {s.init!r}")
            self._views[s.name].copy_(v)

    # ------------------------------------------------------------------ bf16 compute copies
    def _build_compute_copies(self):
        descs = []
        boff = 0
        self._wbf_layout = {}
        block = 0
        for s in self.specs:
            bf_off = bft_off = -1
            N = T = Ci = 1
            if s.kind == "matrix":
                N, T, Ci = s.mat
                bf_off = boff
                boff += _r(N, 16) * primary_kpad(s)
                if s.needs_dgrad:
                    bft_off = boff
                    boff += math.prod(dgrad_shape(s))
                self._wbf_layout[s.name] = (bf_off, bft_off)
            if s.trainable or s.kind == "matrix":
                nblocks = (s.numel + SGD_ELEMS_PER_BLOCK - 1) // SGD_ELEMS_PER_BLOCK
                if s.kind == "vector":
                    N, T, Ci = 1, 1, s.numel
                # tile mode (csrc/optim.hip, pad bit 28): plain layouts with a dgrad copy get 32x32 tiles
                # whose transposed copy is written through LDS
                tile = s.kind == "matrix" and s.needs_dgrad and not s.row_pad and not s.t_pair
                if tile:
                    nblocks = ((N + 31) // 32) * ((T * Ci + 31) // 32)
                assert s.row_cp < (1 << 12), "row-segment channel stride must fit 12 bits"
                descs.append((self.offsets[s.name], bf_off, bft_off, s.numel, N, T, Ci, block,
                              0 if s.trainable else 1,
                              (s.row_pad | (s.row_cp << 16) | ((1 << 30) if s.row_pair else 0)
                               | ((1 << 29) if s.t_pair else 0) | ((1 << 28) if tile else 0))
                              if s.kind == "matrix" else 0))
                block += nblocks
        self.wbf = torch.zeros(max(boff, 8), dtype=torch.bfloat16, device=self.device)
        self._wbf_views = {}
        self._wbft_views = {}
        for s in self.specs:
            if s.kind != "matrix":
                continue
            N, T, Ci = s.mat
            K = T * Ci
            bf_off, bft_off = self._wbf_layout[s.name]
            kp = primary_kpad(s)
            self._wbf_views[s.name] = self.wbf[bf_off: bf_off + _r(N, 16) * kp].view(_r(N, 16), kp)
            if bft_off >= 0:
                shp = dgrad_shape(s)
                self._wbft_views[s.name] = self.wbf[bft_off: bft_off + math.prod(shp)].view(*shp)
        # ParamDesc = {i64 off, i64 bf_off, i64 bft_off, i32 numel, i32 N, i32 T, i32 Ci, i32 block_start, i32 pad}
        raw = []
        frozen = []
        for (off, bf, bft, numel, N, T, Ci, bstart, frz, rpad) in descs:
            raw += [off, bf, bft, (numel & 0xFFFFFFFF) | (N << 32), (T & 0xFFFFFFFF) | (Ci << 32),
                    (bstart & 0xFFFFFFFF) | (rpad << 32)]
            frozen.append(frz)
        self._descs_host = torch.tensor(raw, dtype=torch.int64)
        self._descs = self._descs_host.to(self.device)
        self._ndesc = len(descs)
        self._sgd_blocks = block
        if any(frozen):
            raise NotImplementedError("non-trainable matrix parameters are not supported yet")

    # fused LeNet-5 (csrc/lenet_fused.hip): (frag buffer, conv1 kernel offset, conv2 kernel offset).  The
    # optimizer launch rebuilds the conv-weight MFMA fragments of the next step from the pre-update
    # snapshot ``lenet_snap`` the step's reduce kernel took.  ``lenet_state``: "fresh" = fragments match
    # the master; "snap" = also a snapshot of the current master / momentum exists (a fused step ran);
    # "stale" = the master changed without a rebuild (the next fused step launches its prep kernel).
    lenet_frag = None
    lenet_snap = None
    lenet_state = "stale"

    def _frag_kw(self, update: bool) -> dict:
        if self.lenet_frag is None:
            return {}
        if update and self.lenet_state != "snap":
            self.lenet_state = "stale"  # gradient not from a fused step: no snapshot to rebuild from
            return {}
        buf, o1, o2 = self.lenet_frag
        self.lenet_state = "fresh"
        kw = {"lenet_frag": buf, "frag_w1": int(o1), "frag_w2": int(o2)}
        if update:
            kw["lenet_snap"] = self.lenet_snap
        return kw

    def lenet_conv_momentum(self) -> list:
        """Momentum views of the two conv kernels (for the fused step's snapshot); [] without momentum."""
        if self.momentum is None or self.lenet_frag is None:
            return []
        _, o1, o2 = self.lenet_frag
        return [self.momentum[o1: o1 + 150], self.momentum[o2: o2 + 2400]]

    def refresh_compute(self):
        """Re-emit the bf16 compute copies from the fp32 master (after init / set_vars / load)."""
        if not self.compute_bf16:
            return
        native.require().sgd_multi(self._descs, self._ndesc, self._sgd_blocks, self.master, self.grad, None,
                                   self.wbf, self.hyper, False, descs_host=self._descs_host, **self._frag_kw(False))

    # ------------------------------------------------------------------ optimiser
    def set_hyper(self, lr, momentum=0.0, weight_decay=0.0, grad_scale=1.0, nesterov=False):
        h = (float(lr), float(momentum), float(weight_decay), float(grad_scale), 1.0 if nesterov else 0.0)
        if h != self._hyper_host:
            self.hyper.copy_(torch.tensor(h, dtype=torch.float32), non_blocking=False)
            self._hyper_host = h
        if momentum != 0.0 and self.momentum is None:
            self.momentum = torch.zeros_like(self.master)

    def sgd_step(self, index_stream=None, run_stats=None, ps_gate: int = 0, ps_mirror: int = 0):
        """w -= lr * (grad_scale * g [+ wd w]) (momentum optional); uses the device-side hyper tensor.
        ``index_stream = (stream [nsteps][B], cursor [1], dst [B])`` (GPU): the same launch stages the
        next step's batch indices into ``dst`` and advances ``cursor`` (csrc/optim.hip).
        ``run_stats = (step_stats [2], run [3])``: that workgroup also accumulates the step's
        [loss sum, correct] and counts the update (device run statistics, no extra launch).
        ``ps_gate`` / ``ps_mirror`` (device addresses, async PS with one rank: PSComm.excl_gate / excl_mirror):
        the update runs only if the admission word says accepted, and the new weights are also written to
        the parameter server's shard."""
        if self.compute_bf16:
            src, cur, dst = index_stream if index_stream is not None else (None, None, None)
            kw = self._frag_kw(True)
            if run_stats is not None:
                kw.update(step_stats=run_stats[0], run_stats=run_stats[1])
            if ps_gate:
                kw.update(gate=int(ps_gate), mirror=int(ps_mirror))
            native.require().sgd_multi(self._descs, self._ndesc, self._sgd_blocks, self.master, self.grad,
                                       self.momentum, self.wbf, self.hyper, True, src, cur, dst,
                                       self._descs_host, **kw)
            return
        if index_stream is not None:
            src, cur, dst = index_stream
            nxt = (int(cur[0]) + 1) % src.shape[0]
            dst.copy_(src[nxt])
            cur.fill_(nxt)
        if run_stats is not None:
            run_stats[1][:2] += run_stats[0][:2]
            run_stats[1][2] += 1.0
        lr, mom, wd, gs, nest = self._hyper_host
        if not hasattr(self, "_valid"):
            self._valid = torch.zeros(self.total, dtype=torch.bool, device=self.device)
            for s in self.specs:
                self._valid[self.offsets[s.name]: self.offsets[s.name] + s.numel] = True
        g = torch.where(self._valid, self.grad * gs, torch.zeros((), device=self.device))
        if wd:
            g = g + wd * self.master
        if mom:
            self.momentum.mul_(mom).add_(g)
            g = g + mom * self.momentum if nest else self.momentum
        self.master.sub_(lr * g)

    def apply_delta(self, delta: torch.Tensor, lr: float):
        """master -= lr * delta  (server-side update with an already-aggregated gradient)."""
        self.master.sub_(delta * lr)
        self.refresh_compute()

    # ------------------------------------------------------------------ (de)serialisation
    def get_vars(self) -> list[torch.Tensor]:
        return [self._views[s.name] for s in self.specs]

    def set_vars(self, values):
        for s, v in zip(self.specs, values):
            self._views[s.name].copy_(torch.as_tensor(v).reshape(s.shape))
        self.refresh_compute()

    def set_flat(self, flat: torch.Tensor):
        self.master.copy_(flat.reshape(-1)[: self.total])
        self.refresh_compute()
