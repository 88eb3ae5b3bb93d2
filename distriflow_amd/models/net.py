"""The model executor: a sequential layer graph with explicit forward/backward on preallocated
buffers, a flat parameter store, and hipGraph capture of the whole training step.

This is the engine behind ``DistriModel.fit`` / ``update`` (reference: DistributedTfModel.fit =
``tf.variableGrads(softmaxCE(predictOnBatch(x), y).mean())`` and update = per-tensor ``w -= lr*g``,
/root/reference/src/common/models.ts:128-142).  Deliberate differences:
the loss is a correct, fused softmax-cross-entropy on pre-softmax logits, and a trailing softmax
activation is folded into it rather than executed.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

import os

import torch

from .. import ops
from ..diagnostics import on as diag_on
from .layers import (Activation, BatchNorm, Conv2D, ConvPoolGemm, Dense, Dropout, Flatten, FusedConvPool,
                     KerasConvBlock, Layer, MaxPooling2D,
                     ResidualBlock)
from .params import ParamStore


@dataclass
class Workspace:
    wgrad: torch.Tensor   # fp32 split-m slabs for weight gradients
    bn: torch.Tensor      # fp32 BN partial sums


class Net:
    def __init__(self, layers: list[Layer], input_shape: tuple, num_classes: Optional[int] = None,
                 device="cuda", name: str = "model", seed: int = 0, compute_dtype: Optional[torch.dtype] = None,
                 fuse: bool = True):
        self.name = name
        self.device = torch.device(device)
        self.input_shape = tuple(input_shape)
        self.layers_all = list(layers)
        self.is_gpu = self.device.type == "cuda"
        self.dtype = compute_dtype or (torch.bfloat16 if self.is_gpu else torch.float32)
        self.fuse = fuse
        self._plan()
        specs = []
        for l in self.exec_layers:
            specs += l.specs()
        self.store = ParamStore(specs, self.device, compute_bf16=self.is_gpu, seed=seed)
        if self.lenet_fused:
            # the optimizer launch rebuilds the fused step's conv-weight fragments (no prep launch per step)
            c1, c2 = self.exec_layers[0], self.exec_layers[1]
            frag = torch.zeros(ops.lenet_frag_bytes(), dtype=torch.uint8, device=self.device)
            self.store.lenet_frag = (frag, self.store.offsets[f"{c1.name}/kernel"],
                                     self.store.offsets[f"{c2.name}/kernel"])
            self.store.lenet_snap = torch.zeros(2 * 2550, dtype=torch.float32, device=self.device)
            self.store.refresh_compute()
        for l in self.exec_layers:
            if hasattr(l, "bind_store"):  # composite layers: ResidualBlock, GraphLayer
                l.bind_store(self.store)
            else:
                l.store = self.store
        self.num_classes = num_classes or self.output_shape[-1]
        self.step_dev = torch.zeros((), dtype=torch.int64, device=self.device)
        self.has_dropout = False
        for l in self._all_leaf_layers():
            for d in (l, l.drop):
                if isinstance(d, Dropout):
                    d.step_dev = self.step_dev
                    self.has_dropout = True
        self._gather_step = None  # dropout step counter advanced by the step's gather launch
        self._bound_B = None
        self.graphs: dict = {}
        # side streams for weight gradients that run concurrently with the data-gradient chain
        # measured: cross-stream joins cost more than the overlap wins (LeNet-5); DISTRIFLOW_DIAG=concurrent_backward=1 on
        self.concurrent_backward = diag_on("concurrent_backward")
        self._side = [torch.cuda.Stream(device=self.device) for _ in range(3)] if self.is_gpu else []

    # ------------------------------------------------------------------ planning / fusion
    @property
    def final_softmax(self) -> bool:
        return self.final_act == "softmax"

    def _plan(self):
        shape = self.input_shape
        execd: list[Layer] = []
        # a Dense / Conv2D activation other than relu / linear runs as its own streaming launch right after
        # the GEMM, unless it ends the model (softmax / sigmoid fold into the loss)
        pending = []
        for j, l in enumerate(self.layers_all):
            pending.append(l)
            act = getattr(l, "activation", None) if isinstance(l, (Dense, Conv2D)) else None
            last = j == len(self.layers_all) - 1
            if act not in (None, "linear", "relu") and not (last and act in ("softmax", "sigmoid")):
                if act == "softmax":
                    raise NotImplementedError("a softmax activation is only supported on the output layer")
                pending.append(Activation(act, name=f"{l.name}/{act}", implicit=True))
        i = 0
        self.final_act = "linear"  # what the model applies to the logits: linear | softmax | sigmoid
        while i < len(pending):
            l = pending[i]
            shape = l.build(shape)
            if isinstance(l, Flatten):
                i += 1
                continue
            if isinstance(l, Activation):
                act = l.activation
                prev = execd[-1] if execd else None
                if act in ("linear", None):
                    pass
                elif act == "relu" and prev is not None and prev.can_fuse_relu() and not prev.relu:
                    prev.relu = True  # fused into the producer's epilogue (config() keeps the Keras view)
                elif act in ("softmax", "sigmoid") and i == len(pending) - 1:
                    self.final_act = act  # folded into the training loss / applied by predict()
                elif act == "softmax":
                    raise NotImplementedError("a softmax activation is only supported on the output layer")
                else:
                    execd.append(l)  # its own launch (csrc/act.hip)
                i += 1
                continue
            execd.append(l)
            i += 1
        if not execd:
            raise ValueError("empty model")
        if self.fuse:
            execd = self._fuse_conv_pool(execd)
            if (self.is_gpu and len(execd) >= 2 and isinstance(execd[1], ConvPoolGemm) and ops.kcnn_supported()
                    and diag_on("kcnn_fused")
                    and KerasConvBlock.matches(execd[0], execd[1].conv)):
                execd = [KerasConvBlock(execd[0], execd[1].conv, execd[1].pool)] + execd[2:]
        last = execd[-1]
        if isinstance(last, Dense):
            if last.activation in ("softmax", "sigmoid"):
                self.final_act = last.activation
            last.out_f32 = True
            if last.relu:
                raise ValueError("the logits layer must not end in ReLU")
        else:
            raise NotImplementedError("the last executed layer must be Dense (logits)")
        # relu' bookkeeping + first-layer dgrad elision
        for j, l in enumerate(execd):
            l.need_dx = j > 0
            l.in_relu = j > 0 and execd[j - 1].relu
        # a ReLU producer whose consumer applies relu' of its input receives an already masked gradient:
        # its own backward can skip re-reading its output as the mask (ResNet blocks / BatchNorm+ReLU)
        for j, l in enumerate(execd):
            l.grad_premasked = bool(l.relu and j + 1 < len(execd) and execd[j + 1].in_relu)
        if self.fuse and self.is_gpu and diag_on("fold_dropout"):
            execd = self._fold_dropout(execd)
        # BatchNorm sums accumulated by their producers' epilogues (csrc/bn_acc.h): the conv that feeds a
        # BatchNorm in the chain, and the layer whose data gradient IS the output gradient of the previous
        # layer's BatchNorms (relu' applied by that data gradient's mask: ResNet blocks, the GAP)
        for j, l in enumerate(execd):
            l.dx_bn_sinks = []
            if isinstance(l, Conv2D) and j + 1 < len(execd) and isinstance(execd[j + 1], BatchNorm):
                l.fwd_bn = execd[j + 1]
            if j == 0 or not l.in_relu:
                continue
            prev = execd[j - 1]
            if isinstance(prev, ResidualBlock):
                l.dx_bn_sinks = [prev.bn2] + ([prev.proj_bn] if prev.proj is not None else [])
            elif isinstance(prev, BatchNorm) and prev.relu and prev.grad_premasked:
                l.dx_bn_sinks = [prev]
        self.exec_layers = execd
        self.output_shape = shape
        self.head_start = self._plan_head(execd) if self.fuse else None
        self.khead = self._plan_khead(execd) if self.fuse else False
        if self.khead:
            self.head_start = len(execd) - 2
        self.lenet_fused = self._plan_lenet(execd) if self.fuse else False

    def _plan_lenet(self, execd) -> bool:
        """True when the executed graph is exactly LeNet-5 (conv5x5x6 'same' + relu + pool, conv5x5x16 +
        relu + pool, dense 120 relu, 84 relu, 10) on the GPU: the whole training step then runs as
        two launches (csrc/lenet_fused.hip).  ``DISTRIFLOW_DIAG=lenet_fused=0`` keeps the per-layer kernels."""
        import os

        if not self.is_gpu or not diag_on("lenet_fused") or not ops.lenet_supported():
            return False
        if self.final_act == "sigmoid":  # the fused kernel trains softmax cross-entropy
            return False
        if self.input_shape != (28, 28, 1) or len(execd) != 5:
            return False
        c1, c2, d1, d2, d3 = execd
        if not (isinstance(c1, FusedConvPool) and isinstance(c2, FusedConvPool)):
            return False
        convs_ok = all(c.conv.use_bias and c.conv.k == 5 and c.conv.stride == 1 for c in (c1, c2))
        convs_ok = convs_ok and c1.conv.filters == 6 and c1.conv.pad == 2 and c1.in_shape == (28, 28, 1)
        convs_ok = convs_ok and c2.conv.filters == 16 and c2.conv.pad == 0 and c2.in_shape == (14, 14, 6)
        dense = (d1, d2, d3)
        if not convs_ok or not all(isinstance(d, Dense) and d.use_bias for d in dense):
            return False
        return ((d1.in_features, d1.units, d2.units, d3.units) == (400, 120, 84, 10) and d1.relu and d2.relu
                and not d3.relu)

    def _plan_head(self, execd):
        """Index of the first layer of the trailing Dense chain trained by the fused head kernels
        (csrc/mlphead.hip), or None.  Conditions: <= 4 Dense layers, ReLU on all but the logits layer,
        <= 16 classes, hidden widths <= 256, input width a multiple of 8 and <= 1024."""
        if not self.is_gpu or not ops.head_supported() or self.final_act == "sigmoid":
            return None
        j0 = len(execd)
        while j0 > 0 and isinstance(execd[j0 - 1], Dense) and len(execd) - j0 < 4:
            j0 -= 1
        for j in range(j0, len(execd)):  # the longest trailing chain the head kernels can take
            head = execd[j:]
            if head[-1].units > 16 or head[-1].relu:
                return None
            if any(not l.relu for l in head[:-1]) or any(l.units > 256 for l in head[:-1]):
                continue
            if any(l.drop is not None for l in head):  # a folded dropout inside the chain
                continue
            if head[0].in_features % 8 or head[0].in_features > 1024:
                continue
            return j
        return None

    def _plan_khead(self, execd) -> bool:
        """True when the graph ends in the reference CNN's dense head -- Dense(K -> 128, ReLU) [+ folded
        Dropout] -> Dense(128 -> C <= 16) logits with softmax-CE, K a multiple of 256 -- on the GPU: the
        head's forward, loss and both data gradients then run as ONE split-K launch (csrc/khead.hip) and
        its weight gradients as the fused head weight-gradient launch.  ``DISTRIFLOW_DIAG=khead_fused=0``
        keeps the per-layer path."""
        if not self.is_gpu or not diag_on("khead_fused") or self.final_act == "sigmoid" or len(execd) < 3:
            return False
        d1, d2 = execd[-2], execd[-1]
        if not (isinstance(d1, Dense) and isinstance(d2, Dense)):
            return False
        if not (d1.relu and d1.units == 128 and not d1.out_f32 and d2.drop is None and not d2.relu):
            return False
        if d1.drop is not None and not d2.in_relu:
            return False
        return d2.units <= 16 and d1.need_dx and ops.khead_supported(d1.in_features, d2.units)

    @staticmethod
    def _fold_dropout(execd):
        """Fold each Dropout into its producer's epilogue (Dense+ReLU: igemm epilogues; MaxPooling2D over
        a ReLU output: the pool kernel) when a Dense consumes it.  Forward: the producer writes
        x * keep / (1 - p).  Backward: the kept elements are exactly those where the folded output is
        > 0 (the producer's output is a ReLU output), so the consumer's data gradient takes relu' of its
        own input plus the 1/(1-p) scale, and no dropout launch remains in either direction."""
        out = []
        i = 0
        while i < len(execd):
            l = execd[i]
            prev = out[-1] if out else None
            nxt = execd[i + 1] if i + 1 < len(execd) else None
            if (isinstance(l, Dropout) and l.rate > 0 and prev is not None and prev.drop is None
                    and isinstance(nxt, Dense)
                    and ((isinstance(prev, Dense) and prev.relu and not prev.out_f32)
                         or (isinstance(prev, MaxPooling2D) and prev.in_relu)
                         or (isinstance(prev, ConvPoolGemm) and prev.conv.relu)
                         or isinstance(prev, KerasConvBlock))):
                prev.drop = l
                nxt.in_relu = True
                nxt.dx_scale = 1.0 / (1.0 - l.rate)
                i += 1
                continue
            out.append(l)
            i += 1
        return out

    @staticmethod
    def _fuse_conv_pool(execd):
        out = []
        i = 0
        while i < len(execd):
            l = execd[i]
            nxt = execd[i + 1] if i + 1 < len(execd) else None
            if (isinstance(l, Conv2D) and isinstance(nxt, MaxPooling2D) and l.relu and l.regular and l.stride == 1
                    and nxt.p == 2
                    and l.out_shape[0] % 2 == 0 and l.out_shape[1] % 2 == 0
                    and ops.convpool_supported(l.in_shape[0], l.in_shape[1], l.in_shape[2], l.k, l.k, l.pad,
                                               l.filters)):
                out.append(FusedConvPool(l, nxt))
                i += 2
                continue
            if (isinstance(l, Conv2D) and isinstance(nxt, MaxPooling2D) and l.relu and l.regular and l.stride == 1
                    and nxt.p == 2
                    and l.out_shape[0] % 2 == 0 and l.out_shape[1] % 2 == 0
                    and ops.conv_pool_supported(l.in_shape[0], l.in_shape[1], l.in_shape[2], l.k, l.k, l.stride,
                                                l.pad, l.filters)):
                out.append(ConvPoolGemm(l, nxt))
                i += 2
                continue
            out.append(l)
            i += 1
        return out

    def _all_leaf_layers(self):
        for l in self.exec_layers:
            if hasattr(l, "sublayers"):  # composite layers: ResidualBlock, GraphLayer
                yield from l.sublayers()
            else:
                yield l

    # ------------------------------------------------------------------ buffers
    def bind(self, B: int):
        if self._bound_B == B:
            return
        # split-m weight-gradient slabs: room for 4 slabs of the largest conv kernel (>= 16 MB)
        convs = [c for l in self._all_leaf_layers()
                 for c in ((l.conv,) if isinstance(l, ConvPoolGemm) else
                           (l.conv1, l.conv2) if isinstance(l, KerasConvBlock) else (l,))]
        nk = max([l.filters * l.kh * l.kw * l.in_shape[2] for l in convs if isinstance(l, Conv2D)]
                 + [0])
        ws_wgrad = torch.empty(max(1 << 22, 4 * nk), dtype=torch.float32, device=self.device)
        maxC = max([l.C for l in self._all_leaf_layers() if isinstance(l, BatchNorm)] + [8])
        ws_bn = torch.empty(ops.bn_workspace_floats(maxC), dtype=torch.float32, device=self.device)
        self.ws = Workspace(ws_wgrad, ws_bn)
        for l in self.exec_layers:
            l.alloc(B, self.device, self.dtype, self.ws)
        self.dlogits = torch.empty((B, self.num_classes), dtype=self.dtype, device=self.device)
        self.stats = torch.zeros(2, dtype=torch.float32, device=self.device)
        self.x_buf = torch.empty((B,) + self.input_shape, dtype=self.dtype, device=self.device)
        self.y_buf = torch.empty((B,), dtype=torch.int32, device=self.device)
        if self.head_start is not None:
            ldt = (B + 31) // 32 * 32  # transposed activation / gradient buffers, zero tail columns
            if self.lenet_fused:
                # row stride 256 B past a multiple of 8 KB: the 16 rows of one MFMA operand load land on
                # 16 different L2 channels instead of one (csrc/lenet_fused.hip dense_unit_value)
                ldt += 128
            head = self.exec_layers[self.head_start:]
            z = lambda *shape: torch.zeros(shape, dtype=self.dtype, device=self.device)  # noqa: E731
            self.head_xT = z(head[0].in_features, ldt)
            self.head_hT = [z(l.units, ldt) for l in head[:-1]] + [None]
            self.head_dzT = [z(l.units, ldt) for l in head]
            self.head_loss_part = torch.zeros(2 * ((B + 15) // 16), dtype=torch.float32, device=self.device)
            if self.khead:  # split-K slabs, published dZ1 tiles, tickets / flags / launch tag (zeroed)
                self.khead_ws = torch.zeros(ops.khead_ws_floats(B, head[0].in_features), dtype=torch.float32,
                                            device=self.device)
        if self.lenet_fused:
            nblk = ops.lenet_blocks(B)
            self.lenet_conv_part = torch.empty(2576 * nblk, dtype=torch.float32, device=self.device)
            # reduce-launch scratch: job partial slabs + arrival tickets (must start zeroed)
            self.lenet_dense_part = torch.zeros(ops.lenet_dense_part_floats(B), dtype=torch.float32,
                                                device=self.device)
            self.lenet_loss_part = torch.zeros(2 * nblk, dtype=torch.float32, device=self.device)
        self._bound_B = B
        self.graphs = {}

    # ------------------------------------------------------------------ compute
    _bn_acc_dirty = False

    def _bn_acc_begin(self):
        """A training forward starts.  The BatchNorm accumulators are cleared by their consumers (each pass
        clears the other direction's), which holds for every forward followed by its backward; after a
        training forward whose backward never ran, clear them all first."""
        if self._bn_acc_dirty:
            for l in self._all_leaf_layers():
                if isinstance(l, BatchNorm) and getattr(l, "acc_on", False):
                    l.drop_acc()
        self._bn_acc_dirty = True

    def forward(self, x, training: bool = False) -> torch.Tensor:
        """Returns fp32 logits [B][classes] (a view of an engine buffer).  ``x`` is a tensor or an
        :class:`ops.GatherRef` (rows of the HBM dataset; fused into the first layer when it can)."""
        self.bind(x.shape[0])
        if training:
            self._bn_acc_begin()
        if isinstance(x, ops.GatherRef) and not isinstance(self.exec_layers[0], (FusedConvPool, KerasConvBlock)):
            x = x.materialise(self.x_buf, step_inc=self._take_gather_step())
        h = x
        for l in self.exec_layers:
            h = l.forward(h, training)
        return h

    def _take_gather_step(self):
        s, self._gather_step = self._gather_step, None
        return s

    def backward(self, dlogits: torch.Tensor, grad_ready: Optional[Callable[[int], None]] = None):
        """Backprop dlogits; fills ``store.grad``.  ``grad_ready(i)`` fires after layer i's grads are final
        (reverse order) so a data-parallel wrapper can launch bucketed all-reduces early."""
        d = dlogits
        for i in range(len(self.exec_layers) - 1, -1, -1):
            d = self.exec_layers[i].backward(d)
            if grad_ready is not None:
                grad_ready(i)
        self._bn_acc_dirty = False

    # Scale of the per-example loss gradients: None = 1 / rows of the step (the mean loss).  A FedSGD step
    # over several microbatches per rank (DataParallelTrainer min_updates_per_version) sets 1 / microbatch
    # size, so the step's gradient is the SUM of its microbatches' mean-loss gradients.
    loss_scale: Optional[float] = None

    def _loss_scale(self, rows: int) -> float:
        return 1.0 / rows if self.loss_scale is None else float(self.loss_scale)

    def loss_and_grad(self, logits, labels, grad_scale: Optional[float] = None):
        """The training loss on the logits: softmax cross-entropy (a final softmax or linear output) or,
        for a model that ends in sigmoid, sigmoid cross-entropy against the one-hot labels."""
        B = logits.shape[0]
        self.stats.zero_()
        gs = self._loss_scale(B) if grad_scale is None else grad_scale
        if self.final_act == "sigmoid":
            ops.sigmoid_ce(logits, labels, self.dlogits, self.stats, gs)
        else:
            ops.softmax_ce(logits, labels, self.dlogits, self.stats, gs)
        return self.stats

    def compute_gradients(self, x, labels, grad_ready=None):
        """fwd + fused softmax-CE + bwd; returns the device stats tensor [loss_sum, correct].
        ``labels``: int tensor [B], or an :class:`ops.LabelRef` (dataset labels + batch indices)."""
        if not isinstance(x, ops.GatherRef) and x.dtype != self.dtype:
            x = x.to(self.dtype)
        if self.has_dropout and isinstance(self.exec_layers[0], KerasConvBlock):
            # advanced by the block's backward reduce, so this step's masks read step + 1 (the value
            # the other paths advance to before their step)
            self.exec_layers[0].step_inc = self.step_dev
            for l in self._all_leaf_layers():
                if l.drop is not None:
                    l.drop.step_add = 1
        elif self.has_dropout:
            if (self.is_gpu and isinstance(x, ops.GatherRef) and not self.lenet_fused
                    and not isinstance(self.exec_layers[0], (FusedConvPool, KerasConvBlock))):
                self._gather_step = self.step_dev  # advanced by the gather launch (no extra kernel)
            else:
                self.step_dev.add_(1)
        if self.lenet_fused:
            return self._compute_gradients_lenet(x, labels, grad_ready)
        if self.head_start is not None:
            return self._compute_gradients_head(x, labels, grad_ready)
        if isinstance(labels, ops.LabelRef):
            labels = labels.materialise(self.y_buf)
        if labels.dtype != torch.int32:
            labels = labels.to(torch.int32)
        logits = self.forward(x, training=True)
        stats = self.loss_and_grad(logits, labels)
        self.backward(self.dlogits, grad_ready)
        return stats

    def compute_gradients_and_update(self, x, labels, index_stream=None, ll=None, run_stats=None, ps=None):
        """Fused LeNet-5 step: gradients AND the SGD update (with the store's device hyper-parameters)
        in the step's two launches (the reduce kernel applies the update and rebuilds the next step's
        weight fragments; ``index_stream`` = (stream, cursor, dst) is advanced by it too).  Same
        arithmetic as compute_gradients + ParamStore.sgd_step.  ``ll``: a world > 1 native P2PComm —
        the reduce kernel then sums every gradient over the ranks in its epilogue (csrc/ll_exchange.h),
        so a data-parallel step is still two launches, equal to compute_gradients + all-reduce + SGD."""
        if not self.lenet_fused:
            raise RuntimeError("compute_gradients_and_update needs the fused LeNet-5 plan")
        if self.has_dropout:
            self.step_dev.add_(1)
        st = self.store
        sgd = dict(sgd_master=st.master, sgd_mom=st.momentum, sgd_wbf=st.wbf, sgd_hyper=st.hyper,
                   sgd_descs=st._descs_host)
        if index_stream is not None:
            sgd.update(idx_stream=index_stream[0], idx_cursor=index_stream[1], idx_dst=index_stream[2])
        if ll is not None:
            sgd["ll"] = ll
        if ll is not None or ps is not None:
            sgd["exch_blocks"] = int(getattr(self, "lenet_exch_blocks", 0))
        if run_stats is not None:
            sgd["run_stats"] = run_stats
        if ps is not None:
            # asynchronous SGD: the reduce launch applies the gradient to the parameter server's shared
            # master (dict: ps, ps_perm, ps_idx, ps_lr, ps_max_stale; parallel/async_ps.py)
            sgd.update(ps)
        stats = self._compute_gradients_lenet(x, labels, None, sgd=sgd)
        st.lenet_state = "fresh"  # the reduce kernel rebuilt the fragments from the new weights
        return stats

    def _compute_gradients_lenet(self, x, labels, grad_ready, sgd=None):
        """The whole LeNet-5 step in two launches (csrc/lenet_fused.hip); every gradient is final when
        they end, so all gradient hooks fire afterwards (one bucket's all-reduce)."""
        B = x.shape[0]
        self.bind(B)
        st = self.store
        c1, c2, d1, d2, d3 = self.exec_layers
        conv = [st[f"{c1.name}/kernel"], st[f"{c1.name}/bias"], st[f"{c2.name}/kernel"], st[f"{c2.name}/bias"]]
        cgrads = [st.gradient(f"{c1.name}/kernel"), st.gradient(f"{c1.name}/bias"),
                  st.gradient(f"{c2.name}/kernel"), st.gradient(f"{c2.name}/bias")]
        dense = (d1, d2, d3)
        ops.lenet_train(x, labels, conv, [st.weight(f"{d.name}/kernel") for d in dense],
                        [st.weight_t(f"{d.name}/kernel") for d in dense], [st[f"{d.name}/bias"] for d in dense],
                        cgrads, [st.grad_matrix(f"{d.name}/kernel") for d in dense],
                        [st.gradient(f"{d.name}/bias") for d in dense], [self.head_xT] + self.head_hT[:2],
                        self.head_dzT, self.lenet_conv_part, self.lenet_dense_part, self.lenet_loss_part, self.stats,
                        self._loss_scale(B), frag=st.lenet_frag[0] if st.lenet_frag is not None else None,
                        prep=st.lenet_frag is None or st.lenet_state == "stale", snap=st.lenet_snap,
                        conv_mom=st.lenet_conv_momentum(), sgd=sgd if st.lenet_frag is not None else None)
        if st.lenet_frag is not None:
            st.lenet_state = "snap"
        if grad_ready is not None:
            for i in range(len(self.exec_layers) - 1, -1, -1):
                grad_ready(i)
        return self.stats

    def _wgrad_side(self, layer):
        """Side stream for ``layer``'s weight gradients (ResNet blocks on the GPU), else None.  Off by
        default since the halo-tiled weight gradients (csrc/wgrad_halo.hip) fill whole CUs and the overlap
        then slows the data-gradient chain more than it hides; ``DISTRIFLOW_DIAG=wgrad_overlap=1`` turns it
        on."""
        if not isinstance(layer, ResidualBlock):
            return None
        on = self.is_gpu and diag_on("wgrad_overlap")
        return self._side[0] if on else None

    def _proj_side(self, layer):
        """Stream for a ResNet block's projection shortcut branch (joined inside the block), else None.
        Off by default (measured slower beside the halo-tiled kernels); ``DISTRIFLOW_DIAG=proj_overlap=1``
        turns it on."""
        if not (isinstance(layer, ResidualBlock) and layer.proj is not None and self.is_gpu):
            return None
        return self._side[1] if diag_on("proj_overlap") else None

    def _compute_gradients_head(self, x, labels, grad_ready):
        """Body layers one by one, then the fused dense head (2 launches: forward + CE + backward data
        chain, then all head weight gradients), then the body's backward from the head's dX."""
        self.bind(x.shape[0])
        self._bn_acc_begin()
        if isinstance(x, ops.GatherRef) and not isinstance(self.exec_layers[0], (FusedConvPool, KerasConvBlock)):
            x = x.materialise(self.x_buf, step_inc=self._take_gather_step())
        h = x
        for l in self.exec_layers[: self.head_start]:
            ps = self._proj_side(l)
            if ps is not None:
                l.proj_stream = ps  # only for this call (joined inside the block)
                try:
                    h = l.forward(h, True)
                finally:
                    l.proj_stream = None
            else:
                h = l.forward(h, True)
        head = self.exec_layers[self.head_start:]
        if isinstance(labels, ops.LabelRef):
            lab, idx = labels.labels, labels.idx
        else:
            lab, idx = (labels if labels.dtype == torch.int32 else labels.to(torch.int32)), None
        st = self.store
        first = head[0]
        args = dict(
            w=[st.weight(f"{l.name}/kernel") for l in head],
            wt=[st.weight_t(f"{l.name}/kernel") for l in head],
            b=[st[f"{l.name}/bias"] if l.use_bias else None for l in head],
            gw=[st.grad_matrix(f"{l.name}/kernel") for l in head],
            gb=[st.gradient(f"{l.name}/bias") if l.use_bias else None for l in head],
            hT=self.head_hT, dzT=self.head_dzT, K=[l.in_features for l in head], N=[l.units for l in head],
            x=h, x_relu=first.in_relu, dx_scale=first.dx_scale, xT=self.head_xT,
            dx=first.dx if first.need_dx else None,
            logits=head[-1].out, labels=lab, idx=idx, grad_scale=self._loss_scale(x.shape[0]),
            loss_part=self.head_loss_part, stats=self.stats)
        head_ids = range(len(self.exec_layers) - 1, self.head_start - 1, -1)
        if not self.concurrent_backward:
            self._head_launch(args, head, h, lab, idx, 3)
            if grad_ready is not None:
                for i in head_ids:
                    grad_ready(i)
            d = first.dx if first.need_dx else None
            # fused conv+pool weight gradients defer their split-m slab reductions; consecutive ones are
            # flushed in ONE launch right before the next gradient hook needs them (or at the end)
            pending, waiting = [], []
            side_used = False
            for i in range(self.head_start - 1, -1, -1):
                l = self.exec_layers[i]
                if isinstance(l, FusedConvPool) and self.is_gpu:
                    d = l.backward(d, defer=pending)
                    waiting.append(i)
                    continue
                if pending:
                    ops.flush_slab_reductions(pending)
                wside = self._wgrad_side(l)
                if side_used and (wside is None or grad_ready is not None):
                    # join the weight-gradient stream before a gradient hook or a layer that shares its
                    # workspace (the stem conv's wgrad) runs on the main stream
                    torch.cuda.current_stream(self.device).wait_stream(self._side[0])
                    side_used = False
                if wside is not None:
                    l.side_stream = wside  # only for this call: other backward paths run in order
                    l.proj_stream = self._proj_side(l)
                    try:
                        d = l.backward(d)
                    finally:
                        l.side_stream = l.proj_stream = None
                else:
                    d = l.backward(d)
                side_used = side_used or wside is not None
                if grad_ready is not None:
                    if side_used:
                        torch.cuda.current_stream(self.device).wait_stream(self._side[0])
                        side_used = False
                    for j in waiting + [i]:
                        grad_ready(j)
                waiting = []
            if pending:
                ops.flush_slab_reductions(pending)
            if side_used:
                torch.cuda.current_stream(self.device).wait_stream(self._side[0])
            if grad_ready is not None:
                for j in waiting:
                    grad_ready(j)
            self._bn_acc_dirty = False
            return self.stats
        # critical path on the main stream: head fwd/CE/bwd-data -> each body layer's data gradient;
        # weight gradients fork onto side streams as soon as their input gradient exists.  Gradient
        # hooks (bucketed all-reduce) fire after the join: a bucket spans layers whose gradients
        # complete on different streams.
        main = torch.cuda.current_stream(self.device)
        self._head_launch(args, head, h, lab, idx, 1)
        ev = main.record_event()
        side = self._side
        side[0].wait_event(ev)
        with torch.cuda.stream(side[0]):
            self._head_launch(args, head, h, lab, idx, 2)
        d = first.dx if first.need_dx else None
        k = 1
        for i in range(self.head_start - 1, -1, -1):
            l = self.exec_layers[i]
            if l.split_backward:
                s = side[k]
                k = 1 + (k % (len(side) - 1))
                s.wait_event(main.record_event())
                with torch.cuda.stream(s):
                    l.backward_weights(d)
                d = l.backward_data(d)
            else:
                d = l.backward(d)
        for s in side:
            main.wait_stream(s)
        if grad_ready is not None:
            for i in range(len(self.exec_layers) - 1, -1, -1):
                grad_ready(i)
        self._bn_acc_dirty = False
        return self.stats

    def _head_launch(self, args, head, x, labels, idx, phases):
        """The dense head's launches: bit 1 forward + loss + data gradients, bit 2 weight gradients +
        stats (csrc/mlphead.hip; the reference CNN's head: csrc/khead.hip)."""
        if not self.khead:
            ops.head_train(**args, phases=phases)
            return
        if phases & 1:
            st = self.store
            d1, d2 = head
            ops.khead_train(x, self.head_xT, d1.dx, st.weight(f"{d1.name}/kernel"), st.weight_t(f"{d1.name}/kernel"),
                            st[f"{d1.name}/bias"] if d1.use_bias else None, st.weight(f"{d2.name}/kernel"),
                            st.weight_t(f"{d2.name}/kernel"), st[f"{d2.name}/bias"] if d2.use_bias else None,
                            self.head_hT[0], self.head_dzT[0], self.head_dzT[1], d2.out, labels, idx,
                            args["grad_scale"], self.head_loss_part, self.khead_ws, drop=d1.drop_spec(True),
                            dh_scale=d2.dx_scale, dp_scale=d1.dx_scale, dp_mask=d1.in_relu)
        if phases & 2:
            st = self.store
            d1, d2 = head
            ops.khead_wgrad(self.head_xT, self.head_hT[0], self.head_dzT[0], self.head_dzT[1],
                            st.grad_matrix(f"{d1.name}/kernel"),
                            st.gradient(f"{d1.name}/bias") if d1.use_bias else None,
                            st.grad_matrix(f"{d2.name}/kernel"),
                            st.gradient(f"{d2.name}/bias") if d2.use_bias else None,
                            x.shape[0], d1.in_features, d2.units, self.head_loss_part, self.stats)

    @torch.no_grad()
    def evaluate(self, x, labels, batch_size: int = 4096):
        """-> (mean loss, accuracy) over the given examples (inference mode, chunked)."""
        n = x.shape[0]
        loss = 0.0
        correct = 0.0
        for s in range(0, n, batch_size):
            xb = x[s: s + batch_size].to(self.device, self.dtype)
            yb = labels[s: s + batch_size].to(self.device, torch.int32)
            logits = self._forward_eval(xb)
            st = torch.zeros(2, dtype=torch.float32, device=self.device)
            if self.final_act == "sigmoid":
                ops.sigmoid_ce(logits, yb, None, st, 1.0)
            else:
                ops.softmax_ce(logits, yb, None, st, 1.0)
            loss += float(st[0])
            correct += float(st[1])
        return loss / max(n, 1), correct / max(n, 1)

    def _forward_eval(self, xb):
        """Logits for any batch size WITHOUT rebinding: a bound engine (whose buffers a captured
        hipGraph may reference) runs the batch in chunks of its bound size, padding the tail."""
        B = xb.shape[0]
        if self._bound_B is None:
            self.bind(B)
        bb = self._bound_B
        if B == bb:
            return self.forward(xb, training=False).clone()
        outs = []
        for s in range(0, B, bb):
            chunk = xb[s: s + bb]
            n = chunk.shape[0]
            if n < bb:
                chunk = torch.cat([chunk, chunk.new_zeros((bb - n,) + tuple(chunk.shape[1:]))])
            outs.append(self.forward(chunk, training=False)[:n].clone())
        return torch.cat(outs)

    @torch.no_grad()
    def predict(self, x, batch_size: int = 4096) -> torch.Tensor:
        outs = []
        for s in range(0, x.shape[0], batch_size):
            xb = x[s: s + batch_size].to(self.device, self.dtype)
            z = self._forward_eval(xb)
            outs.append(torch.softmax(z, dim=1) if self.final_act == "softmax" else
                        torch.sigmoid(z) if self.final_act == "sigmoid" else z)
        return torch.cat(outs)

    # ------------------------------------------------------------------ mutable state
    def state_tensors(self) -> list:
        """Every tensor a training step mutates besides gradients/activations: master weights,
        optimizer state, BN running statistics, the dropout step counter."""
        out = [self.store.master, self.step_dev]
        if self.store.momentum is not None:
            out.append(self.store.momentum)
        for l in self._all_leaf_layers():
            if isinstance(l, BatchNorm) and hasattr(l, "run_mean"):
                out += [l.run_mean, l.run_var]
        return out

    def snapshot_state(self) -> list:
        return [t.clone() for t in self.state_tensors()]

    def restore_state(self, snap: list):
        for t, v in zip(self.state_tensors(), snap):
            t.copy_(v)
        self.store.refresh_compute()

    # ------------------------------------------------------------------ introspection
    def num_params(self) -> int:
        return sum(s.numel for s in self.store.specs)

    def summary(self) -> str:
        lines = [f"Net {self.name}: input {self.input_shape}, {self.num_params():,} params"]
        for l in self.exec_layers:
            lines.append(f"  {type(l).__name__:<22} {l.name:<24} {str(l.in_shape):<16} -> {str(l.out_shape):<16}"
                         f"{' +relu' if l.relu else ''}")
        return "\n".join(lines)

    def flops_per_example(self) -> int:
        """Training FLOPs per example (fwd + dgrad + wgrad of every GEMM-shaped layer)."""
        total = 0

        def layer_flops(l):
            if isinstance(l, Dense):
                f = 2 * l.in_features * l.units
                return f * (3 if l.need_dx else 2)
            if isinstance(l, (FusedConvPool, ConvPoolGemm)):
                c = l.conv
                OH, OW, N = c.out_shape
                f = 2 * OH * OW * N * c.kh * c.kw * c.in_shape[2]
                return f * (3 if l.need_dx else 2)
            if isinstance(l, Conv2D):
                OH, OW, N = l.out_shape
                f = 2 * OH * OW * N * l.kh * l.kw * l.in_shape[2]
                return f * (3 if l.need_dx else 2)
            return 0

        for l in self._all_leaf_layers():
            if isinstance(l, KerasConvBlock):
                total += layer_flops(l.conv1) + layer_flops(l.conv2)
                continue
            total += layer_flops(l)
        return total
