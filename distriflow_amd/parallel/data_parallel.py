"""Synchronous data-parallel SGD over RCCL / xGMI (BASELINE.json configs[1], the headline benchmark).

The reference's synchronous mode is a parameter server: K uploads of a gradient tagged with the
current version are stacked on the host, averaged and applied, then new weights are broadcast to
every client (/root/reference/src/server/federated_server.ts:71-117, client side
/root/reference/src/client/federated_client.ts:68-132).  On one MI355X node every rank is both
"server" and "worker": the K-way host-side stack+mean becomes ONE in-place RCCL all-reduce (SUM) of
the flat gradient buffer and the 1/world factor of the mean is folded into the fused SGD kernel,
so every rank applies the identical update and no weight broadcast is needed after step 0.

MI355X specifics:
  * gradient buckets are contiguous slices of the flat gradient buffer; a bucket's all-reduce is
    issued (async, on RCCL's stream) as soon as backward has produced its last gradient, so it
    overlaps the remaining backward kernels on the compute stream;
  * the whole step — batch gather from the HBM-resident dataset, forward, fused loss, backward,
    bucketed all-reduce, fused SGD — is captured into one hipGraph and replayed, removing all
    host launch overhead (``graph="full"``); ``"split"`` captures compute only and runs the
    all-reduce eagerly between two graphs, ``"none"`` is fully eager.
"""
from __future__ import annotations

import os
import time
from typing import Optional

import torch
import torch.distributed as dist

from .. import native, ops
from ..diagnostics import on as _diag_on


class DataParallelTrainer:
    def __init__(self, net, lr: float = 0.001, momentum: float = 0.0, weight_decay: float = 0.0,
                 group=None, bucket_mb: Optional[float] = None, overlap: bool = True, graph: str = "full",
                 broadcast_init: bool = True, allreduce: str = "auto", p2p_max_mb: float = 4.0,
                 min_updates_per_version: Optional[int] = None):
        self.net = net
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        # FedSGD count barrier on the device (reference FederatedServer: a version is the mean of
        # minUpdatesPerVersion microbatch gradients of the current version, federated_server.ts:73-90,
        # default 20, utils.ts:188-191).  K microbatches per version, split over the ranks as evenly as they
        # go (rank r takes K // W + (r < K % W) of them, as one step over their concatenated rows); every
        # row's loss gradient is scaled by 1 / (K * microbatch), the step sums them and the exchange sums
        # over the ranks: the mean of the K microbatch means.  Every gradient of a version is computed on that version, so the
        # reference's stale-upload drop never has anything to drop.  None: one microbatch per rank (K = W).
        self.min_updates = None if min_updates_per_version in (None, 0) else int(min_updates_per_version)
        if self.min_updates is not None and self.min_updates < self.world:
            raise ValueError(f"min_updates_per_version must be >= world ({self.world}), got {self.min_updates}")
        self.micro_per_rank = ([self.min_updates // self.world + (1 if r < self.min_updates % self.world else 0)
                                for r in range(self.world)] if self.min_updates is not None else [1] * self.world)
        self.lr, self.momentum, self.weight_decay = lr, momentum, weight_decay
        self.overlap = overlap
        self.graph_mode = graph if net.is_gpu else "none"
        # bucket size: small models still get >= 2 buckets (the head's gradient all-reduce then overlaps
        # the convolution backward); large ones use up to 32 MB (few, large RCCL calls over xGMI)
        total_bytes = net.store.total * 4
        if bucket_mb is None and getattr(net, "lenet_fused", False):
            # the fused LeNet-5 step produces every gradient at once: nothing to overlap, so ONE bucket
            # (one all-reduce launch over xGMI instead of several latency-bound ones), issued in stream
            # order after the reduction launch (no side-stream hop)
            self.bucket_bytes = total_bytes
            self.overlap = False
        elif bucket_mb is None:
            self.bucket_bytes = int(min(32 << 20, max(64 << 10, total_bytes // 4)))
        else:
            self.bucket_bytes = int(bucket_mb * (1 << 20))
        self._build_buckets()
        self._setup_p2p(allreduce, int(p2p_max_mb * (1 << 20)))
        # gloo cannot run inside a hipGraph capture (it stages device tensors through the host): with a
        # gloo process group on GPUs (the one-GPU rehearsal mode) any bucket that is not on the one-shot
        # p2p path makes the step "split" (compute graph, eager all-reduce, SGD graph) from the start
        if (self.world > 1 and self.net.is_gpu and self.graph_mode == "full" and self._step_all_reduces
                and dist.is_initialized()
                and dist.get_backend(self.group) == "gloo"
                and any(self.p2p is None or (hi - lo) * 4 > self.p2p_limit for _, lo, hi in self.buckets)):
            self.graph_mode = "split"
            self.capture_error = "gloo collectives are not capturable"
        self._works = []
        self._graph = None
        self._multi, self._multi_u = None, 0  # multi-step graph (prepare_run)
        self._graph_B = None
        self._index_stream = None
        self.preprocess_callbacks: list = []
        self.steps = 0
        # device run statistics [loss sum, correct, updates, -]: accumulated inside the step's own last
        # launch (no extra launch), read back asynchronously per replay when callbacks are registered
        self.run_stats = torch.zeros(4, dtype=torch.float32, device=net.device)
        self._version_cbs, self._upload_cbs = [], []
        self._cb_pending = []
        self._cb_ring = None
        self._cb_last = None
        if broadcast_init and self.world > 1:
            dist.broadcast(net.store.master, src=0, group=group)
            net.store.refresh_compute()
        net.store.set_hyper(lr, momentum, weight_decay, grad_scale=self._grad_scale())

    def _grad_scale(self) -> float:
        """The update's gradient scale: the mean over the ranks' gradients (1 / W).  A FedSGD version of K
        microbatches folds its 1 / K into the loss scale (bind_dataset), so the update takes the plain sum."""
        return 1.0 if self.min_updates is not None else 1.0 / self.world

    # ------------------------------------------------------------------ buckets
    def _build_buckets(self):
        net, store = self.net, self.net.store
        starts = []
        for i, l in enumerate(net.exec_layers):
            names = [s.name for s in l.specs()]
            if names:
                starts.append((i, min(store.offsets[n] for n in names)))
        self.buckets = []  # (trigger layer index, lo, hi)
        hi = store.total
        first_param_layer = starts[0][0] if starts else 0
        for i, lo in reversed(starts):
            if i == first_param_layer:
                self.buckets.append((i, 0, hi))
                break
            if (hi - lo) * 4 >= self.bucket_bytes:
                self.buckets.append((i, lo, hi))
                hi = lo
        self._trigger = {b[0]: b for b in self.buckets}

    def _setup_p2p(self, mode: str, limit_bytes: int):
        """Pick the transport per bucket: the one-shot xGMI kernel (parallel/p2p.py) for buckets up to
        ``limit_bytes``, RCCL above.  ``mode``: auto (p2p when usable) | p2p (required) | rccl."""
        self.p2p = None
        self.p2p_limit = limit_bytes
        self.p2p_reason = "single rank" if self.world == 1 else ("cpu" if not self.net.is_gpu else "")
        if mode not in ("auto", "p2p", "rccl"):
            raise ValueError(f"allreduce must be auto|p2p|rccl, got {mode!r}")
        if self.world == 1 or not self.net.is_gpu or mode == "rccl":
            self.p2p_reason = self.p2p_reason or "disabled"
            return
        sizes = [(hi - lo) * 4 for _, lo, hi in self.buckets] + [self.net.store.total * 4]
        small = [s for s in sizes if s <= limit_bytes]
        if not small:
            self.p2p_reason = "all buckets above the p2p limit"
            return
        from .p2p import make_p2p

        self.p2p = make_p2p(self.group, max_bytes=max(small))
        if self.p2p is None:
            self.p2p_reason = "unavailable (self-test or IPC failed, or DISTRIFLOW_ALLREDUCE=rccl)"
            if mode == "p2p":
                raise RuntimeError("allreduce='p2p' requested but the one-shot path is unusable")
        else:
            self._comm_stream = torch.cuda.Stream(device=self.net.device)
            self._p2p_pending = False
            # ranks that time-share one GPU (rehearsals): the fused LeNet-5 reduce runs fewer exchanging
            # workgroups (each owning several slots) so that every rank's waiting workgroups fit on the chip
            # beside the peers' train kernels; with one rank per GPU every slot gets its own workgroup
            self.net.lenet_exch_blocks = shared_gpu_exch_blocks(self.world)
            # likewise the reference CNN's persistent dense-head grid (csrc/khead.hip): its share of the CUs
            native.require().khead_set_grid_cap(shared_gpu_cus(self.world))

    def _reduce(self, t: torch.Tensor, async_op: bool):
        if self.p2p is not None and t.numel() * 4 <= self.p2p_limit:
            if async_op:  # side stream: overlaps the rest of backward, joined in _allreduce_all
                cur = torch.cuda.current_stream(self.net.device)
                self._comm_stream.wait_stream(cur)
                with torch.cuda.stream(self._comm_stream):
                    self.p2p.all_reduce(t)
                self._p2p_pending = True
            else:
                self.p2p.all_reduce(t)
            return
        w = dist.all_reduce(t, group=self.group, async_op=async_op)
        if async_op:
            self._works.append(w)

    def _grad_ready(self, layer_idx: int):
        b = self._trigger.get(layer_idx)
        if b is None or self.world == 1:
            return
        _, lo, hi = b
        self._reduce(self.net.store.grad[lo:hi], async_op=True)

    def _allreduce_all(self):
        if self.world == 1:
            return
        if self.overlap:
            for w in self._works:
                w.wait()
            if self.p2p is not None and self._p2p_pending:
                torch.cuda.current_stream(self.net.device).wait_stream(self._comm_stream)
                self._p2p_pending = False
        else:
            self._reduce(self.net.store.grad, async_op=False)
        self._works = []

    def check_comm(self):
        """Raise if the one-shot all-reduce recorded a peer timeout, or the reference CNN's dense head a row
        tile's flag-wait timeout (csrc/khead.hip; call outside the timed loop)."""
        if self.p2p is not None:
            self.p2p.check()
        ws = getattr(self.net, "khead_ws", None)
        if ws is not None and self.net._bound_B and ops.khead_error(ws, self.net._bound_B) != 0:
            raise RuntimeError("dense head: a row tile's flag wait timed out (its step's results are invalid)")

    @property
    def allreduce_path(self) -> str:
        return "p2p+rccl" if self.p2p is not None and any(
            (hi - lo) * 4 > self.p2p_limit for _, lo, hi in self.buckets) else ("p2p" if self.p2p else "rccl")

    # ------------------------------------------------------------------ one step
    phase_timer = None  # utils.logging.PhaseTimer: per-phase GPU time of eager steps

    # the step contains the gradient all-reduce (subclasses that exchange gradients otherwise say False)
    _step_all_reduces = True
    # eager warm-up steps before a capture (allocator / communicators / code objects); their effect on the
    # engine state is undone.  A subclass whose step mutates state outside the engine sets 0.
    capture_warmup = 3

    # single rank + fused LeNet-5: the reduce kernel applies the update itself (no optimizer launch)
    fused_update = _diag_on("lenet_fused_update")

    def _step_body(self, x, y):
        hook = self._grad_ready if (self.overlap and self.world > 1) else None
        pt = self.phase_timer
        if pt is not None and torch.cuda.is_current_stream_capturing():
            pt = None
        if pt is None and self._fused_step_ok():
            # the whole step in two launches; at world > 1 the reduce kernel sums the gradients over the
            # ranks itself (in-kernel LL exchange over xGMI) before applying the update
            ll = self.p2p.comm if (self.world > 1 and self._step_all_reduces) else None
            return self.net.compute_gradients_and_update(x, y, self._index_stream, ll=ll, run_stats=self.run_stats)
        if pt is not None:
            pt.start("compute")  # forward + loss + backward (the fused head runs all three)
        stats = self.net.compute_gradients(x, y, grad_ready=hook)
        if pt is not None:
            pt.stop("compute")
            pt.start("comm")  # waits for the overlapped bucket all-reduces
        self._allreduce_all()
        if pt is not None:
            pt.stop("comm")
            pt.start("update")
        self.net.store.sgd_step(self._index_stream, run_stats=(stats, self.run_stats))
        if pt is not None:
            pt.stop("update")
        return stats

    def _fused_step_ok(self) -> bool:
        """The fused LeNet-5 step (train + reduce/exchange/update: two launches) is usable: single rank,
        or every rank on the one-shot p2p path (its communicator carries the LL exchange slots) and the
        exchange passed its real-kernel self-test (:meth:`_verify_fused_exchange`)."""
        if not (self.fused_update and getattr(self.net, "lenet_fused", False)
                and self.net.store.lenet_frag is not None):
            return False
        if self.world == 1 or not self._step_all_reduces:
            return True  # no exchange inside the step (single rank, FedAvg local steps)
        return (self.p2p is not None and getattr(self.p2p.comm, "ll_slots", 0) >= 256
                and self.net.store.total * 4 <= self.p2p_limit and self.fused_selftest.get("ok", True))

    # result of the fused exchange self-test ({} = not run yet; "ok": False disables the fused step)
    fused_selftest: dict = {}

    def _verify_fused_exchange(self):
        """Real-kernel self-test of the multi-rank fused step, run once (collectively) before the first
        step: the production reduce kernel with the production grid (one workgroup per job when every rank
        has its own GPU) and the in-kernel exchange, on rank-distinct batches.  Its summed gradient must equal,
        bit for bit, the rank-order sum of the ranks' local gradients (the same train / reduce kernels
        without the exchange, gathered over the process group), and the updated weights must be
        bit-identical on every rank.  On a mismatch or a peer timeout every rank falls back to the
        unfused step (compute + one-shot all-reduce or RCCL + SGD).  The engine state is restored after.
        Reference semantics held here: the synchronous server's mean of the K uploaded gradients
        (/root/reference/src/server/federated_server.ts:92-117)."""
        if (self.fused_selftest or self.world == 1 or not self._step_all_reduces or not _diag_on("fused_selftest")
                or getattr(self, "data", None) is None):
            return
        if not (self.fused_update and getattr(self.net, "lenet_fused", False) and self.net.store.lenet_frag is not None
                and self.p2p is not None and getattr(self.p2p.comm, "ll_slots", 0) >= 256
                and self.net.store.total * 4 <= self.p2p_limit):
            return
        net, dev = self.net, self.net.device
        t0 = time.perf_counter()
        res = {"ok": True, "why": "", "exch_blocks": int(getattr(net, "lenet_exch_blocks", 0))}
        snap = net.snapshot_state()
        idx0 = self.idx.clone()
        cursor = self._index_stream[1].clone() if self._index_stream is not None else None
        rs0 = self.run_stats.clone()
        comm = self.p2p.comm
        from .p2p import _agree

        gloo = dist.get_backend(self.group) == "gloo"
        # Every collective below is entered by EVERY rank: local work runs under try, and the ranks agree on
        # its outcome before the next collective (a rank that raised must not leave its peers blocked in an
        # all_gather it never reaches -- ADVICE r4).
        g_local = None
        try:
            n_rows = self.data.shape[0]
            self.idx.copy_((torch.arange(self.B, device=dev, dtype=torch.int64) * 7919 + 104729 * self.rank + 17)
                           % n_rows)
            # local gradients through the same kernels without the exchange
            self._gather()
            net.compute_gradients(self.xb, self.yb)
            torch.cuda.synchronize(dev)
            g_local = net.store.grad.clone()
        except Exception as e:  # noqa: BLE001 (any failure -> the unfused path)
            res.update(ok=False, why=f"fused exchange self-test (local gradient) raised {e!r:.200}")
        try:
            if _agree(res["ok"], self.group, dev):
                parts = [torch.empty_like(g_local, device="cpu" if gloo else dev) for _ in range(self.world)]
                dist.all_gather(parts, g_local.cpu() if gloo else g_local, group=self.group)
                ref = parts[0].cpu().clone()
                for r in range(1, self.world):
                    ref += parts[r].cpu()  # rank order, fp32: the in-kernel exchange's summation order
                net.restore_state(snap)
                try:
                    comm.set_timeout(5.0)
                    self._gather()
                    net.compute_gradients_and_update(self.xb, self.yb, None, ll=comm)
                    torch.cuda.synchronize(dev)
                    if comm.error() != 0:
                        res.update(ok=False, why="peer timeout in the fused exchange self-test")
                    elif not torch.equal(net.store.grad.cpu(), ref):
                        bad = int((net.store.grad.cpu() != ref).sum())
                        res.update(ok=False, why=f"fused exchange self-test: {bad} gradient elements differ from "
                                                 f"the rank-order sum")
                except Exception as e:  # noqa: BLE001
                    res.update(ok=False, why=f"fused exchange self-test raised {e!r:.200}")
                # replicas must agree bit for bit (every rank enters both reductions, failed or not)
                w = net.store.master
                lo, hi = w.clone(), w.clone()
                if gloo:
                    lo, hi = lo.cpu(), hi.cpu()
                dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=self.group)
                dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=self.group)
                if res["ok"] and not torch.equal(lo, hi):
                    res.update(ok=False, why="fused exchange self-test: replicas differ after the update")
            elif res["ok"]:
                res.update(ok=False, why="a peer's fused exchange self-test failed (local gradient)")
        finally:
            try:
                comm.set_timeout(30.0)
            except Exception:
                pass
            torch.cuda.synchronize(dev)
            net.restore_state(snap)
            self.idx.copy_(idx0)
            if cursor is not None:
                self._index_stream[1].copy_(cursor)
            self.run_stats.copy_(rs0)
        ok = _agree(res["ok"], self.group, dev)
        if res["ok"] and not ok:
            res.update(ok=False, why="a peer's fused exchange self-test failed")
        res["ms"] = round((time.perf_counter() - t0) * 1e3, 1)
        self.fused_selftest = res
        if not ok:
            self.p2p_reason = res["why"]
            self._graph = None
            self._multi, self._multi_u = None, 0

    @property
    def step_launches(self) -> str:
        """What one training step is made of (diagnostic, reported by bench.py)."""
        if self._fused_step_ok():
            return ("train+reduce/exchange/update" if self.world > 1 and self._step_all_reduces
                    else "train+reduce/update")
        return "compute+allreduce+sgd" if self.world > 1 else "compute+sgd"

    def timed_eager_steps(self, n: int) -> dict:
        """Per-phase GPU milliseconds per step over ``n`` eager (uncaptured) steps on the bound index
        stream: data (batch gather), compute, comm, update.  Diagnostic: eager launches add host gaps."""
        from ..utils.logging import PhaseTimer

        pt = PhaseTimer()
        self.phase_timer = pt
        try:
            for _ in range(n):
                pt.start("data")
                self._gather()
                pt.stop("data")
                self._step_body(self.xb, self.yb)
            out = {k: v / n for k, v in pt.summary().items()}
        finally:
            self.phase_timer = None
        return out

    def set_lr(self, lr: float):
        self.lr = lr
        self.net.store.set_hyper(lr, self.momentum, self.weight_decay, grad_scale=self._grad_scale())

    def train_step(self, x: torch.Tensor, y: torch.Tensor):
        """Eager step on an explicit batch; returns device stats [loss_sum, correct]."""
        self.steps += 1
        return self._step_body(x, y)

    # ------------------------------------------------------------------ graph-captured step over an HBM dataset
    def bind_dataset(self, data: torch.Tensor, labels: torch.Tensor, batch_size: int, scale: float = 1.0):
        """Attach an HBM-resident dataset (uint8/bf16 [N, ...], int32 labels); steps then take index batches.
        ``batch_size``: rows per step per rank; with ``min_updates_per_version`` it is the MICROBATCH size
        and a step takes ``micro_per_rank[rank]`` microbatches (their rows concatenated)."""
        self.data, self.labels, self.scale = data, labels, scale
        self.micro_B = batch_size
        if self.min_updates is not None:
            # the version's gradient = the mean of its K microbatches' mean-loss gradients: every row's loss
            # gradient scaled by 1 / (K * microbatch) in the train kernel (the same bf16 rounding as one
            # step on the union batch) and the ranks' sums added unscaled
            self.net.loss_scale = 1.0 / (batch_size * self.min_updates)
            batch_size *= self.micro_per_rank[self.rank]
        self.B = batch_size
        net = self.net
        net.bind(batch_size)
        self.idx = torch.zeros(batch_size, dtype=torch.int64, device=net.device)
        self.yb = net.y_buf
        if data.dtype == torch.uint8:
            # the first layer reads dataset rows through the index vector (fused gather + cast)
            self.xb = ops.GatherRef(data, self.idx, scale, net.input_shape)
        else:
            self.xb = net.x_buf
        # collective (every rank binds its dataset): the real-kernel check of the fused multi-rank step runs
        # here, never hidden inside a step that only some ranks might take
        self.fused_selftest = {}
        self._verify_fused_exchange()

    # ------------------------------------------------------------------ preprocess callbacks on the device path
    def add_preprocess_callback(self, cb):
        """Run ``cb(Batch) -> Batch`` on every training batch, as the reference's dataset does on every
        dispensed batch (/root/reference/src/server/dataset.ts:87-96).  On the device engine the batch is
        gathered from the HBM dataset (one launch), ``Batch.x`` is its fp32 [B, ...] image tensor and
        ``Batch.y`` its int32 labels, both on the GPU; ``Batch.batch`` is the device step cursor (a
        1-element int64 tensor) and ``Batch.epoch`` is -1 (epochs are a host-side notion here).  The
        callback must be made of device tensor ops with fixed shapes: it is captured into the step's
        hipGraph and replayed with it.  It may return new tensors or modify ``x`` / ``y`` in place."""
        self.preprocess_callbacks.append(cb)
        self._graph = None  # the captured step must include it
        self._multi, self._multi_u = None, 0

    addPreprocessCallback = add_preprocess_callback

    def _gather_preprocessed(self):
        from ..data.dataset import Batch

        net = self.net
        xb, yb = net.x_buf, net.y_buf
        ops.gather_batch(self.data, self.labels, self.idx, xb, yb, self.scale)
        cursor = self._index_stream[1] if self._index_stream is not None else torch.zeros(1, dtype=torch.int64,
                                                                                          device=xb.device)
        b = Batch(cursor, -1, xb.float(), yb, 0, int(xb.shape[0]), self.idx)
        for cb in self.preprocess_callbacks:
            b = cb(b)
        if tuple(b.x.shape) != tuple(xb.shape) or tuple(b.y.shape) != tuple(yb.shape):
            raise ValueError("a preprocess callback must keep the batch shapes "
                             f"(x {tuple(xb.shape)}, y {tuple(yb.shape)})")
        xb.copy_(b.x)
        if b.y is not yb:
            yb.copy_(b.y)
        self.xb, self.yb = xb, yb

    def _gather(self):
        if self.preprocess_callbacks:
            self._gather_preprocessed()
            return
        if isinstance(self.xb, ops.GatherRef):
            if self.net.head_start is not None:
                # the fused head reads labels through the index vector: no gather launch
                self.yb = ops.LabelRef(self.labels, self.idx)
            else:
                ops.gather_labels(self.labels, self.idx, self.yb)
        else:
            ops.gather_batch(self.data, self.labels, self.idx, self.xb, self.yb, self.scale)

    def _capture(self):
        net = self.net
        # warm-up on a side stream (allocator, RCCL communicators, kernel code objects); the warm-up
        # steps are not training steps: the engine state is restored before capture.  The side stream
        # waits for the snapshot copies (taken on the current stream) before its first step.
        snap = net.snapshot_state()
        rs0 = self.run_stats.clone()
        cursor = self._index_stream[1].clone() if self._index_stream is not None else None
        idx0 = self.idx.clone()
        s = torch.cuda.Stream(device=net.device)
        s.wait_stream(torch.cuda.current_stream(net.device))
        with torch.cuda.stream(s):
            for _ in range(self.capture_warmup):
                self._gather()
                self._step_body(self.xb, self.yb)
        torch.cuda.current_stream(net.device).wait_stream(s)
        torch.cuda.synchronize(net.device)
        net.restore_state(snap)
        self.run_stats.copy_(rs0)
        self.idx.copy_(idx0)
        if cursor is not None:
            self._index_stream[1].copy_(cursor)
        torch.cuda.synchronize(net.device)
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream(device=net.device)  # our own capture stream: a failed capture can be ended
        try:
            if self.graph_mode == "full":
                with torch.cuda.graph(g, stream=cs):
                    self._gather()
                    self.stats = self._step_body(self.xb, self.yb)
                self._graph = (g, None)
            else:  # split: compute graph, eager all-reduce, SGD graph
                g2 = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=cs):
                    self._gather()
                    self.stats = self.net.compute_gradients(self.xb, self.yb)
                with torch.cuda.graph(g2, stream=cs):
                    self.net.store.sgd_step(self._index_stream, run_stats=(self.stats, self.run_stats))
                self._graph = (g, g2)
        except Exception:
            # a collective that cannot be captured (e.g. gloo on device tensors) leaves the capture open
            # on ``cs``, which would make every later allocation fail: end it before falling back
            with torch.cuda.stream(cs):
                if torch.cuda.is_current_stream_capturing():
                    try:
                        g.capture_end()
                    except Exception:
                        pass
            net.restore_state(snap)
            self.run_stats.copy_(rs0)
            self.idx.copy_(idx0)
            if cursor is not None:
                self._index_stream[1].copy_(cursor)
            raise
        for gr in self._graph:
            if gr is not None:
                ops.graph_upload(gr)
        torch.cuda.synchronize(net.device)

    def bind_distri_dataset(self, ds, rank: int = 0, world: int = 1, scale: Optional[float] = None):
        """Train from a :class:`~distriflow_amd.data.dataset.DistriDataset`: its tensors become the
        HBM-resident dataset and its dispenser's epochs / shuffles / FCFS order the device index stream
        (reference DistributedDataset, /root/reference/src/server/dataset.ts:47-96).  Returns the
        number of steps in the schedule; ``steps_per_epoch`` is set for epoch bookkeeping."""
        if scale is None:
            scale = 1.0 / 255.0 if ds.x.dtype == torch.uint8 else 1.0
        self.bind_dataset(ds.x, ds.y, ds.batch_size, scale=scale)
        for cb in ds.preprocess_callbacks:  # the dataset's preprocess chain runs on every device batch
            if cb not in self.preprocess_callbacks:
                self.add_preprocess_callback(cb)
        epochs_left = max(1, ds.epochs - ds.epoch)
        if self.min_updates is not None:  # K microbatches of the one FCFS stream per version
            stream = fedsgd_rows(ds.index_stream(0, 1, device=self.net.device, allow_preprocess=True),
                                 self.min_updates, rank, world)
        else:
            stream = ds.index_stream(rank, world, device=self.net.device, allow_preprocess=True)
        self.bind_index_stream(stream)
        self.steps_per_epoch = max(1, stream.shape[0] // epochs_left)
        self.schedule_steps = int(stream.shape[0])
        return self.schedule_steps

    def bind_index_stream(self, stream: torch.Tensor):
        """Device-resident batch schedule ``stream`` [nsteps][B] (int64, this rank's rows): the step's
        optimizer launch stages the next step's indices itself (csrc/optim.hip), so :meth:`step`
        is a bare graph replay.  Wraps around after ``nsteps`` steps."""
        if stream.shape[1] != self.B:
            raise ValueError(f"index stream rows must have {self.B} indices")
        stream = stream.to(self.idx.device, torch.int64).contiguous()
        cursor = torch.zeros(1, dtype=torch.int64, device=self.idx.device)
        self.idx.copy_(stream[0])
        if self._index_stream is None or self._index_stream[0].shape != stream.shape:
            self._graph = None  # the captured optimizer launch references the stream buffers
            self._multi, self._multi_u = None, 0
        self._index_stream = (stream, cursor, self.idx)

    def step(self):
        """One training step on the next batch of the bound index stream."""
        if self._index_stream is None:
            raise RuntimeError("bind_index_stream() first")
        self.steps += 1
        _beat(self.steps)
        if self.graph_mode == "none":
            self._gather()
            st = self._step_body(self.xb, self.yb)
        else:
            if self._graph is None:
                self._capture_with_fallback()
            st = self._last_eager if self._graph is None else self._replay()
        self._after_replay(1)
        return st

    def step_indices(self, idx: torch.Tensor):
        """One training step on dataset rows ``idx`` (device int64 [B])."""
        if self._index_stream is not None:
            raise RuntimeError("an index stream is bound: use step()")
        self.idx.copy_(idx, non_blocking=True)
        self.steps += 1
        if self.graph_mode == "none":
            self._gather()
            return self._step_body(self.xb, self.yb)
        if self._graph is None:
            self._capture_with_fallback()
            if self._graph is None:
                return self._last_eager
        return self._replay()

    def _capture_with_fallback(self):
        """Capture fallback chain full -> split -> none (eager); every failure is recorded.

        The ranks agree on every attempt (MIN of a success flag, outside any capture): if capture
        fails on one rank only, all of them fall back together, so no rank replays a graph whose
        collectives / one-shot epochs its peers never issue."""
        while True:
            ok = True
            try:
                self._capture()
            except Exception as e:  # e.g. collective capture unsupported by this RCCL/driver
                torch.cuda.synchronize(self.net.device)
                self.capture_error = repr(e)
                ok = False
            if self.world > 1:
                flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.net.device)
                dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
                if ok and int(flag.item()) == 0:
                    self.capture_error = "a peer rank failed to capture"
                ok = bool(flag.item())
            if ok:
                return
            self._works = []
            self._graph = None
            self._multi, self._multi_u = None, 0
            if self.graph_mode == "full":
                self.graph_mode = "split"
            else:
                self.graph_mode = "none"
                self._gather()
                self._last_eager = self._step_body(self.xb, self.yb)
                return

    # ------------------------------------------------------------------ callbacks (no launches in the step)
    def on_new_version(self, cb):
        """``cb(old_version, new_version)`` once per replay (reference AbstractServer.onNewVersion,
        /root/reference/src/server/abstract_server.ts:67-69,105-109).  A version is one applied update."""
        self._version_cbs.append(cb)

    def on_upload(self, cb):
        """``cb(stats)`` once per replay with the replay's device statistics (reference onUpload with the
        clients' metrics, abstract_server.ts:77-79,111-115): version, steps, images, loss (mean per
        example), accuracy, updates counted on the device, rank, world."""
        self._upload_cbs.append(cb)

    onNewVersion = on_new_version
    onUpload = on_upload

    def _cb_sources(self) -> list:
        """Device tensors read back per replay for the callbacks (subclasses add their counters)."""
        return [self.run_stats]

    def _cb_stats(self, cur: list, last: list, v0: int, v1: int, n: int) -> dict:
        """The on_upload payload of one replay from the read-back sources (cumulative device counters:
        this replay = cur - last)."""
        dl, dc, du = (cur[0][k] - last[0][k] for k in range(3))
        images = n * self.B
        return {"version": v1, "steps": n, "images": n * self.images_per_step, "loss": dl / max(images, 1),
                "accuracy": dc / max(images, 1), "updates": int(round(du)), "rank": self.rank, "world": self.world}

    @property
    def images_per_step(self) -> int:
        """Examples in one step over all ranks (one version)."""
        if self.min_updates is not None:
            return self.min_updates * self.micro_B
        return self.B * self.world

    def _after_replay(self, nsteps: int):
        """Queue an asynchronous read-back of the device counters after a replay of ``nsteps`` steps (a
        copy into pinned memory behind the replay, outside the captured step) and fire the callbacks of
        every replay whose copy has landed.  Nothing happens without registered callbacks."""
        if not (self._version_cbs or self._upload_cbs):
            return
        v1 = self.steps
        srcs = self._cb_sources()
        if self.net.is_gpu:
            if self._cb_ring is None:
                self._cb_ring = [[torch.empty(t.numel(), dtype=t.dtype, pin_memory=True) for t in srcs]
                                 for _ in range(16)]
                self._cb_next = 0
            if len(self._cb_pending) >= len(self._cb_ring):
                self._drain_callbacks(block_one=True)
            bufs = self._cb_ring[self._cb_next]
            self._cb_next = (self._cb_next + 1) % len(self._cb_ring)
            for b, t in zip(bufs, srcs):
                b.copy_(t.reshape(-1), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._cb_pending.append((ev, bufs, v1 - nsteps, v1, nsteps))
        else:
            self._cb_pending.append((None, [t.reshape(-1).clone() for t in srcs], v1 - nsteps, v1, nsteps))
        self._drain_callbacks()

    def _drain_callbacks(self, block: bool = False, block_one: bool = False):
        while self._cb_pending:
            ev, bufs, v0, v1, n = self._cb_pending[0]
            if ev is not None and not ev.query():
                if not (block or block_one):
                    return
                ev.synchronize()
            self._cb_pending.pop(0)
            cur = [b.tolist() for b in bufs]
            last = self._cb_last or [[0] * len(c) for c in cur]
            self._cb_last = cur
            st = self._cb_stats(cur, last, v0, v1, n)
            change = self._version_change(cur, last, v0, v1)
            if change is not None:
                for cb in self._version_cbs:
                    cb(*change)
            for cb in self._upload_cbs:
                cb(st)
            block_one = False

    def _version_change(self, cur: list, last: list, v0: int, v1: int):
        """(old, new) version of one replay for on_new_version, or None when the replay published none (a
        synchronous step always publishes one: the versions are the step counts)."""
        return v0, v1

    def flush_callbacks(self):
        """Fire the callbacks of every replay issued so far (waits for their read-backs)."""
        self._drain_callbacks(block=True)

    # ------------------------------------------------------------------ multi-step graphs
    MAX_STEPS_PER_GRAPH = 64
    SUPPORTS_MULTISTEP = True

    def prepare_run(self, n: int):
        """Capture (outside any timed region) the graph :meth:`run` replays for ``n`` steps: up to
        MAX_STEPS_PER_GRAPH consecutive full training steps unrolled into ONE hipGraph, so a run of n
        steps is ceil(n / U) graph launches instead of n (the launch-bound inner loop of a small model
        stays on the device).  Every step in it is the complete captured step (gather, forward,
        backward, gradient exchange, update); the batch cursor, dropout counters and one-shot
        all-reduce epochs all advance on the device.  Only in ``full`` graph mode."""
        if self.graph_mode != "full" or not self.net.is_gpu or not self._has_schedule():
            return
        if self._graph is None:
            self._capture_with_fallback()
        from ..diagnostics import diag

        u = max(1, min(int(n), self.MAX_STEPS_PER_GRAPH, diag("graph_steps")))
        if self.graph_mode != "full" or self._graph is None or u <= 1 or self._multi_u == u:
            return
        net = self.net
        snap = net.snapshot_state()
        cursor = self._index_stream[1].clone() if self._index_stream is not None else None
        idx0 = self.idx.clone()
        torch.cuda.synchronize(net.device)
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream(device=net.device)
        ok = True
        try:
            with torch.cuda.graph(g, stream=cs):
                for _ in range(u):
                    self._gather()
                    self.stats = self._step_body(self.xb, self.yb)
        except Exception as e:
            with torch.cuda.stream(cs):
                if torch.cuda.is_current_stream_capturing():
                    try:
                        g.capture_end()
                    except Exception:
                        pass
            self.capture_error = repr(e)
            ok = False
        torch.cuda.synchronize(net.device)
        # capturing launches nothing, but restore anyway: the step state must be as before
        net.restore_state(snap)
        self.idx.copy_(idx0)
        if cursor is not None:
            self._index_stream[1].copy_(cursor)
        if self.world > 1:  # all ranks use multi-step graphs or none do (identical collective sequences)
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=net.device)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
            ok = bool(flag.item())
        if ok:
            ops.graph_upload(g)
        torch.cuda.synchronize(net.device)
        self._multi = g if ok else None
        self._multi_u = u if ok else 0

    def _has_schedule(self) -> bool:
        return self._index_stream is not None

    def run(self, n: int):
        """``n`` training steps: multi-step graph replays (see :meth:`prepare_run`) plus single steps."""
        st = None
        if self._multi is not None and self._multi_u > 1:
            for _ in range(n // self._multi_u):
                self._multi.replay()
                self.steps += self._multi_u
                _beat(self.steps)
                self._after_replay(self._multi_u)
                st = self.stats
            n -= (n // self._multi_u) * self._multi_u
        for _ in range(n):
            st = self.step()
        return st

    def _replay(self):
        g, g2 = self._graph
        g.replay()
        if g2 is not None:
            if self.world > 1 and self._step_all_reduces:
                self._reduce(self.net.store.grad, async_op=False)
            g2.replay()
        return self.stats


def _beat(step: int):
    """Progress beat for the dead-peer / stall watchdog (parallel/watchdog.py; no-op without one)."""
    from .watchdog import beat

    beat(step)


def shared_gpu_cus(world: int) -> int:
    """CUs of one rank's persistent kernels when ranks time-share a GPU (rehearsals), else 0 (no cap)."""
    ndev = max(1, torch.cuda.device_count())
    share = -(-world // ndev) if ndev < world else 1
    if share == 1:
        return 0
    cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    # three quarters of the chip split between the ranks: the rest stays free for their other kernels
    return max(8, cus * 3 // 4 // share // 8 * 8)


def shared_gpu_exch_blocks(world: int) -> int:
    """Job workgroups of the fused LeNet-5 reduce launch per rank: 0 (one per job) with a GPU per rank;
    with ranks time-sharing one GPU, few enough (a multiple of 8, each running <= 16 jobs) that every
    rank's waiting workgroups (256 threads, 4 per CU) fit on the chip at once beside the peers' kernels."""
    ndev = max(1, torch.cuda.device_count())
    share = -(-world // ndev) if ndev < world else 1
    return 0 if share == 1 else max(64, (512 // share) // 8 * 8)


def fedsgd_rows(global_rows: torch.Tensor, k: int, rank: int, world: int, epochs: Optional[list] = None):
    """Per-version rows of one rank for a FedSGD count barrier of ``k`` microbatches per version:
    ``global_rows`` [nb][B] is the one FCFS microbatch stream (every rank holds the same); version v takes
    microbatches v*k .. v*k + k - 1, rank r the ``k // world + (r < k % world)`` of them after the lower
    ranks' share, concatenated -> [nb // k][m_r * B].  ``epochs`` (per microbatch) -> also the epoch of
    each version's first microbatch."""
    counts = [k // world + (1 if r < k % world else 0) for r in range(world)]
    off, m = sum(counts[:rank]), counts[rank]
    nv = global_rows.shape[0] // k
    if nv == 0:
        raise ValueError(f"the stream has {global_rows.shape[0]} microbatches, fewer than one version of {k}")
    ids = (torch.arange(nv, device=global_rows.device)[:, None] * k + off
           + torch.arange(m, device=global_rows.device)[None, :])
    rows = global_rows[ids.reshape(-1)].reshape(nv, m * global_rows.shape[1]).contiguous()
    if epochs is None:
        return rows
    return rows, [epochs[v * k] for v in range(nv)]


def epoch_permutations(n: int, batch: int, steps: int, device, seed: int = 0):
    """Device-resident index stream: concatenated random permutations, sliced per step."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    need = batch * steps
    chunks = []
    while sum(c.numel() for c in chunks) < need:
        chunks.append(torch.randperm(n, generator=g))
    return torch.cat(chunks)[:need].view(steps, batch).to(device)
