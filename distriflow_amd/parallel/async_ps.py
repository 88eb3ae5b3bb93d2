"""Asynchronous SGD against a device-resident, bounded-staleness parameter server (BASELINE.json configs[2]).

Reference: ``AsynchronousSGDServer`` keeps the model, dispenses microbatches first-come-first-serve
and applies every uploaded gradient on arrival; ``AsynchronousSGDClient`` downloads weights plus a
batch, computes a gradient and uploads it
(/root/reference/src/server/asynchronousSGD_server.ts:45-108,
/root/reference/src/client/asynchronousSGD_client.ts:16-84).  The README's ``maximumStaleness``
(/root/reference/README.md:27) is the intended bound and is enforced here.

This is the throughput path.  The message-level roles (``parallel/server.py``/``worker.py``) keep
the reference's protocol and callbacks.  On one MI355X node the server is not a process: its state is
device memory that every rank maps over xGMI (csrc/async_ps.hip, csrc/ps_device.h).  The server rank
holds the control buffer (the version word = count of admitted gradients, the FCFS microbatch cursor,
the completion arrays); the fp32 master is SHARDED by contiguous parameter range over all ranks' HBM, one
shard per rank.  A gradient is admitted by one lock-free CAS on the version word (the staleness bound is
its check) and applied element by element to the owning shards with CAS adds, so the applies of
different ranks run in parallel: no rank ever holds a lock that another waits for.  A worker step is a
bare hipGraph replay of device stages, with no host round trip.

Fused LeNet-5 (the headline model): TWO launches per step, the same shape as a synchronous step.
  1. the whole-network train kernel (forward, loss, backward of the claimed microbatch);
  2. the reduce kernel in parameter-server mode (csrc/lenet_fused.hip): its staging workgroup admits the
     gradient as the launch starts (``version_now - version_pulled <= max_staleness``), completes the
     microbatch and claims / stages the next one; the slot owners reduce the gradient, add
     ``-lr * g`` to their elements of the sharded master (rejected: read the current values) and refresh
     the local master / bf16 copies / conv fragments from the result.  A one-time prologue (pull +
     refresh) precedes the first step.
Other models: ``ps_fetch_pull`` (claim + copy out of the shards), bf16 refresh, the model's kernels,
``ps_apply`` (admit + sharded adds).

Ranks never wait for each other.  A slow rank only makes its own gradients staler, which the bound
then rejects.  The admission CAS is the one serialisation point (one remote atomic per step per rank).

Staleness is exact (an upper bound that always holds): an admitted gradient's last workgroup bumps a
shared ``applied`` counter once every one of its adds has landed, and every refresh records the applied
count it read BEFORE copying; admission compares the version against the minimum of those counts, so
``version - vp <= max_staleness`` bounds the updates missing from any element of the weights the
gradient was computed on (csrc/ps_device.h).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .. import native
from ..diagnostics import diag, on as diag_on
from .data_parallel import DataParallelTrainer, shared_gpu_exch_blocks


class AsyncPSTrainer(DataParallelTrainer):
    _step_all_reduces = False  # gradients go to the parameter server, not through a collective
    fused_update = False       # the update is the parameter server's apply
    SUPPORTS_MULTISTEP = True  # the whole PS protocol of a step is device work: steps unroll like sync ones
    OWNER_MARGIN = 2.0         # calibration: owner-applies only when the CAS adds take over this factor longer

    def __init__(self, net, lr: float = 0.001, max_staleness: int = 4, group=None, server_rank: int = 0,
                 graph: str = "full", timeout_s: float = 30.0, owner_apply: Optional[bool] = None,
                 joinable: bool = False):
        """``joinable``: workers outside this process group may attach later (:meth:`publish` /
        :meth:`attach`, parallel/elastic.py): uncached buffers and no exclusive-writer shortcuts even at one
        rank."""
        if not net.is_gpu:
            raise RuntimeError("AsyncPSTrainer is the GPU path; use AsynchronousSGDServer/Client on CPU")
        super().__init__(net, lr=lr, group=group, overlap=False, graph="full" if graph == "split" else graph,
                         broadcast_init=True, allreduce="rccl")
        self.max_staleness = int(max_staleness)
        self.server_rank = server_rank
        self.joinable, self.joiner = bool(joinable), False
        self.timeout_s = float(timeout_s)
        # collective setup: every rank learns whether every other rank managed its part (no rank is left
        # waiting in a barrier that a failed peer never reaches)
        err, handle, shard = None, b"", b""
        try:
            self.ps = native.require().PSComm(self.rank, self.world, server_rank, net.store.total, timeout_s,
                                              joinable=self.joinable)
            if self.rank == server_rank:
                handle = self.ps.handle()
            shard = self.ps.shard_handle()
        except Exception as e:
            err = e
        self._agree(err, "allocation/export")
        ctrl = [handle]
        shards = [shard] * self.world
        if self.world > 1:
            dist.broadcast_object_list(ctrl, src=server_rank, group=group)
            dist.all_gather_object(shards, shard, group=group)
        try:
            self.ps.open(ctrl[0], shards)
            self.ps.set_lr_source(net.store.hyper)  # applies read the device lr: set_lr holds after capture
        except Exception as e:
            err = e
        self._agree(err, "IPC open")
        self._handles = {"ctrl": ctrl[0], "shards": shards, "inboxes": None}
        # the element add every apply uses, on every shard from every rank at once, against exact sums
        ok = True
        try:
            self.ps.selftest_add()
        except Exception as e:
            err, ok = e, False
        self._agree(err, "shard self-test")
        if not self.ps.selftest_check():
            err = RuntimeError("shard add self-test mismatch")
        self._agree(err, "shard self-test check")
        # Apply path (csrc/async_ps.hip, csrc/ps_device.h):
        #   CAS            per-element compare-and-swap adds on the owning shards (7/8 of them remote at 8 ranks);
        #   owner-applies  admitted gradients go into the owners' inbox rings with plain stores, each shard is
        #                  drained (added in sequence order) by whichever rank holds its drain lock -- no remote
        #                  atomics.  The ring holds max_staleness + 2 gradients; a bounded staleness is required.
        # One rank: CAS (the exclusive writer's plain read-modify-writes).  Several: ``owner_apply`` / the diag
        # switch ps_owner_apply (1 owner, 0 CAS) force a path; by default (-1) both are timed here, every rank at
        # once on the real topology, over this model's size, and the faster one (max over ranks) is taken.
        mode = diag("ps_owner_apply") if owner_apply is None else int(bool(owner_apply))
        self.owner_apply = False
        self.apply_calib = None
        want_inbox = self.world > 1 and self.max_staleness >= 0 and mode != 0
        if mode == 1 and self.max_staleness < 0:
            raise ValueError("owner-applies needs a bounded max_staleness")
        if mode == 1 and self.world == 1:
            want_inbox = True
        if want_inbox:
            oh = b""
            try:
                oh = self.ps.owner_init(self.max_staleness + 2)
            except Exception as e:
                err = e
            self._agree(err, "owner inbox allocation")
            ohs = [oh] * self.world
            if self.world > 1:
                dist.all_gather_object(ohs, oh, group=group)
            self._handles["inboxes"] = ohs
            try:
                self.ps.owner_open(ohs, enable=False)
            except Exception as e:
                err = e
            self._agree(err, "owner inbox open")
            if mode == 1:
                self.owner_apply = True
            else:
                self.apply_calib = self._calibrate_apply(group)
                self.owner_apply = self.apply_calib["path"] == "owner-applies"
            self.ps.owner_enable(self.owner_apply)
        # every rank seeds its own shard (identical weights) -- after the calibration, which adds zeros to them
        try:
            self.ps.init_master(net.store.master)
        except Exception as e:
            err = e
        self._agree(err, "master seed")
        if self.world > 1:
            dist.barrier(group=group)
        self._finish_setup()

    def _finish_setup(self):
        net = self.net
        self._perm = None
        # fused LeNet-5: the reduce launch is the parameter server's apply (2 launches per step)
        self.fused_ps = (bool(getattr(net, "lenet_fused", False)) and net.store.lenet_frag is not None
                         and diag_on("async_fused"))
        # a warm-up step would claim a microbatch and apply a real gradient to the shared master: the
        # capture warms up with a compute-only step instead (_capture).  The reduce launch's owners wait for
        # the staging workgroup's admission decision (no lock is taken), then add or read their slots.
        self.capture_warmup = 0
        if self.fused_ps:
            # ranks that time-share one GPU: fewer protocol workgroups per rank (each owning several
            # slots), so every rank's workgroups waiting for their admission decision fit on the chip beside
            # the other ranks' (one rank per GPU: one workgroup per slot, all resident)
            net.lenet_exch_blocks = shared_gpu_exch_blocks(self.world)
        # one rank, any other model: the exclusive writer's step -- admission + next claim in one workgroup,
        # then the model's own optimizer launch gated on the decision, writing the new weights to the local
        # master, the compute copies and the shard in one pass (no pull copy, no refresh, no separate apply)
        h = net.store._hyper_host
        self.excl_fused = (self.world == 1 and not self.joinable and not self.fused_ps and not self.owner_apply
                           and net.store.compute_bf16 and net.store.lenet_frag is None and diag_on("ps_excl_fused")
                           and h[1] == 0.0 and h[2] == 0.0 and h[3] == 1.0)
        self._primed = False
        self._ps_stats_dev = self.ps.stats_tensor()  # device view of this rank's PS counters (callbacks)
        from .watchdog import register_owner_probe

        register_owner_probe("async_ps", self, lambda o: o.ps.host_error())

    # ------------------------------------------------------------------ elastic membership
    def attach_meta(self) -> dict:
        """What a joiner must agree on (parallel/elastic.py)."""
        return {"n": int(self.net.store.total), "world": self.world, "server_rank": self.server_rank,
                "max_staleness": self.max_staleness, "timeout_s": self.timeout_s,
                "owner_ring": int(self.ps.owner_ring()) if self._handles["inboxes"] else 0,
                "owner_on": bool(self.owner_apply), "fed_K": 0}

    def publish(self, store, prefix: Optional[str] = None):
        """Members (call on every rank; the server rank writes): publish the server's IPC handles so a worker
        outside this process group can :meth:`attach` at any time (reference: a client may connect whenever,
        /root/reference/src/server/asynchronousSGD_server.ts:50-63).  Needs ``joinable=True``."""
        from . import elastic

        if not self.joinable:
            raise RuntimeError("publish(): create the trainer with joinable=True")
        if self.rank == self.server_rank:
            elastic.publish(store, self.attach_meta(), self._handles["ctrl"], self._handles["shards"],
                            self._handles["inboxes"], self._handles.get("fed"), prefix=prefix or elastic.PREFIX)

    @classmethod
    def attach(cls, net, store, joiner_id: int, lr: Optional[float] = None, graph: str = "full",
               prefix: Optional[str] = None, timeout_s: float = 60.0):
        """A late-joining worker: a process OUTSIDE the members' process group maps the published server
        (control buffer, every shard, every inbox) and steps against it like a member -- its first pull
        copies the current master, its claims come from the shared FCFS cursor, its gradients face the same
        staleness bound.  ``joiner_id`` (>= the members' world size, unique per joiner) is its drain-lock id."""
        from . import elastic

        rec = elastic.read(store, prefix or elastic.PREFIX, timeout_s)
        m = rec["meta"]
        if int(m["n"]) != net.store.total:
            raise ValueError(f"attach: the server's master has {m['n']} elements, this model {net.store.total}")
        self = cls.__new__(cls)
        DataParallelTrainer.__init__(self, net, lr=0.001 if lr is None else lr, group=None, overlap=False,
                                     graph="full" if graph == "split" else graph, broadcast_init=False,
                                     allreduce="rccl")
        self.max_staleness = int(m["max_staleness"])
        self.server_rank = int(m["server_rank"])
        self.joinable, self.joiner = True, True
        self.timeout_s = float(m.get("timeout_s", 30.0))
        self._attach_meta = m
        self.ps = elastic.attach_ps(rec, joiner_id)
        self.ps.set_lr_source(net.store.hyper)
        self._handles = {"ctrl": rec["ctrl"], "shards": rec["shards"], "inboxes": rec["inboxes"]}
        self.owner_apply = bool(m.get("owner_on", False))
        self.apply_calib = None
        self._finish_setup()
        return self

    def _calibrate_apply(self, group, reps: int = 20) -> dict:
        """Time both apply paths with every rank at once (collective; the shards are not seeded yet, the
        update is zero): the per-element CAS adds and the owner-applies inbox / shard traffic over this
        model's elements.  The decision is the max over ranks of each, so every rank takes the same path."""
        res, err = [0.0, 0.0], None
        for mode in (0, 1):
            if self.world > 1:
                dist.barrier(group=group)
            try:
                res[mode] = float(self.ps.calibrate(mode, reps))
            except Exception as e:
                err = e
            self._agree(err, f"apply calibration ({'CAS' if mode == 0 else 'owner-applies'})")
        t = torch.tensor(res, dtype=torch.float64)
        if self.world > 1:
            ts = [torch.zeros_like(t) for _ in range(self.world)]
            dist.all_gather_object(ts, t, group=group)
            t = torch.stack(ts).max(0).values
        cas_us, own_us = float(t[0]), float(t[1])
        # owner-applies trades the atomics for freshness: an admitted gradient reaches the other ranks' refreshes
        # only once a lock holder has drained it (the next admission after its flag, then that rank's reduce),
        # so at a tight bound more gradients are rejected (shared-GPU W = 4, bound 2: 34 of 96 admitted against
        # 48 of 96 on the CAS path, tests/test_async_ps_gpu.py).  It is taken only where the remote atomics are
        # the clear bottleneck: CAS adds over twice the owner traffic's time.
        return {"cas_us": round(cas_us, 2), "owner_us": round(own_us, 2),
                "path": "owner-applies" if cas_us > self.OWNER_MARGIN * own_us else "cas", "reps": reps,
                "rule": f"owner-applies iff cas_us > {self.OWNER_MARGIN} x owner_us"}

    def _agree(self, err, what):
        ok = err is None
        if self.world > 1:
            from .p2p import _agree

            ok = _agree(ok, self.group, self.net.device)
        if not ok:
            raise RuntimeError(f"async PS setup failed ({what}) on {'this' if err else 'another'} rank: {err!r}")

    # ------------------------------------------------------------------ schedule
    def bind_schedule(self, perm: torch.Tensor, epochs: int = 0):
        """Global FCFS microbatch table ``perm`` [nbatches][B] (identical on every rank): microbatch id
        ``b`` trains on rows ``perm[b]``.  Dispatch is at-least-once per dataset epoch, as the
        reference's DistributedDataset (/root/reference/src/server/dataset.ts:47-67): a batch is
        complete only when a gradient for it is admitted, rejected (too stale) batches are handed out
        again on the cursor's next lap, and an epoch ends when all ``nbatches`` are complete.  After
        ``epochs`` epochs (0 = unbounded) steps become no-ops and :meth:`finished` turns true."""
        if perm.dim() != 2 or perm.shape[1] != self.B:
            raise ValueError(f"schedule must be [nbatches][{self.B}]")
        self._perm = perm.to(self.idx.device, torch.int64).contiguous()
        self.epochs = int(epochs)
        self.ps.set_schedule(int(perm.shape[0]), self.epochs)
        self._graph = None
        self._multi, self._multi_u = None, 0
        self._primed = False

    def _has_schedule(self) -> bool:
        return self._perm is not None

    # ------------------------------------------------------------------ one step
    def _prime(self):
        """Fused path prologue (eager, once per schedule): claim the first microbatch and pull the master
        into the local weights and compute copies; every later step's reduce launch (or, one rank: its
        admission workgroup and gated optimizer launch) does both itself."""
        if (self.fused_ps or self.excl_fused) and not self._primed:
            self.ps.fetch_pull(self.net.store.master, self._perm, self.idx)
            self.net.store.refresh_compute()
            self._primed = True

    def _gather(self):
        if self.fused_ps or self.excl_fused:
            super()._gather()  # labels through the staged indices (no launch)
            return
        self.ps.fetch_pull(self.net.store.master, self._perm, self.idx)
        self.net.store.refresh_compute()
        super()._gather()

    def _step_body(self, x, y):
        if self.fused_ps:
            ps = dict(ps=self.ps, ps_perm=self._perm, ps_idx=self.idx, ps_lr=float(self.lr),
                      ps_max_stale=int(self.max_staleness))
            return self.net.compute_gradients_and_update(x, y, None, run_stats=self.run_stats, ps=ps)
        stats = self.net.compute_gradients(x, y)
        if self.excl_fused:
            self.ps.excl_step(int(self.max_staleness), self._perm, self.idx)
            self.net.store.sgd_step(ps_gate=self.ps.excl_gate(), ps_mirror=self.ps.excl_mirror())
            return stats
        self.ps.apply(self.net.store.grad, self.lr, self.max_staleness)
        return stats

    @property
    def step_launches(self) -> str:
        if self.fused_ps:
            return "train+reduce/ps-apply/refresh/claim"
        return "compute+admit/claim+gated-update" if self.excl_fused else "pull+refresh+compute+ps-apply"

    def prepare_run(self, n: int):
        self._prime()
        if self.graph_mode == "full" and self._graph is None and self._has_schedule():
            # capture here WITHOUT the eager fallback step of _capture_with_fallback: a step taken outside
            # step() / run() would be a real, uncounted parameter-server update
            try:
                self._capture()
            except Exception as e:
                torch.cuda.synchronize(self.net.device)
                self.capture_error = repr(e)
                self._graph = None
                self.graph_mode = "none"
        super().prepare_run(n)

    def _capture(self):
        # compute-only warm-up (allocator, code objects, the fused kernels' host-built tables for this batch
        # size -- built with a synchronous copy, which a capture refuses) with no claim and no apply; its
        # effect on the local engine state is undone
        snap = self.net.snapshot_state()
        DataParallelTrainer._gather(self)
        self.net.compute_gradients(self.xb, self.yb)
        torch.cuda.synchronize(self.net.device)
        self.net.restore_state(snap)
        super()._capture()

    def _capture_with_fallback(self):
        try:
            self._capture()
        except Exception as e:
            torch.cuda.synchronize(self.net.device)
            self.capture_error = repr(e)
            self._graph = None
            self.graph_mode = "none"
            self._gather()
            self._last_eager = self._step_body(self.xb, self.yb)

    def step(self):
        if self._perm is None:
            raise RuntimeError("bind_schedule() first")
        self._prime()
        self.steps += 1
        if self.graph_mode == "none":
            self._gather()
            st = self._step_body(self.xb, self.yb)
        else:
            if self._graph is None:
                self._capture_with_fallback()
            st = self._last_eager if self._graph is None else self._replay()
        self._after_replay(1)
        return st

    # ------------------------------------------------------------------ callbacks
    def _cb_sources(self) -> list:
        # + the parameter server's local counters [accepted, rejected, sum staleness, max staleness, ...]
        return [self.run_stats, self._ps_stats_dev]

    def _cb_stats(self, cur, last, v0, v1, n) -> dict:
        """Per replay: this rank's admitted / rejected gradients and their staleness, the loss of the
        steps, and the versions it published (a version = one admitted gradient anywhere in the job)."""
        st = super()._cb_stats(cur, last, v0, v1, n)
        acc, rej = cur[1][0] - last[1][0], cur[1][1] - last[1][1]
        st.update(accepted=int(acc), rejected=int(rej),
                  mean_staleness=(cur[1][2] - last[1][2]) / acc if acc else 0.0, max_staleness=int(cur[1][3]),
                  updates=int(acc))
        return st

    # ------------------------------------------------------------------ state
    def ps_stats(self) -> dict:
        acc, rej, ssum, smax, retries, err, version, cursor, noops, applied = self.ps.stats()
        epoch, in_epoch, completed, redisp, skipped, dups, fin = self.ps.schedule_stats()
        return {"accepted": acc, "rejected": rej, "mean_staleness": ssum / acc if acc else 0.0,
                "max_staleness": smax, "admit_retries": retries, "error": err, "version": version,
                "applied": min(self.ps.owner_prefix()) if self.owner_apply else applied,
                "apply_path": "owner-applies" if self.owner_apply else "cas",
                "apply_calibration": self.apply_calib,
                "cursor": cursor, "noop_steps": noops, "epoch": epoch, "completed_in_epoch": in_epoch,
                "completed": completed, "redispatched": redisp, "skipped": skipped, "duplicates": dups,
                "finished": bool(fin)}

    def finished(self) -> bool:
        """Every batch of every configured epoch has an admitted gradient (host read; syncs)."""
        return bool(self.ps.schedule_stats()[6])

    def done_epochs(self) -> list:
        """Per batch id: 1 + the last epoch in which its gradient was applied (0 = never)."""
        return list(self.ps.done_epochs())

    def check_comm(self):
        err = self.ps.stats()[5]
        if err:
            raise RuntimeError(f"async PS: device wait timed out (error bits {err:#x})")

    def drain(self):
        """Owner-applies: add every gradient already flagged in this rank's inbox into its shard (the next
        pull would).  After every rank's last step, one drain on every rank (between two barriers) leaves
        the sharded master = w0 - lr * sum of the admitted gradients.  No-op on the CAS path."""
        if self.owner_apply:
            if not hasattr(self, "_drain_buf"):
                self._drain_buf = torch.empty_like(self.net.store.master)
            self.ps.drain(self._drain_buf)

    def pull_master(self, dst: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Gather the sharded master into ``dst`` (default: this rank's store, compute copies refreshed)."""
        if dst is None:
            self.ps.copy_master(self.net.store.master)
            self.net.store.refresh_compute()
            return self.net.store.master
        self.ps.copy_master(dst)
        return dst
