"""Device FedSGD: the reference's count barrier (minUpdatesPerVersion) with K < W on the parameter
server's shards -- a slow or lost rank never blocks a version.

Reference ``FederatedServer`` (/root/reference/src/server/federated_server.ts:52-117): an upload is
accepted only if its gradient was computed on the current model version (and no update is in progress);
once ``minUpdatesPerVersion`` uploads are accepted the server averages them, applies ``w -= lr * mean``,
bumps the version and broadcasts it; uploads of an older version are dropped.  The barrier counts
updates, not workers.

:class:`~distriflow_amd.parallel.data_parallel.DataParallelTrainer` with ``min_updates_per_version`` is the
throughput form (K >= W: every rank contributes K / W microbatches to every version, one collective step).
This trainer is the straggler-tolerant form for any K: every rank is a client with its own data and
replays its own step at its own pace; the "server" is device memory (csrc/fedsgd_ps.hip):

  fed_pull     the master, copied out of the shards under a version seqlock;
  (forward / backward of the rank's microbatch on exactly that version)
  fed_upload   a ticket for that version (stale / full: dropped), the gradient stored into slot t;
  fed_apply    the K-th gradient to land makes its rank the applier: w -= lr * (sum of the K slots) / K in
               slot order, version + 1.

Client data: each step trains on the rows the caller passes to :meth:`step_indices` (the rank's own
shard, e.g. from a :class:`~distriflow_amd.data.dataset.DistriDataset` dispenser), as
``FederatedClient.DistributedUpdate(x, y)`` trains on the client's own examples
(/root/reference/src/client/federated_client.ts:68-132).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .async_ps import AsyncPSTrainer
from .data_parallel import DataParallelTrainer

# decision codes of the upload (csrc/fedsgd_ps.hip)
ADMITTED, STALE, FULL, FAILED = 1, 2, 3, 4


class FedSGDDeviceTrainer(AsyncPSTrainer):
    SUPPORTS_MULTISTEP = False  # the caller supplies each step's rows (step_indices)

    def __init__(self, net, lr: float = 0.001, min_updates_per_version: int = 20, group=None, server_rank: int = 0,
                 graph: str = "full", timeout_s: float = 30.0, joinable: bool = False):
        super().__init__(net, lr=lr, max_staleness=0, group=group, server_rank=server_rank, graph=graph,
                         timeout_s=timeout_s, owner_apply=False,  # (the FedSGD slots, not the async apply)
                         joinable=joinable)
        self.fused_ps = False  # the generic pull / compute / upload / apply step for every model
        self.K = int(min_updates_per_version)
        if not 1 <= self.K <= 32:
            raise ValueError("min_updates_per_version must be 1..32")
        err, handle = None, b""
        try:
            handle = self.ps.fed_init(self.K)
        except Exception as e:
            err = e
        self._agree(err, "fedsgd slot allocation")
        handles = [handle] * self.world
        if self.world > 1:
            dist.all_gather_object(handles, handle, group=group)
        try:
            self.ps.fed_open(handles)
        except Exception as e:
            err = e
        self._agree(err, "fedsgd slot IPC open")
        self._handles["fed"] = handles
        self._fed_stats_dev = self.ps.fed_stats_tensor()
        self._seq_dev = self.ps.fed_seq_tensor()

    def attach_meta(self) -> dict:
        m = super().attach_meta()
        m["fed_K"] = self.K
        return m

    @classmethod
    def attach(cls, net, store, joiner_id: int, lr=None, graph: str = "full", prefix=None, timeout_s: float = 60.0):
        """A late-joining FedSGD client (parallel/elastic.py): maps the members' shards and gradient slots;
        its first pull is the current version, its uploads take tickets of the current version like a
        member's (reference: a client may connect at any time, federated_server.ts:60-69)."""
        self = super().attach(net, store, joiner_id, lr=lr, graph=graph, prefix=prefix, timeout_s=timeout_s)
        self.fused_ps = False
        self.K = int(self._attach_meta["fed_K"])
        if self.K < 1:
            raise RuntimeError("attach: the published server has no FedSGD slots")
        self._fed_stats_dev = self.ps.fed_stats_tensor()
        self._seq_dev = self.ps.fed_seq_tensor()
        return self

    # ------------------------------------------------------------------ one step
    def _has_schedule(self) -> bool:
        return getattr(self, "data", None) is not None

    def _prime(self):
        pass

    def _gather(self):
        self.ps.fed_pull(self.net.store.master)
        self.net.store.refresh_compute()
        DataParallelTrainer._gather(self)

    def _step_body(self, x, y):
        stats = self.net.compute_gradients(x, y)
        self.ps.fed_upload(self.net.store.grad)
        self.ps.fed_apply(float(self.lr))
        return stats

    @property
    def step_launches(self) -> str:
        return "pull+refresh+compute+upload+apply"

    def step(self):
        raise RuntimeError("FedSGDDeviceTrainer trains on the caller's rows: use step_indices(rows)")

    def step_indices(self, idx: torch.Tensor):
        """One client step on dataset rows ``idx`` (this rank's own data): pull the current version, compute
        the gradient, upload it (admitted, or dropped as stale / beyond the K of its version)."""
        st = DataParallelTrainer.step_indices(self, idx)
        self._after_replay(1)
        return st

    # ------------------------------------------------------------------ callbacks / state
    def _cb_sources(self) -> list:
        return [self.run_stats, self._fed_stats_dev, self._seq_dev]

    def _cb_stats(self, cur, last, v0, v1, n) -> dict:
        d = [cur[1][k] - last[1][k] for k in range(4)]
        return {"version": int(cur[2][0]) // 2, "steps": n, "admitted": int(d[0]), "stale": int(d[1]),
                "full": int(d[2]), "rank": self.rank, "world": self.world}

    def _version_change(self, cur, last, v0, v1):
        """on_new_version(old, new) once for every replay that saw the version move (the reference client
        fires it once per Download of a new version, federated_client.ts:46-53)."""
        old, new = int(last[2][0]) // 2, int(cur[2][0]) // 2
        return (old, new) if new != old else None

    def version(self) -> int:
        """The current model version (host read; syncs)."""
        return int(self.ps.fed_stats()[6]) // 2

    def fed_stats(self) -> dict:
        adm, stale, full, failed, applied, err, seq, recovered = self.ps.fed_stats()
        return {"admitted": adm, "stale": stale, "full": full, "failed": failed, "applied_here": applied,
                "error": err, "version": seq // 2, "recovered": recovered}

    def check_comm(self):
        err = self.ps.fed_stats()[5] | self.ps.stats()[5]
        if err:
            raise RuntimeError(f"device FedSGD: a wait timed out (error bits {err:#x})")
