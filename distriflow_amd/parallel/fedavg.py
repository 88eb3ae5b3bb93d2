"""Federated averaging over one MI355X node: every rank (GPU) is a client with its own non-IID shard,
and weight averaging runs as a collective (BASELINE.json configs[4]).

The reference names federated learning only as an API shape and a stretch goal. Its client uploads one
gradient per ``examplesPerUpdate`` examples (FedSGD; /root/reference/src/client/federated_client.ts:68-132,
/root/reference/README.md:6). The message-level ``FedAvgServer``/``FedAvgClient`` (parallel/server.py,
parallel/worker.py) keep that protocol shape, with local steps added. This trainer is the throughput
path for the same algorithm:

  * each rank runs ``local_steps`` plain SGD steps on its own shard, with NO gradient exchange. Each
    step is a bare replay of the captured graph (gather, forward, loss, backward, fused SGD);
  * a round ends with ``w <- (1/W) sum_k w_k``. That is an in-place all-reduce of the flat fp32
    master: the one-shot xGMI kernel for LeNet-sized models, RCCL above 4 MB. The bf16 compute
    copies are then re-emitted. With equal shard sizes this is exactly FedAvg's example-weighted mean.

Rank 0 is the "server" only in name. Every rank ends a round holding the averaged model, which is
what the server's broadcast achieves in the reference's star topology.
"""
from __future__ import annotations

import torch

from .data_parallel import DataParallelTrainer


class FedAvgTrainer(DataParallelTrainer):
    _step_all_reduces = False  # local steps exchange nothing (the fused LeNet-5 step stays local)

    def __init__(self, net, lr: float = 0.05, local_steps: int = 20, group=None, graph: str = "full",
                 allreduce: str = "auto"):
        super().__init__(net, lr=lr, group=group, overlap=False, graph=graph, allreduce=allreduce)
        self.local_steps = int(local_steps)
        self.rounds = 0
        # local SGD: this rank's own gradient, not a mean over ranks
        net.store.set_hyper(lr, 0.0, 0.0, grad_scale=1.0)

    def set_lr(self, lr: float):
        self.lr = lr
        self.net.store.set_hyper(lr, 0.0, 0.0, grad_scale=1.0)

    # local steps exchange nothing
    def _grad_ready(self, layer_idx: int):
        return

    def _allreduce_all(self):
        return

    def average(self):
        """End of round: every rank's master becomes the mean of all ranks' masters."""
        store = self.net.store
        if self.world > 1:
            self._reduce(store.master, async_op=False)
            store.master.mul_(1.0 / self.world)
        store.refresh_compute()
        self.rounds += 1

    def run_round(self):
        """``local_steps`` captured local steps on the bound index stream, then the average.  The local steps
        run as multi-step graph replays (:meth:`prepare_run`, up to 64 steps per launch): a round of 50 LeNet-5
        steps was 50 graph launches, launch-bound at small batches."""
        if self.graph_mode == "full" and self.net.is_gpu and self._multi_u != min(self.local_steps, 64):
            self.prepare_run(self.local_steps)
        st = self.run(self.local_steps)
        self.average()
        return st
