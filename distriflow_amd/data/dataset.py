"""DistriDataset — the first-come-first-serve microbatch dispenser of the reference, HBM resident.

Reference: ``DistributedDataset`` (/root/reference/src/server/dataset.ts:5-109):
``next()`` hands out the next incomplete batch of the current epoch, ``completeBatch(b)`` retires it,
batches that were dispensed but never completed are re-dispatched once the cursor runs off the
end (at-least-once), a new epoch starts when every batch is complete, preprocessing callbacks run
on each dispensed batch, and ``batchToDataMSG`` serialises a batch for the wire.

MI355X design: the queue bookkeeping is the native ``BatchDispenser`` (csrc/native_runtime.cpp);
the tensors stay where they are put — typically HBM (288 GB per GPU holds every dataset of the
reference thousands of times over), so a dispensed batch is a device-side slice / index gather, and
in the parameter-server modes only batch ids travel to workers that hold their own resident copy
(``DataMsg.x is None``).  Adds what the reference declares but ignores: ``smallLastBatch`` (ragged
last batch; without it the remainder is dropped instead of crashing), optional per-epoch shuffle,
and a serialisable state for checkpoint/resume.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

import torch

from .. import native
from ..config import dataset_config
from ..protocol import DataMsg, serialize_var


@dataclass
class Batch:
    batch: int
    epoch: int
    x: torch.Tensor
    y: torch.Tensor
    start: int = 0
    size: int = 0
    indices: Optional[torch.Tensor] = None


class DistriDataset:
    def __init__(self, x: torch.Tensor, y: torch.Tensor, config: Optional[dict] = None, shuffle: bool = False,
                 seed: int = 0, device=None):
        if x.shape[0] != y.shape[0]:
            raise ValueError(f"x has {x.shape[0]} rows but y has {y.shape[0]}")
        cfg = dataset_config(config)
        self.config = cfg
        self.x = x.to(device) if device is not None else x
        self.y = y.to(device) if device is not None else y
        self.epochs = int(cfg["epochs"])
        self.batch_size = int(cfg["batchSize"])
        self.small_last_batch = bool(cfg["smallLastBatch"])
        self.shuffle = shuffle
        self._disp = native.require().BatchDispenser(int(x.shape[0]), self.batch_size, self.epochs,
                                                     self.small_last_batch, shuffle, seed)
        self.preprocess_callbacks: list[Callable[[Batch], Batch]] = []

    # reference-compatible names ------------------------------------------------------------
    @property
    def epoch(self) -> int:
        return self._disp.epoch

    @property
    def batches(self) -> int:
        return self._disp.num_batches

    @property
    def remaining(self) -> int:
        return self._disp.remaining

    def next(self):
        """-> (Batch or None, done)."""
        done, b, epoch, start, size = self._disp.next()
        if done:
            return None, True
        batch = self.get_batch(b, epoch)
        return self.preprocess(batch), False

    def next_id(self):
        """Dispense only the batch id/range (no tensor work): -> (batch, epoch, start, size) or None."""
        done, b, epoch, start, size = self._disp.next()
        return None if done else (b, epoch, start, size)

    def complete_batch(self, batch: int, epoch: Optional[int] = None) -> bool:
        return self._disp.complete(int(batch), self.epoch if epoch is None else int(epoch))

    completeBatch = complete_batch

    def example_indices(self, batch: int) -> torch.Tensor:
        return torch.tensor(self._disp.example_indices(int(batch)), dtype=torch.int64)

    def get_batch(self, b: int, epoch: Optional[int] = None) -> Batch:
        start = b * self.batch_size
        size = min(self.batch_size, self.x.shape[0] - start)
        if self.shuffle:
            idx = self.example_indices(b).to(self.x.device)
            x, y = self.x.index_select(0, idx), self.y.index_select(0, idx)
        else:
            idx = None
            x, y = self.x[start: start + size], self.y[start: start + size]
        return Batch(b, self.epoch if epoch is None else epoch, x, y, start, size, idx)

    def preprocess(self, batch: Batch) -> Batch:
        for cb in self.preprocess_callbacks:
            batch = cb(batch)
        return batch

    def add_preprocess_callback(self, cb: Callable[[Batch], Batch]):
        self.preprocess_callbacks.append(cb)

    addPreprocessCallback = add_preprocess_callback

    def index_stream(self, rank: int = 0, world: int = 1, device=None, with_epochs: bool = False,
                     allow_preprocess: bool = False):
        """Device batch schedule for the data-parallel engine (``DataParallelTrainer.bind_distri_dataset``):
        drains the dispenser in its FCFS order over every remaining epoch, giving the k-th dispensed
        full-size batch to rank k % world, and completes each batch as it is scheduled (the sync engine
        applies every step, so at-least-once dispatch is exactly-once here).  Returns this rank's
        [steps][batch_size] int64 example indices (the epochs' shuffles included); every rank gets the
        same number of steps.  A ragged last batch is skipped: a captured step has a fixed shape.
        ``with_epochs``: also return, per step, the dataset epoch of that step's first global batch
        (identical on every rank: epoch boundaries for checkpoints / barriers).
        The stream carries indices only: the preprocess callbacks run on the gathered batch, so a caller
        that applies them itself (``allow_preprocess``: the device engines'
        ``DataParallelTrainer.add_preprocess_callback``) gets the stream; any other caller would drop them
        silently and is refused."""
        if self.preprocess_callbacks and not allow_preprocess:
            raise ValueError("this dataset has preprocess callbacks: bind it with a trainer's bind_distri_dataset "
                             "(which runs them on every device batch) or use the message-level roles")
        rows, epochs, k = [], [], 0
        while True:
            done, b, epoch, start, size = self._disp.next()
            if done:
                break
            if size == self.batch_size:
                if k % world == rank:
                    rows.append(self.example_indices(b))
                if k % world == 0:
                    epochs.append(int(epoch))
                k += 1
            self._disp.complete(int(b), int(epoch))
        steps = k // world
        if steps == 0:
            raise ValueError("the dataset yields no full batch per rank")
        out = torch.stack(rows[:steps]).to(device if device is not None else self.x.device)
        return (out, epochs[:steps]) if with_epochs else out

    def state(self) -> dict:
        return dict(self._disp.state())

    def load_state(self, st: dict):
        self._disp.load_state(st)

    @property
    def done(self) -> bool:
        return self._disp.done


def batch_to_data_msg(batch: Batch, ship_tensors: bool = True) -> DataMsg:
    """Reference ``batchToDataMSG`` (dataset.ts:99-109).  ``ship_tensors=False`` sends only ids/range."""
    if ship_tensors:
        return DataMsg(batch.batch, batch.epoch, serialize_var(batch.x), serialize_var(batch.y), batch.start,
                       batch.size)
    return DataMsg(batch.batch, batch.epoch, None, None, batch.start, batch.size)


# reference names
DistributedDataset = DistriDataset
batchToDataMSG = batch_to_data_msg
