"""Client-side example-buffer helpers (reference ``src/client/utils.ts``).

The reference keeps a worker's not-yet-uploaded examples in a tf.js tensor that grows by ``concat`` and
shrinks by ``slice``; tf.js cannot concatenate onto a 0-row tensor, hence its ``concatWithEmptyTensors``
/ ``sliceWithEmptyTensors`` special cases (/root/reference/src/client/utils.ts:22-38), and ``addRows``
accepts either one example or a batch (:40-47).  PyTorch handles empty tensors natively, so these are
thin, shape-checked equivalents; ``FederatedClient`` itself buffers through :class:`ExampleRing`, a
preallocated device FIFO that replaces the concat/slice reallocation of every call.  ``from_event`` (:5-19, one-shot event
with a timeout) maps to :func:`wait_for` over a polling callable.
"""
from __future__ import annotations

import time
from typing import Callable, Optional, Sequence, TypeVar

import torch

T = TypeVar("T")


def concat_with_empty(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``concatWithEmptyTensors``: row-concatenate, where either side may have 0 rows."""
    if a.shape[0] == 0:
        return b.to(a.device, a.dtype) if b.dim() == a.dim() else b.to(a.device, a.dtype).reshape((-1,) + a.shape[1:])
    if b.shape[0] == 0:
        return a
    return torch.cat([a, b.to(a.device, a.dtype)])


def slice_with_empty(a: torch.Tensor, start: int, size: Optional[int] = None) -> torch.Tensor:
    """``sliceWithEmptyTensors``: rows [start, start + size) (to the end when ``size`` is None); an
    out-of-range slice is an empty tensor of the same row shape instead of an error."""
    n = a.shape[0]
    start = min(max(start, 0), n)
    end = n if size is None else min(start + size, n)
    return a[start:end]


def add_rows(existing: torch.Tensor, new: torch.Tensor, unit_shape: Sequence[int]) -> torch.Tensor:
    """``addRows``: append one example (shape == unit_shape) or a batch ([k, *unit_shape])."""
    unit_shape = tuple(unit_shape)
    if tuple(new.shape) == unit_shape:
        new = new.unsqueeze(0)
    elif tuple(new.shape[1:]) != unit_shape:
        raise ValueError(f"rows of shape {tuple(new.shape[1:])} do not match unit shape {unit_shape}")
    return concat_with_empty(existing, new)


class ExampleRing:
    """Preallocated FIFO of examples on the model's device: the worker-side buffer of
    ``FederatedClient.DistributedUpdate`` (/root/reference/src/client/federated_client.ts:70-86,
    125-130 grows a tensor with ``concat`` and drops uploaded rows with ``slice`` on every call).

    Rows live in one ``[capacity, *unit_shape]`` tensor addressed by ``head`` / ``count`` modulo the
    capacity: :meth:`push` copies new rows into the free slots (two copies when they wrap), :meth:`peek`
    returns the oldest ``n`` rows as a view when they are contiguous (one gather into a scratch tensor
    when they wrap), :meth:`pop` only advances ``head``.  Capacity doubles (one copy, rows re-linearised)
    only when a push does not fit, so steady-state streaming allocates nothing."""

    def __init__(self, unit_shape: Sequence[int], dtype=torch.float32, device="cpu", capacity: int = 64):
        self.unit_shape = tuple(unit_shape)
        self.buf = torch.empty((max(1, capacity),) + self.unit_shape, dtype=dtype, device=device)
        self.head = 0
        self.count = 0
        self._scratch: Optional[torch.Tensor] = None
        self.grows = 0

    @property
    def capacity(self) -> int:
        return self.buf.shape[0]

    def __len__(self) -> int:
        return self.count

    def _grow(self, need: int):
        cap = self.capacity
        while cap < need:
            cap *= 2
        nb = torch.empty((cap,) + self.unit_shape, dtype=self.buf.dtype, device=self.buf.device)
        if self.count:
            nb[: self.count] = self.peek(self.count)
        self.buf, self.head = nb, 0
        self.grows += 1

    def push(self, rows: torch.Tensor):
        """Append one example (shape == unit_shape) or a batch ``[k, *unit_shape]`` (reference addRows)."""
        if tuple(rows.shape) == self.unit_shape:
            rows = rows.unsqueeze(0)
        elif tuple(rows.shape[1:]) != self.unit_shape:
            raise ValueError(f"rows of shape {tuple(rows.shape[1:])} do not match unit shape {self.unit_shape}")
        k = rows.shape[0]
        if k == 0:
            return
        if self.count + k > self.capacity:
            self._grow(self.count + k)
        cap = self.capacity
        tail = (self.head + self.count) % cap
        first = min(k, cap - tail)
        self.buf[tail: tail + first] = rows[:first]
        if first < k:
            self.buf[: k - first] = rows[first:]
        self.count += k

    def peek(self, n: int) -> torch.Tensor:
        """The oldest ``n`` rows (a view unless they wrap around the end of the storage)."""
        if n > self.count:
            raise IndexError(f"peek({n}) with {self.count} rows buffered")
        cap = self.capacity
        if self.head + n <= cap:
            return self.buf[self.head: self.head + n]
        if self._scratch is None or self._scratch.shape[0] < n:
            self._scratch = torch.empty((max(n, 1),) + self.unit_shape, dtype=self.buf.dtype, device=self.buf.device)
        first = cap - self.head
        out = self._scratch[:n]
        out[:first] = self.buf[self.head:]
        out[first:] = self.buf[: n - first]
        return out

    def pop(self, n: int):
        if n > self.count:
            raise IndexError(f"pop({n}) with {self.count} rows buffered")
        self.head = (self.head + n) % self.capacity
        self.count -= n
        if self.count == 0:
            self.head = 0


def wait_for(poll: Callable[[], Optional[T]], timeout: float, what: str = "event", interval: float = 0.0) -> T:
    """``fromEvent``: block until ``poll()`` returns a value, or raise ``TimeoutError`` after ``timeout`` s."""
    deadline = time.monotonic() + timeout
    while True:
        v = poll()
        if v is not None:
            return v
        if time.monotonic() > deadline:
            raise TimeoutError(f"timed out after {timeout}s waiting for {what}")
        if interval:
            time.sleep(interval)
