"""Client-side example-buffer helpers (reference ``src/client/utils.ts``).

The reference keeps a worker's not-yet-uploaded examples in a tf.js tensor that grows by ``concat`` and
shrinks by ``slice``; tf.js cannot concatenate onto a 0-row tensor, hence its ``concatWithEmptyTensors``
/ ``sliceWithEmptyTensors`` special cases (/root/reference/src/client/utils.ts:22-38), and ``addRows``
accepts either one example or a batch (:40-47).  PyTorch handles empty tensors natively, so these are
thin, shape-checked equivalents used by ``FederatedClient``.  ``from_event`` (:5-19, one-shot event
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
