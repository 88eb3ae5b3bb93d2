"""Logging, timers and a JSONL metrics sink.

Reference: ``log(...)`` prints ``'Distributed Server:' / 'Distributed Client:'`` when verbose and
``time(msg, action)`` logs ``"<msg> took <ms>ms"`` (/root/reference/src/server/abstract_server.ts:92-103,
/root/reference/src/client/abstract_client.ts:138-142,175-180).  Added: a JSONL
metrics sink (one record per event, rank-tagged) and GPU-accurate phase timers (:class:`PhaseTimer`,
hipEvent based) for the fwd / bwd / comm / update breakdown.
"""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Callable, Optional

import torch


class Logger:
    def __init__(self, role: str, verbose: bool = False, metrics_file: Optional[str] = None):
        self.role = role
        self.verbose = verbose
        self.metrics_file = metrics_file or os.environ.get("DISTRIFLOW_METRICS")
        self._fh = None

    def log(self, *args):
        if self.verbose:
            print(f"{self.role}:", *args, file=sys.stdout, flush=True)

    def time(self, msg: str, fn: Callable):
        t1 = time.perf_counter()
        out = fn()
        ms = (time.perf_counter() - t1) * 1e3
        self.log(f"{msg} took {ms:.0f}ms")
        return out

    def metric(self, **rec):
        if not self.metrics_file:
            return
        if self._fh is None:
            d = os.path.dirname(self.metrics_file)
            if d:
                os.makedirs(d, exist_ok=True)
            self._fh = open(self.metrics_file, "a")
        rec.setdefault("ts", time.time())
        rec.setdefault("role", self.role)
        rec.setdefault("rank", int(os.environ.get("RANK", "0")))
        self._fh.write(json.dumps(rec) + "\n")
        self._fh.flush()


class PhaseTimer:
    """Accumulates per-phase GPU time with HIP events (no host sync until :meth:`summary`)."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._events: dict = {}
        self._open: dict = {}

    def start(self, name: str):
        if not self.enabled:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self._open[name] = e

    def stop(self, name: str):
        if not self.enabled or name not in self._open:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self._events.setdefault(name, []).append((self._open.pop(name), e))

    def summary(self) -> dict:
        if not self.enabled:
            return {}
        torch.cuda.synchronize()
        return {k: sum(a.elapsed_time(b) for a, b in v) for k, v in self._events.items()}

    def reset(self):
        self._events.clear()
        self._open.clear()
