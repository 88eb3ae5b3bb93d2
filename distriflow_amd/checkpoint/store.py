"""Versioned checkpoint directories with a ``current`` symlink, plus a resume record.

Reference behaviour (/root/reference/src/server/models.ts:17-30, 98-151):
``<saveDir>/<version>/`` per model version, ``<saveDir>/current -> <version>``, resume = load the
last version.  Fixed here: ``list`` no longer drops every entry after
``current`` (``splice(idx)`` bug), versions are strictly increasing even when two saves land in the
same millisecond, the symlink swap is atomic (rename), and ``keep_last`` bounds disk growth (the
reference writes a full checkpoint on every version forever).

The resume record (``resume.json``) stores what the reference never saved: the model version, the
dataset dispenser state (epoch, incomplete microbatches, shuffle permutation) and optimizer-state
locations, so an interrupted run continues exactly where it stopped.
"""
from __future__ import annotations

import json
import os
import shutil
import time
from typing import Optional

CURRENT = "current"
RESUME = "resume.json"


def _vkey(v: str):
    return (0, int(v), v) if v.isdigit() else (1, 0, v)


def force_symlink(target: str, link: str):
    tmp = f"{link}.tmp{os.getpid()}"
    if os.path.lexists(tmp):
        os.remove(tmp)
    os.symlink(target, tmp)
    os.replace(tmp, link)


class VersionedStore:
    def __init__(self, save_dir: str, keep_last: Optional[int] = None):
        self.save_dir = os.path.abspath(save_dir)
        self.keep_last = keep_last
        self._last_issued = 0

    def setup(self):
        os.makedirs(self.save_dir, exist_ok=True)

    def list(self) -> list[str]:
        if not os.path.isdir(self.save_dir):
            return []
        vs = [d for d in os.listdir(self.save_dir)
              if d != CURRENT and not d.startswith(".") and os.path.isdir(os.path.join(self.save_dir, d))
              and not os.path.islink(os.path.join(self.save_dir, d))]
        return sorted(vs, key=_vkey)

    def last(self) -> Optional[str]:
        vs = self.list()
        return vs[-1] if vs else None

    def new_version(self) -> str:
        """Millisecond timestamp like the reference (Date.now()), but strictly increasing."""
        last = self.last()
        floor = max(self._last_issued, int(last) if last and last.isdigit() else 0)
        v = max(int(time.time() * 1000), floor + 1)
        self._last_issued = v
        return str(v)

    def path(self, version: str) -> str:
        return os.path.join(self.save_dir, version)

    def mark_current(self, version: str):
        force_symlink(version, os.path.join(self.save_dir, CURRENT))

    def current(self) -> Optional[str]:
        link = os.path.join(self.save_dir, CURRENT)
        if os.path.islink(link):
            return os.readlink(link)
        return None

    def prune(self):
        if not self.keep_last:
            return
        vs = self.list()
        cur = self.current()
        for v in vs[: max(0, len(vs) - self.keep_last)]:
            if v != cur:
                shutil.rmtree(self.path(v), ignore_errors=True)

    # ------------------------------------------------------------------ resume record
    def write_resume(self, record: dict):
        self.setup()
        p = os.path.join(self.save_dir, RESUME)
        with open(p + ".tmp", "w") as f:
            json.dump(record, f)
        os.replace(p + ".tmp", p)

    def read_resume(self) -> Optional[dict]:
        p = os.path.join(self.save_dir, RESUME)
        if not os.path.exists(p):
            return None
        with open(p) as f:
            return json.load(f)
