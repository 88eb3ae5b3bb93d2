"""Dead-peer / stall detection that ends a rank promptly and non-zero.

The reference's parameter server tolerates lost workers by construction: its sync barrier counts
accepted uploads, not workers, and a ``disconnect`` only decrements a counter
(/root/reference/src/server/federated_server.ts:64-67, 87-90).  An RCCL world is fixed-membership
instead: if a rank dies, its peers block inside the next collective until the process-group
timeout (600 s, ``parallel/comm.py``), and the device-side waits of the one-shot all-reduce and the
async parameter server only set a sticky error word.  This watchdog turns all of those into a
prompt exit that a restart loop (``launch.py --max-restarts``, torchrun) can act on:

  * **liveness**: a daemon thread bumps ``<prefix>/hb/<rank>`` in the job's TCPStore every
    ``interval_s`` over its own client connection, and reads every peer's counter.  A peer whose
    counter has not moved for ``dead_after_s`` (killed, SIGSTOPped, or its host gone), or a store
    that stays unreachable that long (rank 0 hosting it died), is a dead peer;
  * **device errors**: registered probes read host-mapped error words that the kernels write with
    system-scope stores (``P2PComm.host_error``, ``PSComm.host_error``), so a device-side peer
    timeout is seen even while the GPU is still busy, with no HIP call from this thread;
  * **progress** (optional): ``beat(step)`` from the training loop; no new step for
    ``stall_after_s`` means this rank is stuck (e.g. in a collective whose peer hangs while alive).

On any of these the rank prints one line to stderr and leaves with ``os._exit(exit_code)`` (75 by
default), from the watchdog thread, because the main thread may be blocked in a collective.  It
never execs.  A rank that finishes normally calls :meth:`stop`, which marks it done so that peers
still shutting down do not count it as dead.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from typing import Callable, Dict, Optional

_PROBES: Dict[str, Callable[[], int]] = {}
_ACTIVE: Optional["PeerWatchdog"] = None


def register_probe(name: str, fn: Callable[[], int]):
    """Register a device error word reader (returns non-zero on error).  Must not call into HIP."""
    _PROBES[name] = fn


def unregister_probe(name: str):
    _PROBES.pop(name, None)


def clear_probes():
    """Forget every probe (end of a job inside a long-lived interpreter: tests, in-process restarts)."""
    _PROBES.clear()


_PROBE_SEQ = [0]


def register_owner_probe(kind: str, owner, read: Callable[[object], int]) -> str:
    """Register a probe that holds only a weak reference to ``owner``: it reads ``read(owner)`` while the
    owner lives and unregisters itself once the owner is collected, so a torn-down communicator (and its
    sticky error word) can neither be kept alive by the watchdog nor fire it later.  Returns the key
    (unique per registration, unlike ``id()`` values, which the interpreter reuses)."""
    import weakref

    _PROBE_SEQ[0] += 1
    key = f"{kind}#{_PROBE_SEQ[0]}"
    ref = weakref.ref(owner, lambda _r, k=key: _PROBES.pop(k, None))

    def probe() -> int:
        o = ref()
        return 0 if o is None else int(read(o))

    _PROBES[key] = probe
    return key


def active() -> Optional["PeerWatchdog"]:
    return _ACTIVE


def beat(step: int):
    """Progress beat for the active watchdog (no-op without one)."""
    if _ACTIVE is not None:
        _ACTIVE.beat(step)


class PeerWatchdog:
    def __init__(self, rank: int, world: int, dead_after_s: Optional[float] = None, interval_s: float = 0.5,
                 stall_after_s: Optional[float] = None, exit_code: int = 75, host: Optional[str] = None,
                 port: Optional[int] = None, prefix: Optional[str] = None, on_fail: Optional[Callable] = None):
        self.rank, self.world = rank, world
        env_dead = os.environ.get("DISTRIFLOW_DEAD_AFTER_S")
        self.dead_after_s = float(dead_after_s if dead_after_s is not None else (env_dead or 30.0))
        env_stall = os.environ.get("DISTRIFLOW_STALL_AFTER_S")
        self.stall_after_s = stall_after_s if stall_after_s is not None else (float(env_stall) if env_stall else None)
        self.interval_s = interval_s
        self.exit_code = exit_code
        self.host = host or os.environ.get("MASTER_ADDR", "127.0.0.1")
        self.port = int(port or os.environ.get("MASTER_PORT", "29500"))
        restart = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
        self.prefix = prefix or f"dfa/wd/{restart}"
        self.on_fail = on_fail
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._store = None
        self._step = -1
        self._step_t = time.monotonic()
        self._done_marked = False
        self.failure: Optional[str] = None

    # ------------------------------------------------------------------ public
    def start(self) -> "PeerWatchdog":
        global _ACTIVE
        from torch.distributed import TCPStore

        self._store = TCPStore(self.host, self.port, is_master=False, timeout=_td(max(5.0, self.dead_after_s)))
        self._store.add(self._key("hb", self.rank), 1)
        self._thread = threading.Thread(target=self._run, name="dfa-watchdog", daemon=True)
        self._thread.start()
        _ACTIVE = self
        return self

    def beat(self, step: int):
        if step != self._step:
            self._step = step
            self._step_t = time.monotonic()

    def mark_done(self):
        """This rank completed normally: peers stop counting its heartbeat.  The thread keeps watching
        the peers (shutdown() calls this BEFORE its final barrier, so a peer that dies while the others
        wait there is still caught within ``dead_after_s``)."""
        if self._done_marked:
            return
        self._done_marked = True
        try:
            if self._store is not None:
                self._store.add(self._key("done", self.rank), 1)
        except Exception:
            pass

    def stop(self):
        """Normal completion: mark this rank done (peers stop watching it) and end the thread."""
        global _ACTIVE
        self.mark_done()
        self._stop.set()
        if self._thread is not None:
            self._thread.join(5 * self.interval_s + 1.0)
        if _ACTIVE is self:
            _ACTIVE = None

    # ------------------------------------------------------------------ thread
    def _key(self, kind: str, r: int) -> str:
        return f"{self.prefix}/{kind}/{r}"

    def _fail(self, why: str):
        self.failure = why
        msg = f"[watchdog] rank {self.rank}: {why}; exiting with {self.exit_code}"
        print(msg, file=sys.stderr, flush=True)
        if self.on_fail is not None:  # tests: observe instead of exiting
            self.on_fail(why)
            self._stop.set()
            return
        os._exit(self.exit_code)

    def _run(self):
        now = time.monotonic()
        last_val = {r: -1 for r in range(self.world) if r != self.rank}
        last_seen = {r: now for r in last_val}
        done = set()
        store_ok_t = now
        while not self._stop.wait(self.interval_s):
            now = time.monotonic()
            for name, fn in list(_PROBES.items()):
                try:
                    v = int(fn())
                except Exception:
                    v = 0
                if v:
                    return self._fail(f"device error word {name} = {v:#x} (peer timed out on the device)")
            # a rank that finished (waiting for slow peers in the final barrier, evaluating, checkpointing)
            # makes no training progress by design: only the peers' liveness is watched then
            if (self.stall_after_s is not None and not self._done_marked and self._step >= 0
                    and now - self._step_t > self.stall_after_s):
                return self._fail(f"no training progress for {now - self._step_t:.0f} s (step {self._step})")
            try:
                self._store.add(self._key("hb", self.rank), 1)
                for r in last_val:
                    if r in done:
                        continue
                    v = self._store.add(self._key("hb", r), 0)
                    if v != last_val[r]:
                        last_val[r], last_seen[r] = v, now
                    elif now - last_seen[r] > self.dead_after_s:
                        if self._store.add(self._key("done", r), 0) > 0:
                            done.add(r)
                            continue
                        return self._fail(f"peer rank {r} sent no heartbeat for {now - last_seen[r]:.1f} s")
                store_ok_t = now
            except Exception as e:  # store host (rank 0 / launcher agent) gone
                if now - store_ok_t > self.dead_after_s:
                    return self._fail(f"rendezvous store unreachable for {now - store_ok_t:.1f} s ({e!r:.120})")


def _td(s: float):
    import datetime

    return datetime.timedelta(seconds=s)


def start_watchdog(rank: int, world: int, **kw) -> Optional[PeerWatchdog]:
    """Start a watchdog for a multi-rank job (None for one rank or ``DISTRIFLOW_WATCHDOG=0``)."""
    if world <= 1 or os.environ.get("DISTRIFLOW_WATCHDOG", "1") == "0":
        return None
    return PeerWatchdog(rank, world, **kw).start()
