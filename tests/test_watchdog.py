"""Dead-peer / stall detection (parallel/watchdog.py) on CPU.

The multi-process case SIGSTOPs one of three gloo ranks while the others sit in an all-reduce with
it: without the watchdog they would wait for the collective timeout; with it they must leave with
exit code 75 within a few seconds.  The in-process cases check the device-error probe and the
progress-stall path with an observer instead of ``os._exit``."""
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import os, sys, time, datetime
import torch, torch.distributed as dist
from distriflow_amd.parallel.watchdog import start_watchdog
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600))
wd = start_watchdog(rank, world, dead_after_s=3.0, interval_s=0.2)
print("running", flush=True)
x = torch.ones(4)
step = 0
while True:
    dist.all_reduce(x)
    x.fill_(1.0)
    wd.beat(step)
    step += 1
    time.sleep(0.01)
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(120)
def test_stopped_peer_ends_survivors_promptly():
    port = _port()
    env = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="3")
    procs = [subprocess.Popen([sys.executable, "-c", WORKER], env=dict(env, RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(3)]
    try:
        for p in procs:
            line = ""
            while line.strip() != "running":
                line = p.stdout.readline()
                assert line, "worker exited before running"
        time.sleep(1.0)
        os.kill(procs[2].pid, signal.SIGSTOP)  # alive but silent: RCCL/gloo would wait for it forever
        t0 = time.time()
        codes = [procs[r].wait(timeout=60) for r in (0, 1)]
        elapsed = time.time() - t0
        err = procs[0].stderr.read() + procs[1].stderr.read()
    finally:
        for p in procs:
            if p.poll() is None:
                os.kill(p.pid, signal.SIGCONT)
                p.kill()
                p.wait()
    assert codes == [75, 75], err[-2000:]
    assert elapsed < 20, elapsed
    assert "peer rank 2 sent no heartbeat" in err


def _store():
    from torch.distributed import TCPStore

    port = _port()
    return TCPStore("127.0.0.1", port, is_master=True, wait_for_workers=False), port


@pytest.mark.timeout(60)
def test_device_error_probe_fires():
    from distriflow_amd.parallel.watchdog import PeerWatchdog, register_probe, unregister_probe

    store, port = _store()
    seen = []
    flag = {"v": 0}
    register_probe("fake_p2p", lambda: flag["v"])
    try:
        wd = PeerWatchdog(0, 2, dead_after_s=30.0, interval_s=0.05, port=port, prefix="t1",
                          on_fail=seen.append).start()
        store.add("t1/hb/1", 1)  # a live peer
        time.sleep(0.3)
        assert not seen
        flag["v"] = 1
        t0 = time.time()
        while not seen and time.time() - t0 < 5:
            time.sleep(0.02)
        wd.stop()
    finally:
        unregister_probe("fake_p2p")
    assert seen and "fake_p2p" in seen[0]


@pytest.mark.timeout(60)
def test_progress_stall_and_clean_stop():
    from distriflow_amd.parallel.watchdog import PeerWatchdog

    store, port = _store()
    seen = []
    wd = PeerWatchdog(0, 2, dead_after_s=30.0, interval_s=0.05, stall_after_s=0.5, port=port, prefix="t2",
                      on_fail=seen.append).start()
    store.add("t2/hb/1", 1)
    for i in range(5):
        wd.beat(i)
        time.sleep(0.1)
    assert not seen  # progressing
    t0 = time.time()
    while not seen and time.time() - t0 < 5:
        time.sleep(0.02)
    assert seen and "no training progress" in seen[0]
    # a peer that finished normally is not reported dead once its heartbeats stop
    seen.clear()
    wd2 = PeerWatchdog(0, 2, dead_after_s=0.3, interval_s=0.05, port=port, prefix="t3", on_fail=seen.append).start()
    store.add("t3/hb/1", 1)
    store.add("t3/done/1", 1)
    time.sleep(1.0)
    wd2.stop()
    assert not seen


@pytest.mark.timeout(60)
def test_dropped_comm_with_sticky_error_does_not_fire_later_watchdog():
    """a communicator torn down with its sticky error word set must neither stay alive in the
    probe table nor make a later watchdog in the same interpreter exit a healthy job."""
    import gc
    import weakref

    from distriflow_amd.parallel import watchdog as W

    class FakeComm:  # a torn-down P2PComm / PSComm whose host error word stayed set
        err = 1

    c = FakeComm()
    ref = weakref.ref(c)
    key = W.register_owner_probe("fake_comm", c, lambda o: o.err)
    assert key in W._PROBES
    del c
    gc.collect()
    assert ref() is None, "the probe table kept the communicator alive"
    assert key not in W._PROBES
    store, port = _store()
    seen = []
    wd = W.PeerWatchdog(0, 2, dead_after_s=30.0, interval_s=0.05, port=port, prefix="t4", on_fail=seen.append).start()
    store.add("t4/hb/1", 1)
    time.sleep(0.5)
    wd.stop()
    assert not seen
    # keys are unique per registration (id() values get reused)
    a, b = FakeComm(), FakeComm()
    ka = W.register_owner_probe("x", a, lambda o: 0)
    kb = W.register_owner_probe("x", b, lambda o: 0)
    assert ka != kb
    W.clear_probes()
    assert not W._PROBES


@pytest.mark.timeout(60)
def test_mark_done_keeps_watching_peers():
    """shutdown() marks the rank done before its final barrier but keeps watching the peers until then."""
    from distriflow_amd.parallel.watchdog import PeerWatchdog

    store, port = _store()
    seen = []
    wd = PeerWatchdog(0, 2, dead_after_s=0.3, interval_s=0.05, port=port, prefix="t5", on_fail=seen.append).start()
    store.add("t5/hb/1", 1)
    wd.mark_done()
    assert store.add("t5/done/0", 0) == 1
    t0 = time.time()
    while not seen and time.time() - t0 < 5:
        time.sleep(0.02)
    wd.stop()
    assert seen and "peer rank 1" in seen[0]


def test_done_rank_waiting_on_slow_peer_is_not_a_stall():
    """a rank that finished its steps (mark_done) and waits for a slow but live peer longer than
    stall_after_s must not be failed for 'no training progress'; the live peer keeps beating."""
    from distriflow_amd.parallel.watchdog import PeerWatchdog

    store, port = _store()
    seen = []
    wd = PeerWatchdog(0, 2, dead_after_s=5.0, interval_s=0.05, port=port, prefix="t6", stall_after_s=0.2,
                      on_fail=seen.append).start()
    wd.beat(10)  # trained, then finished
    wd.mark_done()
    t0 = time.time()
    while time.time() - t0 < 1.0:  # the peer is slow but alive: its heartbeat advances
        store.add("t6/hb/1", 1)
        time.sleep(0.05)
    wd.stop()
    assert not seen, seen
