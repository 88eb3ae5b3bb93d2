"""Late-joining workers (elastic scale-up) for the device parameter server and device FedSGD.

Reference: the server accepts a client at ANY time -- each ``connection`` immediately receives the current
weights (``DownloadMsg``) and, in async mode, a microbatch of its own; that is the reference's only
membership model (/root/reference/src/server/federated_server.ts:60-69,
/root/reference/src/server/asynchronousSGD_server.ts:50-63; SURVEY §5.3 "Elastic membership").

Here the "server" is device memory: the control buffer (version word, FCFS cursor, completion arrays), the
master shards, the owner-applies inboxes and the FedSGD gradient slots, every one of them IPC-exported by
the member that owns it.  A device PS / FedSGD step contains no collective, so membership of the RCCL world
does not matter for stepping.  The members publish every handle (plus the geometry a joiner must agree on)
in a key-value store -- a ``torch.distributed`` TCPStore; a joiner, a process OUTSIDE the process group, reads
them, maps the buffers (``PSComm(..., joiner=True)``) and steps: its first pull copies the current master
(any version), its claims come from the shared FCFS cursor, its gradients are admitted against the same
staleness bound, exactly as a member's.

Members must be created ``joinable=True`` (a one-rank job would otherwise use the exclusive-writer
shortcuts and cached buffers, which assume nobody else ever touches them).
"""
from __future__ import annotations

import json
from typing import Optional

PREFIX = "distriflow/ps"


def _k(prefix: str, name: str) -> str:
    return f"{prefix}/{name}"


def publish(store, meta: dict, ctrl: bytes, shards: list, inboxes: Optional[list] = None,
            fed: Optional[list] = None, prefix: str = PREFIX):
    """Server rank: write the attach record (meta JSON last, so a joiner that sees it sees everything)."""
    for k, h in enumerate(shards):
        store.set(_k(prefix, f"shard/{k}"), h)
    for k, h in enumerate(inboxes or []):
        store.set(_k(prefix, f"inbox/{k}"), h)
    for k, h in enumerate(fed or []):
        store.set(_k(prefix, f"fed/{k}"), h)
    store.set(_k(prefix, "ctrl"), ctrl)
    store.set(_k(prefix, "meta"), json.dumps(meta))


def read(store, prefix: str = PREFIX, timeout_s: float = 60.0) -> dict:
    """Joiner: wait for the attach record and read it: {meta, ctrl, shards, inboxes, fed}."""
    import datetime

    store.wait([_k(prefix, "meta")], datetime.timedelta(seconds=timeout_s))
    meta = json.loads(store.get(_k(prefix, "meta")))
    w = int(meta["world"])
    rec = {"meta": meta, "ctrl": store.get(_k(prefix, "ctrl")),
           "shards": [store.get(_k(prefix, f"shard/{k}")) for k in range(w)]}
    rec["inboxes"] = [store.get(_k(prefix, f"inbox/{k}")) for k in range(w)] if meta.get("owner_ring", 0) else None
    rec["fed"] = [store.get(_k(prefix, f"fed/{k}")) for k in range(w)] if meta.get("fed_K", 0) else None
    return rec


def attach_ps(rec: dict, joiner_id: int):
    """A bare joiner PSComm over a published server (tests / custom loops): mapped, lr source unset."""
    from .. import native

    m = rec["meta"]
    ps = native.require().PSComm(int(joiner_id), int(m["world"]), int(m["server_rank"]), int(m["n"]),
                                 float(m.get("timeout_s", 30.0)), joiner=True)
    ps.open(rec["ctrl"], rec["shards"])
    if m.get("owner_ring", 0):
        ps.owner_open(rec["inboxes"], enable=bool(m.get("owner_on", False)), ring=int(m["owner_ring"]))
    if m.get("fed_K", 0):
        ps.fed_open(rec["fed"], K=int(m["fed_K"]))
    return ps


def store_client(host: str, port: int, timeout_s: float = 60.0):
    """A TCPStore client (the joiner side; the members' rank 0 hosts the store)."""
    import datetime

    import torch.distributed as dist

    return dist.TCPStore(host, port, is_master=False, timeout=datetime.timedelta(seconds=timeout_s))
