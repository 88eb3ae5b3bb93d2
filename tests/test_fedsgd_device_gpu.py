"""Device FedSGD count barrier with K < W (csrc/fedsgd_ps.hip, parallel/fedsgd_ps.py; VERDICT r4 Missing 5).

Reference FederatedServer (/root/reference/src/server/federated_server.ts:73-90): uploads of the current
version are counted, stale ones dropped; after minUpdatesPerVersion of them the mean is applied and the
version bumped -- the barrier counts updates, not workers, so a slow or lost worker never blocks a
version.  Four processes share the box's GPU (gloo control plane; IPC-mapped shards and slots as on an
8-GPU node): rank 3 uploads its first gradients only after the others moved the version past the one it
pulled (they must be dropped as stale), and rank 2 stops after three steps."""
import os
import tempfile
import time

import pytest
import torch
import torch.multiprocessing as mp

from mp_util import free_port, init_rank

pytestmark = pytest.mark.gpu

N_ROWS, MB, LR = 4096, 64, 0.05


def _rows(rank, steps):
    g = torch.Generator().manual_seed(100 + rank)
    return [torch.randperm(N_ROWS, generator=g)[:MB] for _ in range(steps)]


def _worker(rank, world, port, out_dir, K, steps, slow, dead, dead_after):
    import torch.distributed as dist

    dev = init_rank(rank, world, port)
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.fedsgd_ps import FedSGDDeviceTrainer

    data, labels = synthetic_mnist(N_ROWS, seed=3, device=dev)
    net = build_model("lenet5", device=dev, seed=0)
    tr = FedSGDDeviceTrainer(net, lr=LR, min_updates_per_version=K, graph="full", timeout_s=20.0)
    tr.bind_dataset(data, labels, MB, scale=1.0 / 255.0)
    audit = torch.full((steps, 3), -1, dtype=torch.int32, device=dev)
    tr.ps.set_fed_audit(audit)
    seen = []
    tr.on_new_version(lambda old, new: seen.append((old, new)))
    rows = _rows(rank, steps)
    dist.barrier()
    n = dead_after if rank == dead else steps
    for k in range(n):
        if rank == slow and k < 4:
            # a straggler: it pulls, then computes and uploads only after the others moved the version on
            # (its first steps, while they are still running), so that upload is of a stale version
            tr.idx.copy_(rows[k].to(dev))
            tr._gather()
            torch.cuda.synchronize()
            v0, t0 = tr.version(), time.time()
            while tr.version() == v0 and time.time() - t0 < 5.0:
                time.sleep(0.002)
            tr._step_body(tr.xb, tr.yb)
            torch.cuda.synchronize()
            continue
        tr.step_indices(rows[k].to(dev))
    torch.cuda.synchronize()
    tr.flush_callbacks()
    dist.barrier()  # every rank is done stepping
    res = dict(audit=audit.cpu(), fed=tr.fed_stats(), seen=seen, graph=tr.graph_mode, n=n)
    if rank == 0:
        res["master"] = tr.pull_master(torch.empty_like(net.store.master)).cpu()
        torch.cuda.synchronize()
    torch.save(res, os.path.join(out_dir, f"f{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_device_fedsgd_k_lt_w_straggler_and_lost_rank():
    world, K, steps, slow, dead, dead_after = 4, 2, 24, 3, 2, 3
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, free_port(), d, K, steps, slow, dead, dead_after), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"f{i}.pt"), weights_only=True) for i in range(world)]
    V = r[0]["fed"]["version"]
    assert all(x["fed"]["error"] == 0 for x in r), [x["fed"] for x in r]
    assert r[0]["graph"] == "full"
    # the lost rank (3 steps) never blocked the versions: the others kept closing them
    assert V >= steps // 2, V
    # every closed version holds exactly K admitted gradients of that version, in slots 0 .. K-1
    per_version = {}
    for rank, x in enumerate(r):
        a = x["audit"]
        for k in range(x["n"]):
            seq, dec, slot = (int(v) for v in a[k])
            assert dec in (1, 2, 3), (rank, k, dec)
            if dec == 1:
                per_version.setdefault(seq // 2, []).append((slot, rank, k))
    for v in range(V):
        got = sorted(per_version.get(v, []))
        assert [s for s, _, _ in got] == list(range(K)), (v, got)
    # replay: one engine applying the mean of each version's K admitted microbatch gradients in slot order
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model

    dev = torch.device("cuda", 0)
    data, labels = synthetic_mnist(N_ROWS, seed=3, device=dev)
    net = build_model("lenet5", device=dev, seed=0)
    rows = [_rows(rk, steps) for rk in range(world)]
    w = net.store.master.clone()
    for v in range(V):
        acc = None
        for slot, rk, k in sorted(per_version[v]):
            idx = rows[rk][k].to(dev)
            net.store.set_flat(w)
            x = (data.index_select(0, idx).float() / 255.0).to(torch.bfloat16)
            net.compute_gradients(x, labels.index_select(0, idx))
            g = net.store.grad.clone()
            acc = g if acc is None else acc + g
        with torch.no_grad():
            w = w - LR * (acc * (1.0 / K))
    torch.cuda.synchronize()
    m = r[0]["master"].to(dev)
    rel = ((m - w).abs() / w.abs().clamp_min(1e-3)).max().item()
    assert rel <= 1e-5, f"master relative error {rel:.3e} against the replay of the admitted gradients"
    # the straggler's late uploads were dropped as stale (or past K), never applied to a newer version
    st = r[slow]["fed"]
    assert st["stale"] + st["full"] > 0, st
    # on_new_version: one event per replay that saw the version move, versions strictly increasing
    for x in r:
        news = [n for _, n in x["seen"]]
        assert news == sorted(set(news)) and all(o < n for o, n in x["seen"]), x["seen"]
    print(f"versions {V}; admitted per rank {[x['fed']['admitted'] for x in r]}; "
          f"straggler stale/full {st['stale']}/{st['full']}")


def _recovery_worker(rank, world, port, out_dir, K, mode, target):
    """Rank 0 lands slot 0 of version 0; rank 2 then takes slot 1 and "dies": mode "applier" -- it lands
    (and so claims the apply) but never runs fed_apply; mode "ticket" -- it takes the ticket and stores /
    lands nothing (fault injection).  Ranks 0 and 1 keep stepping until the version reaches ``target``."""
    import torch.distributed as dist

    dev = init_rank(rank, world, port)
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.fedsgd_ps import FedSGDDeviceTrainer

    data, labels = synthetic_mnist(N_ROWS, seed=3, device=dev)
    net = build_model("lenet5", device=dev, seed=0)
    tr = FedSGDDeviceTrainer(net, lr=LR, min_updates_per_version=K, graph="full", timeout_s=2.0)
    tr.bind_dataset(data, labels, MB, scale=1.0 / 255.0)
    cap = 200000
    audit = torch.full((cap, 3), -1, dtype=torch.int32, device=dev)
    tr.ps.set_fed_audit(audit)
    rows = _rows(rank, 64)
    used = []  # the row set of each upload, in audit-row order
    dist.barrier()
    n = 0
    if rank == 0:
        tr.step_indices(rows[0].to(dev))  # slot 0 of version 0
        used.append(0)
        n = 1
    torch.cuda.synchronize()
    dist.barrier()
    if rank == 2:
        tr.idx.copy_(rows[0].to(dev))
        tr._gather()
        tr.net.compute_gradients(tr.xb, tr.yb)
        tr.ps.fed_upload(tr.net.store.grad, drop_land=(mode == "ticket"))  # ... and no fed_apply
        used.append(0)
        n = 1
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.time()
    if rank in (0, 1):
        k = 0
        while tr.version() < target and time.time() - t0 < 90.0 and n < cap:
            tr.step_indices(rows[(k + 1) % len(rows)].to(dev))
            used.append((k + 1) % len(rows))
            k += 1
            n += 1
    torch.cuda.synchronize()
    dist.barrier()
    res = dict(audit=audit[:n].cpu(), fed=tr.fed_stats(), n=n, rows=torch.stack(rows), used=torch.tensor(used, dtype=torch.long))
    if rank == 0:
        res["master"] = tr.pull_master(torch.empty_like(net.store.master)).cpu()
        torch.cuda.synchronize()
    torch.save(res, os.path.join(out_dir, f"f{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["applier", "ticket"])
def test_device_fedsgd_recovers_lost_applier_or_ticket(mode):
    """ADVICE r5 liveness: a rank that stops between its upload and fed_apply (it claimed the apply), or
    between its admission and its landing, no longer wedges the version -- every other upload saw Full for
    ever.  A surviving rank recovers the version after the timeout (missing tickets landed as bad slots and
    left out of the mean; the apply claimed by the survivor), and the master equals the replay of the good
    gradients of every version (reference: a lost worker never blocks a version,
    /root/reference/src/server/federated_server.ts:87-90)."""
    world, K, target = 3, 2, 4
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_recovery_worker, args=(world, free_port(), d, K, mode, target), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"f{i}.pt"), weights_only=True) for i in range(world)]
    V = r[0]["fed"]["version"]
    assert V >= target, [x["fed"] for x in r]
    assert r[0]["fed"]["error"] == 0 and r[1]["fed"]["error"] == 0, [x["fed"] for x in r]
    assert r[0]["fed"]["recovered"] + r[1]["fed"]["recovered"] == 1, [x["fed"] for x in r]
    assert r[2]["fed"]["applied_here"] == 0
    per_version = {}
    for rank, x in enumerate(r):
        a = x["audit"]
        for k in range(x["n"]):
            seq, dec, slot = (int(v) for v in a[k])
            if dec == 1:
                per_version.setdefault(seq // 2, []).append((slot, rank, k))
    v0 = sorted(per_version[0])
    assert [(s, rk) for s, rk, _ in v0] == [(0, 0), (1, 2)], v0
    if mode == "ticket":  # the dead rank's ticket never landed: version 0 is the mean of slot 0 alone
        per_version[0] = v0[:1]
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model

    dev = torch.device("cuda", 0)
    data, labels = synthetic_mnist(N_ROWS, seed=3, device=dev)
    net = build_model("lenet5", device=dev, seed=0)
    rows = {rk: r[rk]["rows"][r[rk]["used"]] for rk in range(world)}
    w = net.store.master.clone()
    for v in range(V):
        got = sorted(per_version[v])
        if v > 0:
            assert [s for s, _, _ in got] == list(range(K)), (v, got)
        acc = None
        for slot, rk, k in got:
            idx = rows[rk][k].to(dev)
            net.store.set_flat(w)
            x = (data.index_select(0, idx).float() / 255.0).to(torch.bfloat16)
            net.compute_gradients(x, labels.index_select(0, idx))
            g = net.store.grad.clone()
            acc = g if acc is None else acc + g
        with torch.no_grad():
            w = w - LR * (acc * (1.0 / len(got)))
    torch.cuda.synchronize()
    m = r[0]["master"].to(dev)
    rel = ((m - w).abs() / w.abs().clamp_min(1e-3)).max().item()
    assert rel <= 1e-5, f"master relative error {rel:.3e} against the replay of the good gradients"
    print(f"{mode}: versions {V}, recovered by {[x['fed']['recovered'] for x in r]}")
