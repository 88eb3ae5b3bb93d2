"""Late-joining workers (elastic scale-up) on the device parameter server and device FedSGD
(parallel/elastic.py; VERDICT r5 Missing 3 / Next 7).

Reference: any client may connect at any time and immediately receives the current weights (plus, in async
mode, a microbatch) -- /root/reference/src/server/federated_server.ts:60-69,
/root/reference/src/server/asynchronousSGD_server.ts:50-63; SURVEY §5.3.  Here a process that is NOT in
the members' process group reads the published IPC handles from a TCPStore, maps the server's device
memory and steps against it.  Members share the box's GPU over gloo (one-GPU pool); the joiner shares it
too, outside any process group."""
import os
import tempfile
import time

import pytest
import torch
import torch.multiprocessing as mp

from mp_util import free_port, init_rank

pytestmark = pytest.mark.gpu

N = 8192


def _grads(seed, steps, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    half = N // 2
    gr = torch.rand(steps, N - half, device=dev, generator=g) * 2 - 1
    gbuf = torch.empty(steps, N, device=dev)
    gbuf[:, :half] = -1.0  # lr 1: every admitted gradient adds exactly 1 to the counter half
    gbuf[:, half:] = gr
    return gbuf, gr


def _bare_proc(idx, members, port, sport, out_dir, max_stale, pre, steps, owner):
    """Members 0 .. members-1 run the bare parameter server (pull, count, upload); process ``members`` joins
    once the version is >= 10, outside the process group."""
    import datetime

    import torch.distributed as dist

    from distriflow_amd import native
    from distriflow_amd.parallel import elastic

    joiner = idx == members
    half = N // 2
    if not joiner:
        dev = init_rank(idx, members, port)
        store = dist.TCPStore("127.0.0.1", sport, is_master=(idx == 0), wait_for_workers=False,
                              timeout=datetime.timedelta(seconds=120))
        ps = native.require().PSComm(idx, members, 0, N, 20.0, joinable=True)
        ctrl = [ps.handle() if idx == 0 else b""]
        sh = ps.shard_handle()
        shards = [sh] * members
        dist.broadcast_object_list(ctrl, src=0)
        dist.all_gather_object(shards, sh)
        ps.open(ctrl[0], shards)
        ring, ohs = 0, None
        if owner:
            ring = max_stale + 2
            oh = ps.owner_init(ring)
            ohs = [oh] * members
            dist.all_gather_object(ohs, oh)
            ps.owner_open(ohs)
        ps.init_master(torch.zeros(N, device=dev))
        dist.barrier()
        if idx == 0:
            elastic.publish(store, {"n": N, "world": members, "server_rank": 0, "max_staleness": max_stale,
                                    "timeout_s": 20.0, "owner_ring": ring, "owner_on": bool(owner), "fed_K": 0},
                            ctrl[0], shards, ohs)
    else:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        store = elastic.store_client("127.0.0.1", sport, timeout_s=120.0)
        ps = elastic.attach_ps(elastic.read(store), joiner_id=members)
        t0 = time.time()
        while ps.stats()[6] < 10 and time.time() - t0 < 60:  # join once >= 10 versions exist
            time.sleep(0.01)
        store.set("joiner/attached", "1")
    nsteps = steps if joiner else pre + steps
    audit = torch.full((nsteps, 3), -1, dtype=torch.int32, device=dev)
    ps.set_audit(audit)
    gbuf, gr = _grads(1000 + idx, nsteps, dev)
    w = torch.empty(N, device=dev)
    inc = torch.empty(nsteps, device=dev)
    for k in range(nsteps):
        if not joiner and k == pre:  # the rest of the members' steps overlap the joiner's
            torch.cuda.synchronize()
            store.wait(["joiner/attached"], datetime.timedelta(seconds=120))
        ps.fetch_pull(w)
        torch.amin(w[:half], 0, out=inc[k])
        ps.apply(gbuf[k], 1.0, max_stale)
    torch.cuda.synchronize()
    res = dict(audit=audit.cpu(), inc=inc.cpu(), gr=gr.cpu(), stats=ps.stats())
    if joiner:
        torch.save(res, os.path.join(out_dir, "joiner.pt"))
        store.set("joiner/done", "1")
        return
    dist.barrier()
    store.wait(["joiner/done"], datetime.timedelta(seconds=120))
    if owner:  # every flagged gradient drained into its shard (any member may drain any shard)
        ps.drain(w)
        torch.cuda.synchronize()
        dist.barrier()
    res["stats"] = ps.stats()  # (after the joiner's last step)
    if idx == 0:
        m = torch.empty(N, device=dev)
        ps.copy_master(m)
        torch.cuda.synchronize()
        res["master"] = m.cpu()
        res["pref"] = ps.owner_prefix() if owner else None
    torch.save(res, os.path.join(out_dir, f"m{idx}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("owner", [False, True])
def test_late_joiner_sees_current_version_and_its_gradients_land(owner):
    """A 3-member job; a 4th process started after >= 10 versions: its first pull already contains >= 10
    admitted updates on every element, it gets gradients admitted under the same staleness bound, and the
    final master equals w0 - lr * (sum of every admitted gradient, members' and joiner's)."""
    members, max_stale, pre, steps = 3, 4, 16, 40
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_bare_proc, args=(members, free_port(), free_port(), d, max_stale, pre, steps, owner),
                 nprocs=members + 1, join=True)
        r = [torch.load(os.path.join(d, f"m{i}.pt"), weights_only=True) for i in range(members)]
        j = torch.load(os.path.join(d, "joiner.pt"), weights_only=True)
    # the joiner's first pull: the current master (>= 10 versions in), not the initial weights
    assert float(j["inc"][0]) >= 10, float(j["inc"][0])
    assert int(j["audit"][0, 1]) >= 10 or int(j["audit"][0, 2]) != 1, j["audit"][0]
    half = N // 2
    expect = torch.zeros(N - half, dtype=torch.float64)
    total = 0
    for x in r + [j]:
        assert x["stats"][5] == 0, x["stats"]
        a = x["audit"]
        for k in torch.nonzero(a[:, 2] == 1).flatten().tolist():
            v, vp, inc = int(a[k, 0]), int(a[k, 1]), float(x["inc"][k])
            assert v - int(inc) <= v - vp <= max_stale, (k, v, vp, inc)
            expect -= x["gr"][k].double()
            total += 1
    j_adm = int((j["audit"][:, 2] == 1).sum())
    assert j_adm > 0, "the joiner never got a gradient admitted"
    assert r[0]["stats"][6] == total
    if owner:
        assert all(p == total for p in r[0]["pref"])
    m = r[0]["master"]
    assert torch.equal(m[:half], torch.full((half,), float(total)))
    torch.testing.assert_close(m[half:].double(), expect, rtol=0, atol=1e-4)
    print(f"{'owner-applies' if owner else 'CAS'}: {total} admitted, joiner {j_adm} of {steps}, "
          f"joiner's first pull contained {int(j['inc'][0])} updates")


def _model_proc(idx, members, port, sport, out_dir, steps):
    """The trainer API: members AsyncPSTrainer(joinable=True).publish(store); the joiner
    AsyncPSTrainer.attach(...) on the fused LeNet-5 step, claiming microbatches from the shared cursor."""
    import datetime

    import torch.distributed as dist

    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel import elastic
    from distriflow_amd.parallel.async_ps import AsyncPSTrainer
    from distriflow_amd.parallel.data_parallel import epoch_permutations

    joiner = idx == members
    if joiner:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        store = elastic.store_client("127.0.0.1", sport, timeout_s=120.0)
    else:
        dev = init_rank(idx, members, port)
        store = dist.TCPStore("127.0.0.1", sport, is_master=(idx == 0), wait_for_workers=False,
                              timeout=datetime.timedelta(seconds=120))
    data, labels = synthetic_mnist(8192, seed=3, device=dev)
    net = build_model("lenet5", device=dev, seed=idx)
    if joiner:
        tr = AsyncPSTrainer.attach(net, store, joiner_id=members, lr=0.05, graph="full")
    else:
        tr = AsyncPSTrainer(net, lr=0.05, max_staleness=4, graph="full", timeout_s=20.0, joinable=True)
        tr.publish(store)
    tr.bind_dataset(data, labels, 256, scale=1.0 / 255.0)
    tr.bind_schedule(epoch_permutations(8192, 256, 32, dev, seed=0))
    if joiner:
        t0 = time.time()
        while tr.ps_stats()["version"] < 10 and time.time() - t0 < 60:
            time.sleep(0.01)
        v_join = tr.ps_stats()["version"]
        store.set("joiner/attached", "1")
    losses = []
    for k in range(steps):
        if not joiner and k == 12:
            torch.cuda.synchronize()
            store.wait(["joiner/attached"], datetime.timedelta(seconds=120))
        st = tr.step()
        losses.append(float(st[0].item()) / 256)
    torch.cuda.synchronize()
    res = dict(tr.ps_stats(), losses=losses, fused=tr.fused_ps, graph=tr.graph_mode)
    if joiner:
        res["v_join"] = v_join
        torch.save(res, os.path.join(out_dir, "joiner.pt"))
        store.set("joiner/done", "1")
        return
    dist.barrier()
    store.wait(["joiner/done"], datetime.timedelta(seconds=120))
    tr.drain()
    torch.cuda.synchronize()
    dist.barrier()
    res.update(tr.ps_stats())
    res["finite"] = bool(torch.isfinite(tr.pull_master()).all())
    torch.save(res, os.path.join(out_dir, f"m{idx}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_late_joiner_trains_lenet_through_the_trainer_api():
    members, steps = 2, 30
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_model_proc, args=(members, free_port(), free_port(), d, steps), nprocs=members + 1, join=True)
        r = [torch.load(os.path.join(d, f"m{i}.pt"), weights_only=True) for i in range(members)]
        j = torch.load(os.path.join(d, "joiner.pt"), weights_only=True)
    assert j["fused"] and j["graph"] == "full" and j["v_join"] >= 10
    assert j["accepted"] > 0, j
    assert all(x["error"] == 0 for x in r) and j["error"] == 0
    acc = sum(x["accepted"] for x in r) + j["accepted"]
    assert r[0]["version"] == acc  # one version per admitted gradient, the joiner's included
    assert r[0]["completed"] + r[0]["duplicates"] == acc
    assert all(x["finite"] for x in r)
    print(f"joiner admitted {j['accepted']} of {steps} (joined at version {j['v_join']}); total {acc}")


@pytest.mark.timeout(240)
def test_launch_join_cli():
    """``launch async --store-port P --wait-joiners 1`` (one member) and ``launch join --store 127.0.0.1:P``
    (a second process, no process group): both train the one FCFS schedule to its end; every batch of every
    epoch completes once (the member's record), the joiner's gradients among them."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    sport = free_port()
    common = ["--model", "lenet5", "--num-examples", "16384", "--batch", "256", "--epochs", "6", "--lr", "0.05"]
    mem = subprocess.Popen([sys.executable, "-m", "distriflow_amd.launch", "--master-port", str(free_port()), "async",
                            *common, "--max-staleness", "4", "--store-port", str(sport), "--wait-joiners", "1"],
                           cwd=root, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        j = subprocess.run([sys.executable, "-m", "distriflow_amd.launch", "join", *common, "--store",
                            f"127.0.0.1:{sport}", "--joiner-id", "5"], cwd=root, env=env, capture_output=True,
                           text=True, timeout=200)
        mo, me = mem.communicate(timeout=200)
    finally:
        if mem.poll() is None:
            mem.kill()
    assert j.returncode == 0, j.stderr[-2000:]
    assert mem.returncode == 0, me[-2000:]
    jo = json.loads([l for l in j.stdout.splitlines() if l.startswith("{")][-1])
    mo = json.loads([l for l in mo.splitlines() if l.startswith("{")][-1])
    assert mo["finished"] and mo["epoch"] == 6 and mo["completed"] == 6 * (16384 // 256), mo
    assert jo["error"] == 0 and mo["error"] == 0
    assert jo["accepted"] > 0, jo
    assert mo["version"] == mo["accepted"] + jo["accepted"]
    print("member accepted", mo["accepted"], "joiner accepted", jo["accepted"], "eval", mo.get("eval_accuracy"))
