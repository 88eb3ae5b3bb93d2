#!/usr/bin/env python3
"""Headline benchmark: images/sec (whole node) of MNIST CNN synchronous data-parallel SGD on MI355X.

BASELINE.json metric "images/sec (whole node), MNIST CNN sync-SGD at 1/2/4/8 MI355X" on config
"MNIST LeNet-5 CNN sync all-reduce SGD bf16 on 8xMI355X".  Synthetic MNIST-shaped data (60,000 x
28x28x1 uint8, HBM resident) and random-init weights; every timed step is the full training step:
batch gather, forward, fused softmax-CE, backward, RCCL all-reduce of the gradients, fused SGD update.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--model lenet5] [--batch-per-gpu B]
For N > 1 either launch with torch.distributed.run (one rank per GPU), or run it plainly: with
WORLD_SIZE unset, ``--gpus N`` makes this process a launcher that starts N fresh rank processes
(before anything touches the GPU) and exits with the first failing child's code.  Rank 0 prints
one JSON line; ``world`` / ``backend`` in it come from the live process group.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec (whole node), MNIST CNN sync-SGD at 1/2/4/8 MI355X; async speedup"
BASELINE_VALUE = None  # the reference publishes no number


def _spawn_ranks(n: int) -> int:
    """Launcher mode (``--gpus N`` without torchrun): N child processes of this script with
    torchrun-style env.  Runs before any HIP call in this process, and never execs.  On the first
    child failure the survivors are stopped (their exact PIDs) and that exit code is returned."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n))
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r))) for r in range(n)]
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0] if bad[0] > 0 else 128 - bad[0]
            break
        if all(c == 0 for c in codes):
            return 0
        time.sleep(0.1)
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    deadline = time.time() + 30
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    print(f"bench: a rank exited with {rc}; job stopped", file=sys.stderr, flush=True)
    return rc


# every fused fast path off: the per-layer kernels and the BatchNorm statistics passes (the guard's
# reference engine)
_UNFUSED = "lenet_fused=0,kcnn_fused=0,khead_fused=0,fold_dropout=0,bn_acc=0"


def correctness_guard(model: str, B: int, dev, data, labels) -> dict:
    """One training step's gradient of the benchmarked engine against the per-layer kernels (every fused
    path off) on the same weights and the same B-image batch of the benchmark's data: the flat-gradient
    cosine and the loss must agree.  Catches a fast but wrong kernel at the benchmarked shape."""
    from distriflow_amd.models.zoo import build_model

    torch.manual_seed(1234)
    idx = torch.randint(0, data.shape[0], (B,), device=dev)
    x = (data[idx].float() / 255.0).to(torch.bfloat16).float()
    y = labels[idx].to(torch.int32)
    fast = build_model(model, device=dev, seed=0)
    old = os.environ.get("DISTRIFLOW_DIAG")
    os.environ["DISTRIFLOW_DIAG"] = ",".join(v for v in (old, _UNFUSED) if v)
    try:
        ref = build_model(model, device=dev, seed=0)
    finally:
        if old is None:
            os.environ.pop("DISTRIFLOW_DIAG", None)
        else:
            os.environ["DISTRIFLOW_DIAG"] = old
    ref.store.set_flat(fast.store.master)
    s_fast = fast.compute_gradients(x, y).float().cpu()
    g_fast = fast.store.grad.double().clone()
    s_ref = ref.compute_gradients(x, y).float().cpu()
    g_ref = ref.store.grad.double()
    cos = float((g_fast @ g_ref) / (g_fast.norm() * g_ref.norm() + 1e-30))
    rel = float((g_fast - g_ref).norm() / (g_ref.norm() + 1e-30))
    lf, lr_ = float(s_fast[0]) / B, float(s_ref[0]) / B
    finite = bool(torch.isfinite(g_fast).all()) and bool(torch.isfinite(s_fast).all())
    # bf16 activations: the two engines round at different points (fused layers keep more in fp32)
    ok = finite and cos >= 0.99 and abs(lf - lr_) <= 0.02 * abs(lr_) + 1e-3
    out = {"ok": ok, "grad_cosine": round(cos, 6), "grad_rel_l2": round(rel, 6), "loss": round(lf, 6),
           "loss_per_layer": round(lr_, 6), "finite": finite, "batch": B, "reference": "per-layer kernels"}
    if model in _ORACLE_MODELS:
        # ResNet-18's fused and per-layer engines share the halo / igemm64 conv kernels (only the BatchNorm path
        # differs), so its gradient is ALSO checked against a different implementation: the CPU engine on plain
        # PyTorch fp32 ops (bf16 activation buffers, the GPU engine's rounding points), same bf16-representable
        # weights, the first images of the batch
        out["oracle"] = _cpu_oracle(model, build_model(model, device=dev, seed=0), x, y, min(B, _ORACLE_MODELS[model]))
        out["ok"] = out["ok"] and out["oracle"]["ok"]
    return out


_ORACLE_MODELS = {"resnet18_cifar": 64, "keras_cnn": 256}


def _cpu_oracle(model, fast, x, y, Bo) -> dict:
    """``fast``: a freshly built GPU engine (its dropout counters at the start, like the CPU engine's: both draw
    the same counter-based masks)."""
    from distriflow_amd.models.net import Net
    from distriflow_amd.models.zoo import MODELS

    layers, shape = MODELS[model]()
    c = Net(layers, shape, device="cpu", name=model, seed=0, compute_dtype=torch.bfloat16)
    w = fast.store.master.to(torch.bfloat16).float()
    fast.store.set_flat(w)
    c.store.master.copy_(w.cpu())
    # (labels past the model's classes -- the 5-class reference CNN on 10-class data -- are clamped by the
    # GPU loss kernels; the CPU loss indexes them, so both sides get the clamped labels)
    xo, yo = x[:Bo].contiguous(), y[:Bo].clamp(max=fast.num_classes - 1).contiguous()
    s_f = fast.compute_gradients(xo, yo).float().cpu()
    g_f = fast.store.grad.double().cpu()
    s_c = c.compute_gradients(xo.cpu(), yo.cpu()).float()
    g_c = c.store.grad.double()
    cos = float((g_f @ g_c) / (g_f.norm() * g_c.norm() + 1e-30))
    rel = float((g_f - g_c).norm() / (g_c.norm() + 1e-30))
    lf, lc = float(s_f[0]) / Bo, float(s_c[0]) / Bo
    # measured: ResNet-18 0.984 at 64 images (bf16 rounding compounds over 20 conv + BN layers; per-tensor
    # cosines 0.97-1.0, tests/test_engine_gpu.py::test_model_gradients_match_cpu)
    ok = bool(torch.isfinite(g_f).all()) and cos >= 0.97 and abs(lf - lc) <= 0.02 * abs(lc) + 1e-2
    return {"ok": ok, "grad_cosine": round(cos, 6), "grad_rel_l2": round(rel, 6), "loss": round(lf, 6),
            "loss_cpu": round(lc, 6), "batch": Bo, "reference": "cpu engine, plain PyTorch fp32 ops"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", default="lenet5")
    ap.add_argument("--batch-per-gpu", type=int, default=4096)
    ap.add_argument("--lr", type=float, default=0.001)
    ap.add_argument("--graph", default="full", choices=["full", "split", "none"],
                    help="hipGraph mode: full = whole step incl. bucketed RCCL all-reduces (falls back to split "
                         "= captured compute + SGD with an eager all-reduce between, then none, if capture fails)")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--allreduce", default="auto", choices=["auto", "p2p", "rccl"],
                    help="gradient all-reduce: one-shot xGMI kernel for small buckets (auto/p2p) or RCCL only")
    ap.add_argument("--mode", default="sync", choices=["sync", "async"],
                    help="sync = all-reduce data parallel (headline); async = device-resident bounded-staleness "
                         "parameter server on rank 0 (parallel/async_ps.py)")
    ap.add_argument("--max-staleness", type=int, default=4)
    ap.add_argument("--settle-ms", type=float, default=40.0,
                    help="before the W warm-up steps, run untimed training steps (whole K-step replays) for about this "
                         "long: the GPU's clocks ramp up over the first ~15 ms of continuous load after idle "
                         "(profiles/r6/lenet_clock_ramp_r6.txt), so without it a short timed run measures the ramp; "
                         "0 disables; reported as \"settle\" in the JSON")
    ap.add_argument("--async-steps", type=int, default=None,
                    help="after the sync measurement, also time this many steps of the async parameter-server "
                         "engine and report the async speedup (default: --steps; 0 disables)")
    ap.add_argument("--json-extra", action="store_true", help="add diagnostic fields")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the correctness guard (1-step gradient vs the per-layer kernels); the loss and "
                         "finiteness checks of the timed run always run")
    ap.add_argument("--phases", type=int, default=0,
                    help="after timing, run this many EAGER steps with hipEvent phase timers and report the "
                         "data/compute/comm/update breakdown (diagnostic, not part of the timed number)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn_ranks(args.gpus))

    from distriflow_amd.data.dataset import DistriDataset
    from distriflow_amd.diagnostics import active as diag_active, on as diag_on
    from distriflow_amd.data.synthetic import synthetic_cifar10, synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.comm import init_distributed, shutdown
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer, epoch_permutations

    env = init_distributed(watchdog=True)  # a lost rank ends the job promptly (parallel/watchdog.py)
    world, rank = env.world_size, env.rank
    live_world = dist.get_world_size() if dist.is_initialized() else 1
    live_backend = dist.get_backend() if dist.is_initialized() else "none"
    if args.gpus != world or live_world != world:
        print(f"bench: --gpus {args.gpus} but the process group has {live_world} ranks "
              f"(WORLD_SIZE={world}); refusing to report a mislabelled number", file=sys.stderr, flush=True)
        sys.exit(3)
    dev = env.device

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
    net = build_model(args.model, device=dev, seed=0)
    B = args.batch_per_gpu
    # ONE dataset (same seed on every rank), sharded by the dispenser: rank r trains on the FCFS
    # microbatches k with k % world == r (DistriDataset.index_stream)
    if args.model == "resnet18_cifar":
        data, labels = synthetic_cifar10(50000, seed=0, device=dev)
    else:
        data, labels = synthetic_mnist(60000, seed=0, device=dev)
    SETTLE_MAX_STEPS = 1024  # cap of the settle phase's steps (the datasets below are sized for it)
    total = args.warmup + args.steps + (SETTLE_MAX_STEPS if args.settle_ms > 0 else 0)

    def make_trainer(mode, net):
        if mode == "async":
            from distriflow_amd.parallel.async_ps import AsyncPSTrainer

            tr = AsyncPSTrainer(net, lr=args.lr, max_staleness=args.max_staleness, graph=args.graph)
            tr.bind_dataset(data, labels, B, scale=1.0 / 255.0)
            # one global FCFS microbatch table; ranks claim ids from the shared counter
            tr.bind_schedule(epoch_permutations(data.shape[0], B, max(total, data.shape[0] // B), dev, seed=0))
        else:
            tr = DataParallelTrainer(net, lr=args.lr, graph=args.graph, overlap=not args.no_overlap,
                                     allreduce=args.allreduce)
            # device-resident batch schedule: this rank's share of the one DistriDataset (FCFS dispenser,
            # per-epoch shuffle); each step's update launch stages the next step's indices
            epochs = -(-total * world // (data.shape[0] // B))
            ds = DistriDataset(data, labels, {"batchSize": B, "epochs": epochs}, shuffle=True, seed=0)
            tr.bind_distri_dataset(ds, rank=rank, world=world, scale=1.0 / 255.0)
        return tr

    settle_recs = []

    def settle(tr, steps, multi):
        """Untimed training steps (replays of the timed run's own multi-step graph) until about
        ``--settle-ms`` of continuous device work: the clock ramp after idle is ~15 ms long
        (``scripts/launch_overhead_probe.py --ramp``: LeNet-5 B = 4096 62.4 -> 57.1 us per step), so a
        short timed run would measure the power manager's ramp, not the step.  Every rank runs the same
        number of chunks (rank 0 decides after each one): the steps are complete training steps, with the
        same collectives on every rank."""
        if args.settle_ms <= 0 or dev.type != "cuda":
            return
        u = getattr(tr, "_multi_u", 0) if multi else 0
        chunk = u if u > 1 else max(1, min(steps, 16))  # one multi-step replay, or up to 16 single steps
        n, chunks = 0, 0
        t0 = time.perf_counter()
        while True:
            if u > 1:
                tr.run(chunk)
            else:
                for _ in range(chunk):
                    tr.step()
            n += chunk
            chunks += 1
            sync()
            go = (time.perf_counter() - t0) * 1e3 < args.settle_ms and n + chunk <= SETTLE_MAX_STEPS
            if world > 1:
                f = torch.tensor([1 if go else 0], dtype=torch.int32, device=dev)
                dist.broadcast(f, src=0)
                go = bool(f.item())
            if not go:
                break
        settle_recs.append({"steps": n, "replays": chunks, "ms": round((time.perf_counter() - t0) * 1e3, 1)})

    def timed(tr, steps):
        """Settle (see :func:`settle`), W untimed warm-up steps, then ``steps`` timed ones between barrier +
        device syncs; max over ranks.  The sync trainer replays its steps from multi-step hipGraphs (captured
        here, before timing)."""
        multi = getattr(tr, "SUPPORTS_MULTISTEP", False) and diag_on("multistep")
        # ranks time-sharing one device (rehearsals) must yield the GPU at graph boundaries: a long unrolled
        # graph whose one-shot all-reduce spins on a descheduled peer's flag runs at the hardware
        # scheduler's time-slice (measured: 4 ranks on one GPU, 0.48 -> 14.9 ms per step)
        if world > 1 and dev.type == "cuda" and torch.cuda.device_count() < world:
            multi = False
        if multi:
            tr.prepare_run(steps)
        settle(tr, steps, multi)
        if multi:
            tr.run(args.warmup)
        else:
            for _ in range(args.warmup):
                tr.step()
        sync()
        if world > 1:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        if multi:
            st = tr.run(steps)
        else:
            for _ in range(steps):
                st = tr.step()
        sync()
        if world > 1:
            dist.barrier()
        sync()
        el = time.perf_counter() - t0
        tr.check_comm()  # sticky device timeout flags (never set on a healthy run)
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, st

    trainer = make_trainer(args.mode, net)
    elapsed, st = timed(trainer, args.steps)
    loss = float(st[0].item()) / B
    # the timed run's own health: a finite loss and finite weights after the last timed step
    w_finite = bool(torch.isfinite(net.store.master).all()) if args.mode == "sync" else True
    check = {"final_loss_finite": bool(torch.isfinite(torch.tensor(loss))), "weights_finite": w_finite}
    ms = elapsed / args.steps * 1e3
    value = world * B * args.steps / elapsed
    phases = None
    if args.phases > 0 and args.mode == "sync" and dev.type == "cuda":
        phases = {k: round(v, 4) for k, v in trainer.timed_eager_steps(args.phases).items()}
    if not args.no_check and dev.type == "cuda":
        check["gradient"] = correctness_guard(args.model, B, dev, data, labels)
    check["ok"] = (check["final_loss_finite"] and check["weights_finite"]
                   and check.get("gradient", {"ok": True})["ok"])
    async_rec = None
    async_steps = args.steps if args.async_steps is None else args.async_steps
    if args.mode == "sync" and async_steps > 0 and dev.type == "cuda":
        # BASELINE metric "...; async speedup": same model / batch / rank count through the async engine
        try:
            anet = build_model(args.model, device=dev, seed=0)
            atr = make_trainer("async", anet)
            ael, _ = timed(atr, async_steps)
            aval = world * B * async_steps / ael
            # the sync trainer timed again right after, the same way (each run settles first, but the box's
            # clocks still drift between runs); the ratio is against their mean step time (the async run sits
            # between them)
            sel2, _ = timed(trainer, async_steps)
            sync_ms = 0.5 * (elapsed / args.steps + sel2 / async_steps) * 1e3
            async_ms = ael / async_steps * 1e3
            async_rec = dict(images_per_s=round(aval, 1), ms_per_step=round(async_ms, 4),
                             steps=async_steps, speedup_vs_sync=round(sync_ms / async_ms, 4),
                             sync_rerun_ms_per_step=round(sel2 / async_steps * 1e3, 4),
                             sync_bracket_ms_per_step=round(sync_ms, 4),
                             speedup_vs_first_sync=round(aval / value, 4),
                             max_staleness_bound=args.max_staleness, **atr.ps_stats())
        except Exception as e:  # reported, never fatal to the headline number
            async_rec = {"error": repr(e)[:300]}
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "images/s",
            "n_gpus": world,
            "world": live_world,
            "backend": live_backend,
            "steps": args.steps,
            "warmup": args.warmup,
            # untimed steps before the warm-up of each timed run (the clock ramp, see settle()); the timed
            # region is exactly ``steps`` steps either way
            "settle": {"target_ms": args.settle_ms, "runs": settle_recs} if settle_recs else None,
            "ms_per_step": round(ms, 4),
            "final_loss": round(loss, 6),
            "check": check,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if BASELINE_VALUE is None else value / BASELINE_VALUE,
            "dtype": "bf16" if dev.type == "cuda" else "fp32",
            "data": ("synthetic (CIFAR-10-shaped 50000x32x32x3 uint8" if args.model == "resnet18_cifar" else
                     "synthetic (MNIST-shaped 60000x28x28x1 uint8") + ", HBM resident), random-init weights",
            "config": {
                "model": args.model,
                "global_batch": B * world,
                "per_gpu_batch": B,
                "seq_len": None,
                "parallelism": f"dp{world}" if args.mode == "sync" else f"async-ps{world}",
                "optimizer": "sgd",
                "graph": trainer.graph_mode,
                "steps_per_graph": getattr(trainer, "_multi_u", 0) or 1,
                "allreduce": trainer.allreduce_path if world > 1 else None,
                # why the one-shot / in-kernel exchange path was or was not taken, and the real-kernel
                # self-test of the fused multi-rank step (parallel/data_parallel.py _verify_fused_exchange)
                "p2p_reason": getattr(trainer, "p2p_reason", None) or None,
                "fused_selftest": getattr(trainer, "fused_selftest", None) or None,
                "step": trainer.step_launches,
                "params": net.num_params(),
            },
        }
        if args.mode == "async":
            out["async"] = dict(trainer.ps_stats(), max_staleness_bound=args.max_staleness)
        elif async_rec is not None:
            out["async"] = async_rec
        if phases is not None:
            out["phases_ms_eager"] = phases
        if diag_active():
            out["diagnostics"] = diag_active()  # a diagnostic run: never a production number
        if os.environ.get("DISTRIFLOW_DIAG", "").strip():
            # verbatim, including switches only the native code reads (csrc/diag.h)
            out["distriflow_diag"] = os.environ["DISTRIFLOW_DIAG"]
        if args.json_extra:
            out["extra"] = {"final_loss": loss, "train_tflops": value * net.flops_per_example() / 1e12,
                            "capture_error": getattr(trainer, "capture_error", None)}
        print(json.dumps(out), flush=True)
    shutdown()
    if not check["ok"]:
        print(f"bench: correctness check FAILED: {check}", file=sys.stderr, flush=True)
        sys.exit(4)


if __name__ == "__main__":
    main()
