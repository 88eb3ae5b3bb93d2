"""Command-line launcher: ``python -m distriflow_amd.launch [--nproc N] MODE [options]``.

The reference has no CLI — its experiments are two hand-written TypeScript mains
(/root/reference/experiment/mnist/mnist_server.ts:16-37, mnist_client.ts:15-31; SURVEY §5.6 asks
for ``python -m distriflow.launch``).  One process per GPU, torchrun-compatible environment
(RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT); with ``--nproc N`` this module is its
own launcher (children are spawned before anything touches the GPU) and, with ``--max-restarts``,
restarts a failed job from its last checkpoint (``--resume``), which is the all-reduce mode's
answer to a lost rank.

Modes
  sync    synchronous data parallelism: RCCL all-reduce SGD (DataParallelTrainer), tf.js
          checkpoints + resume record per epoch (``--save-dir``)
  async   asynchronous parameter server (rank 0) with bounded staleness; workers hold the dataset
          in HBM and receive batch ids (``--ship-data`` sends tensors instead, as the reference)
  fedsgd  the reference's FederatedServer / FederatedClient (count barrier + version gating)
  fedavg  federated averaging over non-IID label shards

With WORLD_SIZE == 1 the parameter-server modes run in one process: server + ``--workers``
worker threads over the in-process transport (same GPU).

Fault injection (tests / drills): ``--fault-kill-rank R --fault-kill-step S`` makes rank R exit
abruptly at its step S; ``--fault-delay-rank R --fault-delay-ms D`` slows rank R's every step.
Metrics: ``--metrics FILE`` appends rank-tagged JSONL records (also ``DISTRIFLOW_METRICS``).
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import Optional


# ------------------------------------------------------------------------------------------ CLI
def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="python -m distriflow_amd.launch", description=__doc__.split("\n")[0])
    ap.add_argument("--nproc", type=int, default=1, help="spawn N local ranks (one per GPU)")
    ap.add_argument("--max-restarts", type=int, default=0, help="restart the job from its checkpoint on failure")
    ap.add_argument("--master-port", type=int, default=0)
    sub = ap.add_subparsers(dest="mode", required=True)

    def common(p):
        p.add_argument("--model", default="lenet5", help="mlp_mnist | lenet5 | keras_cnn | resnet18_cifar")
        p.add_argument("--data", default="synthetic", help="synthetic | mnist:<dir with IDX files>")
        p.add_argument("--num-examples", type=int, default=60000)
        p.add_argument("--batch", type=int, default=256, help="per-rank batch (sync) / microbatch (PS modes)")
        p.add_argument("--lr", type=float, default=0.05)
        p.add_argument("--epochs", type=int, default=1)
        p.add_argument("--seed", type=int, default=0)
        p.add_argument("--device", default="auto", help="auto | cuda | cpu")
        p.add_argument("--metrics", default=None, help="JSONL metrics file")
        p.add_argument("--verbose", action="store_true")
        p.add_argument("--fault-kill-rank", type=int, default=-1)
        p.add_argument("--fault-kill-step", type=int, default=-1)
        p.add_argument("--fault-delay-rank", type=int, default=-1)
        p.add_argument("--fault-delay-ms", type=float, default=0.0)

    p = sub.add_parser("sync", help="synchronous all-reduce data parallelism")
    common(p)
    p.add_argument("--momentum", type=float, default=0.0)
    p.add_argument("--graph", default=None, choices=["full", "split", "none"])
    p.add_argument("--save-dir", default=None)
    p.add_argument("--resume", action="store_true")
    p.add_argument("--steps", type=int, default=0, help="stop after this many steps (0 = full epochs)")
    p.add_argument("--min-updates", type=int, default=0,
                   help="FedSGD count barrier on the device: K microbatches of --batch rows per version, split over "
                        "the ranks (reference minUpdatesPerVersion; 0 = one per rank)")

    p = sub.add_parser("async", help="asynchronous parameter server, bounded staleness")
    common(p)
    p.add_argument("--workers", type=int, default=2, help="worker threads when running in one process")
    p.add_argument("--max-staleness", type=int, default=-1)
    p.add_argument("--ship-data", action="store_true")
    p.add_argument("--store-port", type=int, default=0,
                   help="device engine: rank 0 hosts a TCPStore on this port and publishes the parameter server's "
                        "handles there, so workers outside the job can attach later (launch join)")
    p.add_argument("--wait-joiners", type=int, default=0,
                   help="with --store-port: start stepping only once this many joiners have attached")
    p.add_argument("--engine", default="auto", choices=["auto", "device", "roles"],
                   help="device = GPU-resident parameter server (parallel/async_ps.py, every rank a worker); "
                        "roles = message-level AsynchronousSGDServer/Client (reference protocol); "
                        "auto = device on GPUs, roles on CPU")

    p = sub.add_parser("join", help="a late-joining async worker: attach to a running device parameter server "
                                    "(started with async --store-port) and train until its schedule finishes")
    common(p)
    p.add_argument("--store", required=True, help="HOST:PORT of the members' TCPStore")
    p.add_argument("--joiner-id", type=int, default=64, help="unique id >= the members' world size")

    p = sub.add_parser("fedsgd", help="FederatedServer / FederatedClient (reference sync PS)")
    common(p)
    p.add_argument("--workers", type=int, default=2)
    p.add_argument("--min-updates", type=int, default=2)
    p.add_argument("--updates-per-worker", type=int, default=20)

    p = sub.add_parser("fedavg", help="federated averaging over non-IID shards")
    common(p)
    p.add_argument("--workers", type=int, default=2)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--local-steps", type=int, default=20)
    p.add_argument("--classes-per-client", type=int, default=2)
    p.add_argument("--engine", default="auto", choices=["auto", "device", "roles"],
                   help="device = every rank a client, graph-captured local steps, collective weight average "
                        "(parallel/fedavg.py); roles = FedAvgServer/FedAvgClient messages; auto = device on GPUs")
    return ap


# ------------------------------------------------------------------------------------------ spawner
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn(argv: list, nproc: int, max_restarts: int, port: int) -> int:
    """Run ``nproc`` ranks of this module; on a failure stop the others (their exact PIDs) and
    restart everything with ``--resume`` up to ``max_restarts`` times."""
    child_argv = [a for a in argv]
    attempt = 0
    while True:
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port or _free_port()), WORLD_SIZE=str(nproc))
        procs = []
        for r in range(nproc):
            e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen([sys.executable, "-m", "distriflow_amd.launch"] + child_argv, env=e))
        failed = None
        while True:
            codes = [p.poll() for p in procs]
            bad = [(i, c) for i, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                failed = bad[0]
                break
            if all(c == 0 for c in codes):
                return 0
            time.sleep(0.2)
        for p in procs:  # stop the survivors of a failed job
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        deadline = time.time() + 20
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        print(f"[launch] rank {failed[0]} exited with {failed[1]} (attempt {attempt})", file=sys.stderr, flush=True)
        if attempt >= max_restarts:
            return failed[1] or 1
        attempt += 1
        # a restarted job resumes from its checkpoint and runs without the injected fault
        child_argv = [a for a in child_argv if a != "--resume"]
        child_argv = _strip_opt(child_argv, "--fault-kill-rank") + ["--resume"] if "sync" in child_argv else child_argv
        child_argv = _strip_opt(child_argv, "--fault-kill-step")


def _strip_opt(argv: list, name: str) -> list:
    out, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        if a == name:
            skip = True
            continue
        if a.startswith(name + "="):
            continue
        out.append(a)
    return out


# ------------------------------------------------------------------------------------------ helpers
class Faults:
    def __init__(self, args, rank: int):
        self.kill = args.fault_kill_rank == rank and args.fault_kill_step >= 0
        self.kill_step = args.fault_kill_step
        self.delay = (args.fault_delay_ms / 1e3) if args.fault_delay_rank == rank else 0.0

    def step(self, i: int):
        from .parallel.watchdog import beat

        beat(i)
        if self.delay:
            time.sleep(self.delay)
        if self.kill and i >= self.kill_step:
            print(f"[fault] rank {os.environ.get('RANK', '0')} killed at step {i}", file=sys.stderr, flush=True)
            os._exit(17)


def _device(args):
    import torch

    if args.device == "auto":
        return "cuda" if torch.cuda.is_available() else "cpu"
    return args.device


def _load_data(args, device, seed=0):
    from .data.synthetic import synthetic_cifar10, synthetic_mnist

    if args.data.startswith("mnist:"):
        from .data.mnist import load_mnist

        x, y = load_mnist(args.data.split(":", 1)[1], "train")
        return x.to(device), y.to(device)
    if args.model == "resnet18_cifar":
        return synthetic_cifar10(args.num_examples, seed=seed, device=device)
    return synthetic_mnist(args.num_examples, seed=seed, device=device)


def _logger(args, role):
    from .utils.logging import Logger

    return Logger(role, verbose=args.verbose, metrics_file=args.metrics)


# ------------------------------------------------------------------------------------------ sync
def run_sync(args) -> dict:
    import torch
    import torch.distributed as dist

    from .checkpoint.store import VersionedStore
    from .checkpoint.tfjs import load_layers_model_weights, save_layers_model
    from .models.zoo import build_model
    from .parallel.comm import init_distributed, shutdown
    from .data.dataset import DistriDataset
    from .parallel.data_parallel import DataParallelTrainer, fedsgd_rows

    env = init_distributed(device=_device(args), watchdog=True)
    rank, world, dev = env.rank, env.world_size, env.device
    log = _logger(args, f"Distributed Worker {rank}")
    faults = Faults(args, rank)
    net = build_model(args.model, device=dev, seed=args.seed)
    x, y = _load_data(args, dev)
    n = x.shape[0]
    B = args.batch
    start_step = 0
    store = VersionedStore(args.save_dir) if args.save_dir else None
    if store is not None:
        store.setup()
        if args.resume and store.last() is not None:
            load_layers_model_weights(net, os.path.join(store.path(store.last()), "model.json"))
            rec = store.read_resume() or {}
            start_step = int(rec.get("step", 0))
            log.log(f"resumed from version {store.last()} at step {start_step} (after epoch {rec.get('epoch')})")
    graph = args.graph or "full"
    tr = DataParallelTrainer(net, lr=args.lr, momentum=args.momentum, graph=graph if dev.type == "cuda" else "none",
                             min_updates_per_version=args.min_updates or None)
    scale = 1.0 / 255.0 if x.dtype == torch.uint8 else 1.0
    # the DistriDataset's dispenser (epochs, per-epoch shuffle, FCFS order, completion) becomes the device
    # index stream: batch k of the schedule goes to rank k % world, and every step's update launch stages
    # the next step's indices (no host work per step).  The schedule is always built from the ORIGINAL seed
    # and epoch count, and a resumed job skips the steps already taken: it trains on exactly the batches an
    # uninterrupted job would have.
    ds = DistriDataset(x, y, {"batchSize": B, "epochs": args.epochs}, shuffle=True, seed=args.seed)
    tr.bind_dataset(ds.x, ds.y, B, scale=scale)
    if tr.min_updates is not None:  # K microbatches of the one FCFS stream per version (count barrier)
        g_rows, g_epochs = ds.index_stream(0, 1, device=dev, with_epochs=True)
        rows, row_epoch = fedsgd_rows(g_rows, tr.min_updates, rank, world, g_epochs)
    else:
        rows, row_epoch = ds.index_stream(rank, world, device=dev, with_epochs=True)
    total = rows.shape[0]
    start = min(start_step, total)
    if start < total:
        tr.bind_index_stream(rows[start:])
    # per-replay statistics through the trainer callbacks (device counters, read back asynchronously)
    tr.on_upload(lambda st: log.metric(event="upload", **st))
    tr.on_new_version(lambda old, new: log.log(f"updated model: {old} -> {new}"))
    step = start
    # without per-step fault hooks the steps between two epoch boundaries run as multi-step graph replays
    # (no per-step host work in the loop); with faults injected, one step at a time
    chunked = not (faults.kill or faults.delay)
    if chunked:
        tr.prepare_run(DataParallelTrainer.MAX_STEPS_PER_GRAPH)
    t0 = time.perf_counter()
    seen = 0
    last_loss = float("nan")
    st = None
    limit = min(total, args.steps) if args.steps else total
    i = start
    while i < limit:
        j = i + 1  # end (exclusive) of this chunk: the epoch's last step or the step limit
        while j < limit and row_epoch[j] == row_epoch[i]:
            j += 1
        if chunked:
            st = tr.run(j - i)
        else:
            for k in range(i, j):
                faults.step(k)
                st = tr.step()
        seen += (j - i) * tr.images_per_step
        step = j
        epoch_end = j == total or row_epoch[j] != row_epoch[j - 1]
        epoch = row_epoch[j - 1]
        i = j
        tr.flush_callbacks()
        last_loss = float(st[0]) / tr.B
        el = time.perf_counter() - t0
        log.metric(event="epoch", epoch=epoch, step=step, loss=last_loss, images_per_s=seen / el)
        log.log(f"epoch {epoch}: loss {last_loss:.4f}, {seen / el:.0f} images/s")
        if epoch_end and store is not None and rank == 0:
            v = store.new_version()
            save_layers_model(net, store.path(v))
            store.mark_current(v)
            store.write_resume({"epoch": epoch, "step": step, "version": v})
        if world > 1:
            dist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    out = {"mode": "sync", "world": world, "steps": step, "images_per_s": seen / max(el, 1e-9), "loss": last_loss,
           "graph": tr.graph_mode}
    if rank == 0:
        print(json.dumps(out), flush=True)
    shutdown()
    return out


# ------------------------------------------------------------------------------------------ parameter-server modes
def _ps_setup(args):
    from .parallel.comm import init_distributed

    env = init_distributed(device=_device(args), watchdog=True)
    return env


def run_async_device(args) -> dict:
    """Async SGD on the device-resident bounded-staleness parameter server: rank 0's HBM holds the
    master weights and the FCFS microbatch counter; every rank (one per GPU) is a worker that replays its
    own captured step.  The epochs' microbatches are split evenly over the ranks."""
    import torch
    import torch.distributed as dist

    from .models.zoo import build_model
    from .parallel.async_ps import AsyncPSTrainer
    from .parallel.comm import init_distributed, shutdown
    from .parallel.data_parallel import epoch_permutations

    env = init_distributed(device=_device(args), watchdog=True)
    rank, world, dev = env.rank, env.world_size, env.device
    log = _logger(args, f"Distributed Worker {rank}")
    x, y = _load_data(args, dev)
    n, B = x.shape[0], args.batch
    nb = n // B
    net = build_model(args.model, device=dev, seed=args.seed)
    joinable = bool(getattr(args, "store_port", 0))
    tr = AsyncPSTrainer(net, lr=args.lr, max_staleness=args.max_staleness, graph="full", joinable=joinable)
    if joinable:  # late joiners (launch join) read the server's handles from this store
        import datetime

        store = dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), args.store_port, is_master=(rank == 0),
                              wait_for_workers=False, timeout=datetime.timedelta(seconds=300))
        tr.publish(store)
        tr._store_keepalive = store
        if args.wait_joiners > 0:
            t_w = time.time()
            while store.add("distriflow/ps/joined", 0) < args.wait_joiners:
                if time.time() - t_w > 300:
                    raise RuntimeError(f"async: {args.wait_joiners} joiner(s) did not attach within 300 s")
                time.sleep(0.05)
    tr.bind_dataset(x, y, B, scale=1.0 / 255.0 if x.dtype == torch.uint8 else 1.0)
    # one table row per microbatch id of an epoch; at-least-once dispatch per epoch on the device
    tr.bind_schedule(epoch_permutations(n, B, nb, dev, seed=args.seed), epochs=args.epochs)
    # per-replay JSONL through the trainer callbacks (device counters, read back asynchronously)
    tr.on_upload(lambda st: log.metric(event="upload", **st))
    faults = Faults(args, rank)
    cap = 4 * nb * args.epochs + 64  # a healthy run ends long before: every claim is a real step
    # without per-step fault hooks the steps run as multi-step graph replays, like the sync loop (no
    # per-step host work); the host only polls finished() between chunks.  Steps after the last epoch are
    # device no-ops.
    chunked = not (faults.kill or faults.delay)
    chunk = 32 if chunked else 8
    if chunked:
        tr.prepare_run(chunk)
    t0 = time.perf_counter()
    steps = 0
    while True:
        if chunked:
            st = tr.run(chunk)
            steps += chunk
        else:
            for _ in range(chunk):
                faults.step(steps)
                st = tr.step()
                steps += 1
        if tr.finished():
            break
        if steps >= cap:
            raise RuntimeError(f"async PS did not finish {args.epochs} epochs in {steps} steps: {tr.ps_stats()}")
    torch.cuda.synchronize(dev)
    tr.flush_callbacks()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    tr.check_comm()
    out = {}
    if rank == 0:
        tr.pull_master()
        loss, acc = net.evaluate(x[:4096].float() * (1.0 / 255.0 if x.dtype == torch.uint8 else 1.0), y[:4096])
        out = dict(mode="async", engine="device", world=world, steps_per_rank=steps,
                   images_per_s=world * steps * B / max(el, 1e-9), last_loss=float(st[0]) / B,
                   eval_loss=float(loss), eval_accuracy=float(acc), max_staleness_bound=args.max_staleness,
                   capture_warmup=tr.capture_warmup if tr.graph_mode == "full" else 0, step=tr.step_launches,
                   graph=tr.graph_mode, capture_error=getattr(tr, "capture_error", None),
                   **tr.ps_stats())
        log.metric(event="async_done", **out)
        print(json.dumps(out), flush=True)
    shutdown()
    return out


def run_join(args) -> dict:
    """A worker outside the members' process group (elastic scale-up, parallel/elastic.py): attach to the
    published device parameter server, train on the shared FCFS schedule until it is finished."""
    import torch

    from .models.zoo import build_model
    from .parallel import elastic
    from .parallel.async_ps import AsyncPSTrainer
    from .parallel.data_parallel import epoch_permutations

    dev = torch.device("cuda", 0) if _device(args) == "cuda" else None
    if dev is None:
        raise RuntimeError("launch join: the device parameter server needs a GPU")
    torch.cuda.set_device(dev)
    host, port = args.store.rsplit(":", 1)
    store = elastic.store_client(host, int(port))
    x, y = _load_data(args, dev)
    n, B = x.shape[0], args.batch
    net = build_model(args.model, device=dev, seed=args.seed)
    tr = AsyncPSTrainer.attach(net, store, joiner_id=args.joiner_id, lr=args.lr, graph="full")
    tr.bind_dataset(x, y, B, scale=1.0 / 255.0 if x.dtype == torch.uint8 else 1.0)
    tr.bind_schedule(epoch_permutations(n, B, n // B, dev, seed=args.seed), epochs=args.epochs)
    v_join = tr.ps_stats()["version"]
    store.add("distriflow/ps/joined", 1)  # (members started with --wait-joiners wait for this)
    steps, cap = 0, 4 * (n // B) * args.epochs + 64
    while not tr.finished() and steps < cap:
        for _ in range(8):
            tr.step()
            steps += 1
    torch.cuda.synchronize(dev)
    tr.check_comm()
    out = dict(mode="join", joiner_id=args.joiner_id, steps=steps, version_at_attach=v_join, **tr.ps_stats())
    print(json.dumps(out), flush=True)
    return out


def run_async(args) -> dict:
    import torch

    engine = args.engine
    if engine == "auto":
        engine = "device" if _device(args) == "cuda" else "roles"
    if engine == "device":
        return run_async_device(args)

    from .data.dataset import DistriDataset
    from .models.distri_model import ClientModel, InMemoryServerModel
    from .parallel.server import AsynchronousSGDServer
    from .parallel.transport import LocalHub, make_star_transports
    from .parallel.worker import AsynchronousSGDClient

    env = _ps_setup(args)
    dev = env.device
    x, y = _load_data(args, dev)
    scale = 1.0 / 255.0 if x.dtype == torch.uint8 else 1.0
    srv_cfg = {"modelDir": False, "verbose": args.verbose,
               "serverHyperparams": {"maximumStaleness": args.max_staleness}}
    compile_cfg = {"learningRate": args.lr}

    def make_server(tp):
        ds = DistriDataset(x, y, {"batchSize": args.batch, "epochs": args.epochs}, shuffle=True, seed=args.seed)
        model = InMemoryServerModel(args.model, compile_cfg, device=dev)
        return AsynchronousSGDServer(tp, model, ds, srv_cfg, ship_data=args.ship_data), ds

    def make_worker(tp, r):
        cm = ClientModel(args.model, compile_cfg, device=dev)
        return AsynchronousSGDClient(tp, cm, {"clientId": f"async-{r}", "verbose": args.verbose},
                                     data=None if args.ship_data else x, labels=None if args.ship_data else y,
                                     data_scale=scale)

    log = _logger(args, "Distributed Server")
    t0 = time.perf_counter()
    if env.world_size == 1:
        hub = LocalHub(1 + args.workers)
        srv, ds = make_server(hub.endpoint(0))
        srv.setup()
        workers = [make_worker(hub.endpoint(r, [0]), r) for r in range(1, 1 + args.workers)]
        faults = [Faults(args, r) for r in range(1, 1 + args.workers)]
        for w, f in zip(workers, faults):
            if f.delay:
                w.on_upload(lambda msg, f=f: time.sleep(f.delay))
        ths = [threading.Thread(target=lambda w=w: (w.setup(), w.run(timeout=3600)), daemon=True) for w in workers]
        for t in ths:
            t.start()
        srv.serve(until=srv.all_done, timeout=3600)
        for t in ths:
            t.join(timeout=30)
        result = srv
    else:
        tp = make_star_transports(0)
        if env.rank == 0:
            srv, ds = make_server(tp)
            srv.setup()
            srv.serve(until=lambda: srv.all_done() and srv.num_clients == 0, timeout=3600)
            result = srv
        else:
            w = make_worker(tp, env.rank)
            faults = Faults(args, env.rank)
            if faults.delay or faults.kill:
                cnt = [0]

                def _hook(msg, f=faults, c=cnt):
                    f.step(c[0])
                    c[0] += 1

                w.on_upload(_hook)
            w.setup()
            w.run(timeout=3600)
            w.dispose()
            result = None
        tp.close()
    el = time.perf_counter() - t0
    out = None
    if result is not None:
        images = result.num_updates * args.batch
        out = {"mode": "async", "world": env.world_size, "workers": args.workers if env.world_size == 1 else
               env.world_size - 1, "updates": result.num_updates, "rejected": result.rejected,
               "staleness_hist": list(result.gate.histogram()), "images_per_s": images / max(el, 1e-9),
               "max_staleness": args.max_staleness}
        log.metric(event="async_done", **{k: v for k, v in out.items() if k != "staleness_hist"})
        print(json.dumps(out), flush=True)
    from .parallel.comm import shutdown

    shutdown()
    return out or {}


def run_fedsgd(args) -> dict:
    import torch

    from .models.distri_model import ClientModel, InMemoryServerModel
    from .parallel.server import FederatedServer
    from .parallel.transport import LocalHub, make_star_transports
    from .parallel.worker import FederatedClient

    env = _ps_setup(args)
    dev = env.device
    x, y = _load_data(args, dev)
    xf = x.float() / 255.0 if x.dtype == torch.uint8 else x
    epu = args.batch
    cfg = {"modelDir": False, "verbose": args.verbose, "serverHyperparams": {"minUpdatesPerVersion": args.min_updates},
           "clientHyperparams": {"examplesPerUpdate": epu}}
    compile_cfg = {"learningRate": args.lr}

    def feed(c, r, nworkers):
        shard = torch.arange(r - 1, x.shape[0], nworkers, device=x.device)[: epu * args.updates_per_worker]
        f = Faults(args, r)
        for i in range(0, shard.numel(), epu):
            f.step(i // epu)
            idx = shard[i: i + epu]
            c.distributed_update(xf.index_select(0, idx), y.index_select(0, idx))

    t0 = time.perf_counter()
    out = None
    if env.world_size == 1:
        hub = LocalHub(1 + args.workers)
        srv = FederatedServer(hub.endpoint(0), InMemoryServerModel(args.model, compile_cfg, device=dev), cfg)
        srv.setup()
        th = threading.Thread(target=srv.serve, kwargs={"timeout": 3600}, daemon=True)
        th.start()
        clients = [FederatedClient(hub.endpoint(r, [0]), ClientModel(args.model, compile_cfg, device=dev),
                                   {"clientId": f"fed-{r}"}) for r in range(1, 1 + args.workers)]
        ths = []
        for r, c in enumerate(clients, 1):
            def go(c=c, r=r):
                c.setup()
                feed(c, r, args.workers)
            ths.append(threading.Thread(target=go, daemon=True))
            ths[-1].start()
        for t in ths:
            t.join()
        time.sleep(0.2)
        srv.stop()
        out = {"mode": "fedsgd", "versions": srv.version_id,
               "uploads": sum(c.num_updates() for c in clients)}
    else:
        tp = make_star_transports(0)
        if env.rank == 0:
            srv = FederatedServer(tp, InMemoryServerModel(args.model, compile_cfg, device=dev), cfg)
            srv.setup()
            srv.serve(until=lambda: srv.num_clients == 0 and srv.version_id > 0, timeout=3600)
            out = {"mode": "fedsgd", "versions": srv.version_id}
        else:
            c = FederatedClient(tp, ClientModel(args.model, compile_cfg, device=dev), {"clientId": f"fed-{env.rank}"})
            c.setup()
            feed(c, env.rank, env.world_size - 1)
            c.poll(0.5)
            c.dispose()
        tp.close()
    el = time.perf_counter() - t0
    if out is not None:
        out["seconds"] = el
        print(json.dumps(out), flush=True)
    from .parallel.comm import shutdown

    shutdown()
    return out or {}


def run_fedavg_device(args) -> dict:
    """FedAvg with every rank a client on its own non-IID shard: captured local SGD steps, then an
    in-place average of the flat master (one-shot xGMI all-reduce / RCCL) each round."""
    import torch

    from .data.synthetic import non_iid_shards
    from .models.zoo import build_model
    from .parallel.comm import init_distributed, shutdown
    from .parallel.fedavg import FedAvgTrainer

    env = init_distributed(device=_device(args), watchdog=True)
    rank, world, dev = env.rank, env.world_size, env.device
    x, y = _load_data(args, dev)
    scale = 1.0 / 255.0 if x.dtype == torch.uint8 else 1.0
    shard = non_iid_shards(y, world, args.classes_per_client, seed=args.seed)[rank].to(dev)
    B = args.batch
    total = args.rounds * args.local_steps
    g = torch.Generator(device="cpu").manual_seed(args.seed + 1000 * rank)
    chunks, need = [], total * B
    while sum(c.numel() for c in chunks) < need:
        chunks.append(shard[torch.randperm(shard.numel(), generator=g).to(dev)])
    stream = torch.cat(chunks)[:need].view(total, B)
    net = build_model(args.model, device=dev, seed=args.seed)
    tr = FedAvgTrainer(net, lr=args.lr, local_steps=args.local_steps,
                       graph="full" if dev.type == "cuda" else "none")
    tr.bind_dataset(x, y, B, scale=scale)
    tr.bind_index_stream(stream)
    if dev.type == "cuda":
        tr.prepare_run(args.local_steps)  # the local steps' multi-step graph, captured before the clock starts
    t0 = time.perf_counter()
    for _ in range(args.rounds):
        tr.run_round()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    tr.check_comm()
    out = {}
    if rank == 0:
        n = min(4096, x.shape[0])
        loss, acc = net.evaluate(x[:n].float() * scale, y[:n])
        out = {"mode": "fedavg", "engine": "device", "clients": world, "rounds": tr.rounds,
               "local_steps": args.local_steps, "rounds_per_s": tr.rounds / max(el, 1e-9),
               "images_per_s": world * total * B / max(el, 1e-9), "test_loss": float(loss),
               "test_accuracy": float(acc), "allreduce": tr.allreduce_path if world > 1 else None}
        print(json.dumps(out), flush=True)
    shutdown()
    return out


def run_fedavg(args) -> dict:
    import torch

    engine = args.engine
    if engine == "auto":
        engine = "device" if _device(args) == "cuda" else "roles"
    if engine == "device":
        return run_fedavg_device(args)

    from .data.synthetic import non_iid_shards
    from .models.distri_model import ClientModel, InMemoryServerModel
    from .parallel.server import FedAvgServer
    from .parallel.transport import LocalHub, make_star_transports
    from .parallel.worker import FedAvgClient

    env = _ps_setup(args)
    dev = env.device
    x, y = _load_data(args, dev)
    scale = 1.0 / 255.0 if x.dtype == torch.uint8 else 1.0
    nclients = args.workers if env.world_size == 1 else env.world_size - 1
    shards = non_iid_shards(y, nclients, args.classes_per_client, seed=args.seed)
    compile_cfg = {"learningRate": args.lr}
    test_x = x[: min(4096, x.shape[0])]
    test_y = y[: test_x.shape[0]]

    def make_client(tp, r):
        idx = shards[r - 1].to(x.device)
        return FedAvgClient(tp, ClientModel(args.model, compile_cfg, device=dev), x.index_select(0, idx),
                            y.index_select(0, idx), {"clientId": f"avg-{r}"}, batch_size=args.batch,
                            local_steps=args.local_steps, data_scale=scale, seed=args.seed + r)

    t0 = time.perf_counter()
    out = None
    if env.world_size == 1:
        hub = LocalHub(1 + nclients)
        model = InMemoryServerModel(args.model, compile_cfg, device=dev)
        srv = FedAvgServer(hub.endpoint(0), model, {"modelDir": False}, rounds=args.rounds)
        srv.setup()
        clients = [make_client(hub.endpoint(r, [0]), r) for r in range(1, 1 + nclients)]
        ths = [threading.Thread(target=lambda c=c: (c.setup(), c.run(timeout=3600)), daemon=True) for c in clients]
        for t in ths:
            t.start()
        while len(srv.clients) < nclients:
            srv.step(0.05)
        srv.start_round()
        srv.serve(until=srv.finished, timeout=3600)
        srv.stop()
    else:
        tp = make_star_transports(0)
        if env.rank == 0:
            model = InMemoryServerModel(args.model, compile_cfg, device=dev)
            srv = FedAvgServer(tp, model, {"modelDir": False}, rounds=args.rounds)
            srv.setup()
            while len(srv.clients) < nclients:
                srv.step(0.05)
            srv.start_round()
            srv.serve(until=srv.finished, timeout=3600)
            srv.stop()
        else:
            c = make_client(tp, env.rank)
            c.setup()
            c.run(timeout=3600)
            c.dispose()
            srv = None
        tp.close()
    el = time.perf_counter() - t0
    if env.rank == 0:
        loss, acc = model.evaluate(test_x.float() * scale, test_y)
        out = {"mode": "fedavg", "clients": nclients, "rounds": srv.round, "rounds_per_s": srv.round / max(el, 1e-9),
               "test_loss": loss, "test_accuracy": acc}
        print(json.dumps(out), flush=True)
    from .parallel.comm import shutdown

    shutdown()
    return out or {}


MODES = {"sync": run_sync, "async": run_async, "join": run_join, "fedsgd": run_fedsgd, "fedavg": run_fedavg}


def main(argv: Optional[list] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = build_parser().parse_args(argv)
    if args.nproc > 1 and "WORLD_SIZE" not in os.environ:
        child = _strip_opt(_strip_opt(_strip_opt(argv, "--nproc"), "--max-restarts"), "--master-port")
        return _spawn(child, args.nproc, args.max_restarts, args.master_port)
    MODES[args.mode](args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
