#!/usr/bin/env python3
"""Where the fixed per-run cost of a short timed run goes (LeNet-5, B = 4096, one GPU).

bench.py's timed region is host wall time from a synchronised device to a synchronised device around K
steps replayed from one K-step hipGraph.  Per repeat this prints, for K in --ks:
  wall     the bench's measure (perf_counter around replay + synchronize)
  gpu      hipEvents recorded on the replay stream just before and after the replay
  launch   host time until replay() returns
  ramp     wall - gpu: the host -> device start latency plus the synchronize wake-up
plus an empty synchronize and a one-kernel launch + synchronize round trip for scale.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="20,40,64")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ramp", type=int, default=0,
                    help="then this many back-to-back 64-step replays with an event pair around each (no host sync "
                         "between them): the per-step time along a continuous run")
    args = ap.parse_args()
    from distriflow_amd.data.dataset import DistriDataset
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer

    dev = torch.device("cuda:0")
    net = build_model("lenet5", device=dev, seed=0)
    data, labels = synthetic_mnist(60000, seed=0, device=dev)
    B = 4096
    out = []
    for K in [int(k) for k in args.ks.split(",")]:
        tr = DataParallelTrainer(net, lr=0.001, graph="full")
        ds = DistriDataset(data, labels, {"batchSize": B, "epochs": 100}, shuffle=True, seed=0)
        tr.bind_distri_dataset(ds, rank=0, world=1, scale=1.0 / 255.0)
        tr.prepare_run(K)
        tr.run(K)  # first replay of this graph, untimed
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(st)
            tr.run(K)
            e1.record(st)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            gpu = e0.elapsed_time(e1) * 1e3
            wall = (t2 - t0) * 1e6
            out.append({"K": K, "wall_us": round(wall, 1), "gpu_us": round(gpu, 1), "launch_us": round((t1 - t0) * 1e6, 1),
                        "ramp_us": round(wall - gpu, 1), "wall_per_step": round(wall / K, 2),
                        "gpu_per_step": round(gpu / K, 2)})
            print(json.dumps(out[-1]), flush=True)
    if args.ramp:
        tr = DataParallelTrainer(net, lr=0.001, graph="full")
        ds = DistriDataset(data, labels, {"batchSize": B, "epochs": 10000}, shuffle=True, seed=0)
        tr.bind_distri_dataset(ds, rank=0, world=1, scale=1.0 / 255.0)
        tr.prepare_run(64)
        tr.run(64)
        torch.cuda.synchronize()
        time.sleep(0.5)  # idle, as between the bench's setup and its timed run
        st = torch.cuda.current_stream()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.ramp + 1)]
        evs[0].record(st)
        for i in range(args.ramp):
            tr.run(64)
            evs[i + 1].record(st)
        torch.cuda.synchronize()
        per = [evs[i].elapsed_time(evs[i + 1]) * 1e3 / 64 for i in range(args.ramp)]
        t = 0.0
        for i, v in enumerate(per):
            t += v * 64
            print(json.dumps({"replay": i, "t_ms": round(t / 1e3, 2), "us_per_step": round(v, 2)}), flush=True)
    x = torch.zeros(1, device=dev)
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(json.dumps({"empty_sync_us": round((t1 - t0) * 1e6, 1), "one_kernel_roundtrip_us": round((t2 - t1) * 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
