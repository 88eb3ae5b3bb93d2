#!/usr/bin/env python3
"""LeNet-5 B = 4096 per-step device time of: the gradient launches alone (compute_gradients), the full
eager step (train + reduce with the fused SGD update), and the multi-step hipGraph replay of full steps."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distriflow_amd import ops  # noqa: E402
from distriflow_amd.data.synthetic import synthetic_mnist  # noqa: E402
from distriflow_amd.models.zoo import build_model  # noqa: E402
from distriflow_amd.parallel.data_parallel import DataParallelTrainer, epoch_permutations  # noqa: E402


def timed(fn, n):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    B = 4096
    data, labels = synthetic_mnist(60000, seed=1, device="cuda")
    net = build_model("lenet5", device="cuda", seed=0)
    idx = torch.randperm(60000, device="cuda")[:B]
    xg, yg = ops.GatherRef(data, idx, 1 / 255.0, (28, 28, 1)), ops.LabelRef(labels, idx)
    g = timed(lambda: net.compute_gradients(xg, yg), 200)
    net2 = build_model("lenet5", device="cuda", seed=0)
    tr = DataParallelTrainer(net2, lr=0.001, graph="none")
    tr.bind_dataset(data, labels, B, scale=1 / 255.0)
    tr.bind_index_stream(epoch_permutations(60000, B, 14, "cuda", seed=0))
    e = timed(tr.step, 200)
    net3 = build_model("lenet5", device="cuda", seed=0)
    tr3 = DataParallelTrainer(net3, lr=0.001, graph="full")
    tr3.bind_dataset(data, labels, B, scale=1 / 255.0)
    tr3.bind_index_stream(epoch_permutations(60000, B, 14, "cuda", seed=0))
    tr3.prepare_run(64)
    r = timed(lambda: tr3.run(64), 4) / 64
    print(f"gradients only {g:.2f} us/step; eager full step {e:.2f} us/step; graph replay {r:.2f} us/step "
          f"({tr.step_launches})", flush=True)


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def busy(ms):
    """~ms of unrelated device work (bf16 GEMMs), to tell a clock ramp from a cache / TLB warm-up."""
    import time

    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(10):
            a = (a @ a).clamp_(-1, 1)
        torch.cuda.synchronize()


def host_timed_runs(k=20, reps=10, warm_ms=0):
    """The bench's timing shape: sync, host clock, run(k) (one k-step graph replay), sync, host clock; plus the
    device span between events recorded around the replay."""
    import time

    B = 4096
    data, labels = synthetic_mnist(60000, seed=1, device="cuda")
    net = build_model("lenet5", device="cuda", seed=0)
    tr = DataParallelTrainer(net, lr=0.001, graph="full")
    tr.bind_dataset(data, labels, B, scale=1 / 255.0)
    tr.bind_index_stream(epoch_permutations(60000, B, 14, "cuda", seed=0))
    tr.prepare_run(k)
    tr.run(5)
    if warm_ms > 0:
        busy(warm_ms)
    elif warm_ms < 0:  # touch the whole dataset once (a read of every byte: its lines land in the MALL)
        for _ in range(-warm_ms):
            float(data.sum(dtype=torch.int64))
    hs, ds = [], []
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        tr.run(k)
        e1.record()
        torch.cuda.synchronize()
        hs.append((time.perf_counter() - t0) * 1e6 / k)
        ds.append(e0.elapsed_time(e1) * 1e3 / k)
    print(f"{k}-step replays (after {warm_ms} ms of GEMMs): host us/step {['%.1f' % v for v in hs]}; device span us/step "
          f"{['%.1f' % v for v in ds]}", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1:
    host_timed_runs(int(sys.argv[1]), warm_ms=int(sys.argv[2]) if len(sys.argv) > 2 else 0)
