#!/usr/bin/env python3
"""Device FedSGD (csrc/fedsgd_ps.hip) against an in-process replay, one rank, step by step: after every
step the sharded master must equal w - lr * mean(admitted gradients) computed by a second engine on the
same rows.  Prints the first step / parameter that differs.  Usage: dbg_fedsgd.py [graph] [K] [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    graph = sys.argv[1] if len(sys.argv) > 1 else "full"
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29611", RANK="0", WORLD_SIZE="1")
    dist.init_process_group("gloo", rank=0, world_size=1)
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.fedsgd_ps import FedSGDDeviceTrainer

    dev = torch.device("cuda", 0)
    N, MB, LR = 4096, 64, 0.05
    data, labels = synthetic_mnist(N, seed=3, device=dev)
    net = build_model("lenet5", device=dev, seed=0)
    tr = FedSGDDeviceTrainer(net, lr=LR, min_updates_per_version=K, graph=graph, timeout_s=10.0)
    tr.bind_dataset(data, labels, MB, scale=1.0 / 255.0)
    ref = build_model("lenet5", device=dev, seed=0)
    w = ref.store.master.clone()
    m0 = tr.pull_master(torch.empty_like(w))
    print("initial master equal:", torch.equal(m0, w))
    g = torch.Generator().manual_seed(7)
    acc, n_acc = None, 0
    for k in range(steps):
        idx = torch.randperm(N, generator=g)[:MB].to(dev)
        tr.step_indices(idx)
        torch.cuda.synchronize()
        ref.store.set_flat(w)
        x = (data.index_select(0, idx).float() / 255.0).to(torch.bfloat16)
        ref.compute_gradients(x, labels.index_select(0, idx))
        gr = ref.store.grad.clone()
        gd = net.store.grad.clone()
        print(f"step {k}: fed {tr.fed_stats()}; grad equal {torch.equal(gr, gd)} "
              f"max |dg| {float((gr - gd).abs().max()):.3e} (|g| max {float(gr.abs().max()):.3e})")
        acc = gr if acc is None else acc + gr
        n_acc += 1
        if n_acc == K:
            w = w - LR * (acc * (1.0 / K))
            acc, n_acc = None, 0
        m = tr.pull_master(torch.empty_like(w))
        d = (m - w).abs()
        print(f"   master max |dm| {float(d.max()):.3e}; local store master vs pulled "
              f"{float((net.store.master - m).abs().max()):.3e}")
        if float(d.max()) > 0:
            for s in ref.store.specs:
                o = ref.store.offsets[s.name]
                dd = float(d[o:o + s.numel].max())
                if dd > 0:
                    print(f"     {s.name}: max |dm| {dd:.3e}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
