#!/usr/bin/env python3
"""Phase breakdown of the whole-network LeNet-5 training kernel (csrc/lenet_fused.hip) from in-kernel
s_memtime stamps (thread 0 of every workgroup, after each phase's barrier), B=4096, plus the wall time
of both launches with and without stamping.  Slots: 0 start, 1 staged, 2 conv1, 3 conv2, 4 dense
forward, 5 CE, 6 dense backward, 7 unpool, 8 conv2 wgrad (+dgrad weights), 9 conv2 dgrad, 10 conv1 wgrad."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distriflow_amd import native, ops  # noqa: E402
from distriflow_amd.data.synthetic import synthetic_mnist  # noqa: E402
from distriflow_amd.models.zoo import build_model  # noqa: E402

NAMES = ["stage", "conv1", "conv2", "dense fwd", "CE", "dense bwd", "unpool", "conv2 wgrad", "conv2 dgrad",
         "conv1 wgrad"]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    m = native.require()
    net = build_model("lenet5", device="cuda", seed=0)
    assert net.lenet_fused
    data, labels = synthetic_mnist(60000, seed=1, device="cuda")
    idx = torch.randperm(60000, device="cuda")[:B]
    x, y = ops.GatherRef(data, idx, 1 / 255.0, (28, 28, 1)), ops.LabelRef(labels, idx)

    def wall(n=50):
        for _ in range(3):
            net.compute_gradients(x, y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            net.compute_gradients(x, y)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n * 1e3

    base = wall()
    nblk = ops.lenet_blocks(B)
    buf = torch.zeros(4096 * 32, dtype=torch.int64, device="cuda")
    m.convpool_set_stamps(buf)
    stamped = wall(5)
    m.convpool_set_stamps(None)
    st = buf[: nblk * 16].view(nblk, 16).cpu().numpy().astype(np.int64)
    d = np.diff(st[:, :11], axis=1)
    print(f"B={B}: {nblk} workgroups; both launches {base:.1f} us/step (stamped {stamped:.1f})")
    tot = st[:, 10] - st[:, 0]
    print(f"kernel-1 workgroup lifetime: median {np.median(tot):.0f} cycles, max {tot.max():.0f}; "
          f"start spread {st[:, 0].max() - st[:, 0].min():.0f}")
    for k, name in enumerate(NAMES):
        col = d[:, k]
        print(f"  {name:<12} median {np.median(col):8.0f}  p90 {np.percentile(col, 90):8.0f}  "
              f"share {np.median(col) / np.median(tot) * 100:5.1f}%")
    # reduce launch (fused update path: the trainer's step), clocks at [4096 * 16 + block * 8 + slot]
    if len(sys.argv) > 2 and sys.argv[2] == "step":
        from distriflow_amd.parallel.data_parallel import DataParallelTrainer, epoch_permutations

        tr = DataParallelTrainer(net, lr=0.01, graph="none")
        tr.bind_dataset(data, labels, B, scale=1 / 255.0)
        tr.bind_index_stream(epoch_permutations(60000, B, 8, "cuda", seed=0))
        for _ in range(3):
            tr.step()
        torch.cuda.synchronize()
        buf.zero_()
        m.convpool_set_stamps(buf)
        tr.step()
        torch.cuda.synchronize()
        m.convpool_set_stamps(None)
        t_end_train = buf[: nblk * 16].view(nblk, 16).cpu().numpy().astype(np.int64)[:, 10].max()
        G = 2048
        r = buf[4096 * 16: 4096 * 16 + G * 8].view(G, 8).cpu().numpy().astype(np.int64)
        # job workgroup j runs job j = slot * 8 + chunk: slots are 32 x 32 dense units of (400 -> 120),
        # (120 -> 84), (84 -> 10) incl. bias, then 256-parameter conv slots; then loss, staging
        nd = sum(-(-n // 32) * -(-(k + 1) // 32) for k, n in ((400, 120), (120, 84), (84, 10)))
        nc = -(-2572 // 256)
        nj = 8 * (nd + nc)
        kinds = np.array(["dense"] * (8 * nd) + ["conv"] * (8 * nc) + ["loss", "stage"] + ["-"] * (G - nj - 2))
        valid = r[:, 0] > 0
        for kind in ("dense", "conv"):
            sel = valid & (kinds == kind)
            if sel.any():
                job = r[sel, 6] - r[sel, 0]
                own = sel & (r[:, 7] > 0)
                life = r[sel, 4] - r[sel, 0]
                print(f"  {kind:<6} jobs {sel.sum():4d}: job median {np.median(job):7.0f} max {job.max():7.0f};"
                      f" lifetime median {np.median(life):7.0f} max {life.max():7.0f}")
                if own.any():
                    comb = r[own, 7] - r[own, 6]
                    app = r[own, 3] - r[own, 2]
                    print(f"         owners {own.sum():4d}: ticket+combine median {np.median(comb):7.0f} max "
                          f"{comb.max():7.0f}; apply median {np.median(app):7.0f} max {app.max():7.0f}")
        for kind in ("loss", "stage"):
            sel = valid & (kinds == kind)
            if sel.any():
                print(f"  {kind:<6} workgroup lifetime {int((r[sel, 1] - r[sel, 0])[0]):7d}")
        r = r[valid]
        print(f"reduce launch: {r.shape[0]} stamped workgroups (per-XCD clocks: only in-workgroup spans are "
              f"meaningful)")
        for k, name in enumerate(["jobs (all)", "decision", "apply", "arrive"]):
            ok = (r[:, k + 1] > 0) & (r[:, k] > 0)
            col = r[ok, k + 1] - r[ok, k]
            if col.size:
                print(f"  {name:<18} median {np.median(col):8.0f}  p90 {np.percentile(col, 90):8.0f}  max {col.max():8.0f}")


if __name__ == "__main__":
    main()
