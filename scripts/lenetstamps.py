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
    if "contig" in sys.argv[2:]:  # rows 0 .. B-1, no index indirection (what a pre-staged batch costs)
        x.idx = None
        y = labels[:B].to(torch.int32).contiguous()

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
    # per XCD (dispatch is round-robin: workgroup b runs on XCD b % 8; s_memtime bases differ between XCDs, so
    # start / end spreads are only comparable inside one XCD)
    for x in range(min(8, nblk)):
        sel = np.arange(x, nblk, 8)
        t = tot[sel]
        print(f"  XCD {x}: lifetime median {np.median(t):7.0f} max {t.max():7.0f} | start spread "
              f"{st[sel, 0].max() - st[sel, 0].min():7.0f} end spread {st[sel, 10].max() - st[sel, 10].min():7.0f}")
    for k, name in enumerate(NAMES):
        col = d[:, k]
        print(f"  {name:<12} median {np.median(col):8.0f}  p90 {np.percentile(col, 90):8.0f}  "
              f"share {np.median(col) / np.median(tot) * 100:5.1f}%")
    # reduce launch of the trainer's step: wall-clock stamps (100 MHz) at [4096 * 16 + block * 16 + slot]
    if len(sys.argv) > 2 and sys.argv[2] in ("step", "async"):
        reduce_stamps(m, net, data, labels, B, buf, sys.argv[2] == "async")


def reduce_stamps(m, net, data, labels, B, buf, async_ps):
    """Per-phase microseconds of the reduce launch (sync: fused update; async: parameter-server mode).
    Slots: 0 start, 1 jobs done, 2 decision known, 3 owned slots applied, 4 end, 5 first owned slot's
    rank sums in (LL) / first PS apply done, 6 first job's partial, 7 first ownership combine; staging
    workgroup: 8 admission start, 9 admission done, 10 next batch staged."""
    from distriflow_amd.parallel.data_parallel import DataParallelTrainer, epoch_permutations

    if async_ps:
        from distriflow_amd.parallel.async_ps import AsyncPSTrainer

        tr = AsyncPSTrainer(net, lr=0.01, max_staleness=4, graph="none")
        tr.bind_dataset(data, labels, B, scale=1 / 255.0)
        tr.bind_schedule(epoch_permutations(60000, B, 60000 // B, "cuda", seed=0))
    else:
        tr = DataParallelTrainer(net, lr=0.01, graph="none")
        tr.bind_dataset(data, labels, B, scale=1 / 255.0)
        tr.bind_index_stream(epoch_permutations(60000, B, 8, "cuda", seed=0))
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    rows = []
    for _ in range(5):
        buf.zero_()
        m.convpool_set_stamps(buf)
        tr.step()
        torch.cuda.synchronize()
        m.convpool_set_stamps(None)
        rows.append(buf[4096 * 16: 4096 * 16 + 1024 * 16].view(1024, 16).cpu().numpy().astype(np.int64))
    us = lambda v: v / 100.0  # noqa: E731  wall clock ticks -> us
    print(f"reduce launch ({'async PS' if async_ps else 'sync'}), 5 steps, wall clock (us):")
    for r in rows:
        valid = r[:, 0] > 0
        t0 = r[valid, 0].min()
        end = r[valid][:, [1, 4]].max()
        jobs = valid & (r[:, 6] > 0)
        own = valid & (r[:, 2] > 0) & (r[:, 3] > 0)
        ends = r[valid][:, [1, 4]].max(axis=1)
        line = [f"launch span {us(end - t0):6.2f}",
                f"starts +{us(np.median(r[valid, 0] - t0)):5.2f} med / +{us((r[valid, 0] - t0).max()):5.2f} max",
                f"first job {us(np.median(r[jobs, 6] - r[jobs, 0])):5.2f} (median, from own start)",
                f"ends +{us(np.median(ends - t0)):5.2f} med, last block {int(np.argmax(np.where(valid, r[:, [1, 4]].max(axis=1), 0)))}"
                f" of {int(valid.sum())}, job blocks end max +{us((ends[:-2] - t0).max()):5.2f}",
                f"first job done {us(np.median(r[jobs, 6] - t0)):5.2f} (median)",
                f"jobs done {us(np.median(r[valid & (r[:, 1] > 0), 1] - t0)):5.2f} (median)"]
        if own.any():
            line.append(f"owners {own.sum()}: wait {us(np.median(r[own, 2] - r[own, 1])):5.2f} "
                        f"apply {us(np.median(r[own, 3] - r[own, 2])):5.2f} max {us((r[own, 3] - r[own, 2]).max()):5.2f}")
        ps = own & (r[:, 11] > 0) & (r[:, 13] > 0)
        if ps.any():  # async PS owners: shard update, slot arrival, launch arrival, local emits
            line.append(f"PS rmw {us(np.median(r[ps, 11] - r[ps, 2])):5.2f} slot-arrive "
                        f"{us(np.median(r[ps, 12] - r[ps, 11])):5.2f} arrive {us(np.median(r[ps, 13] - r[ps, 12])):5.2f} "
                        f"emit {us(np.median(r[ps, 5] - r[ps, 13])):5.2f}")
        st = valid & (r[:, 8] > 0)
        if st.any():
            line.append(f"admission {us(float(r[st, 9][0] - r[st, 8][0])):5.2f} (start +{us(float(r[st, 8][0] - t0)):5.2f}),"
                        f" claim+stage {us(float(r[st, 10][0] - r[st, 9][0])):5.2f}")
        print("  " + "; ".join(line))
        jd = np.where(jobs, r[:, 6] - r[:, 0], 0)
        segs = []
        for b0 in range(0, int(valid.sum()), 64):
            sel = jd[b0:b0 + 64][jd[b0:b0 + 64] > 0]
            if sel.size:
                segs.append(f"{b0}:{us(np.median(sel)):.1f}/{us(sel.max()):.1f}")
        print("    job us by block (median/max): " + " ".join(segs))
        lb = int(np.argmax(np.where(valid, r[:, [1, 4]].max(axis=1), 0)))
        rel = {k: (us(float(r[lb, k] - t0)) if r[lb, k] > 0 else None) for k in (0, 6, 7, 1, 2, 11, 12, 13, 3, 5, 4)}
        print(f"    last block {lb}: " + ", ".join(f"s{k} {v:.2f}" for k, v in rel.items() if v is not None))


if __name__ == "__main__":
    main()
