"""Debug helper: where the fused reduce/update differs from compute_gradients + the optimizer launch."""
import sys

import torch

sys.path.insert(0, ".")
from tests.test_lenet_fused_gpu import _nets  # noqa: E402
from distriflow_amd import ops  # noqa: E402
from distriflow_amd.data.synthetic import synthetic_mnist  # noqa: E402

B = 256
g, _ = _nets(B)
h, _ = _nets(B)
h.store.set_flat(g.store.master.clone())
for s in (g.store, h.store):
    s.set_hyper(0.05, momentum=0.9, weight_decay=1e-4, grad_scale=1.0, nesterov=False)
data, labels = synthetic_mnist(2048, seed=4, device="cuda")
stream = torch.randperm(2048, device="cuda")[: 4 * B].view(4, B).contiguous()
idx_g, idx_h = stream[0].clone(), stream[0].clone()
cur_g = torch.zeros(1, dtype=torch.int64, device="cuda")
cur_h = torch.zeros(1, dtype=torch.int64, device="cuda")
for it in range(3):
    xg = ops.GatherRef(data, idx_g, 1 / 255.0, (28, 28, 1))
    xh = ops.GatherRef(data, idx_h, 1 / 255.0, (28, 28, 1))
    sg = g.compute_gradients_and_update(xg, ops.LabelRef(labels, idx_g), (stream, cur_g, idx_g)).clone()
    sh = h.compute_gradients(xh, ops.LabelRef(labels, idx_h)).clone()
    h.store.sgd_step((stream, cur_h, idx_h))
    torch.cuda.synchronize()
    print("iter", it, "stats", sg.tolist(), sh.tolist())
    for name in ("master", "momentum", "grad"):
        a, b = getattr(g.store, name), getattr(h.store, name)
        bad = (a != b).nonzero().flatten()
        print(f"  {name}: numel {a.numel()} mismatches {bad.numel()}")
        for s in g.store.specs:
            o = g.store.offsets[s.name]
            sel = bad[(bad >= o) & (bad < o + s.numel)]
            if sel.numel():
                i = int(sel[0])
                print(f"    {s.name}: {sel.numel()} of {s.numel}, local {(sel[:6] - o).tolist()}: {a[i].item()} vs {b[i].item()}")
