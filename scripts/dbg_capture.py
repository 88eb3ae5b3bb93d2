import sys, torch
sys.path.insert(0, "/root/repo")
from distriflow_amd.models.zoo import build_model
from distriflow_amd.data.synthetic import synthetic_mnist
from distriflow_amd.parallel.data_parallel import DataParallelTrainer, epoch_permutations
net = build_model("lenet5", device="cuda", seed=0)
data, labels = synthetic_mnist(12288, seed=3, device="cuda")
tr = DataParallelTrainer(net, lr=0.05, graph="full")
tr.bind_dataset(data[:8192], labels[:8192], 256, scale=1 / 255)
perm = epoch_permutations(8192, 256, 10, "cuda")
for i in range(3):
    tr.step_indices(perm[i])
torch.cuda.synchronize()
print("mode", tr.graph_mode, "err", getattr(tr, "capture_error", None))
