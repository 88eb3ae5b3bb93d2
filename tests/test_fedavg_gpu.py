"""Device FedAvg (parallel/fedavg.py, BASELINE.json configs[4]) on one MI355X: the local steps of a round run as
multi-step hipGraph replays and give the same weights, bit for bit, as one replay per
step; the round's average is the identity at one rank."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model,B,L", [("lenet5", 512, 20), ("mlp_mnist", 256, 7)])
def test_fedavg_multistep_round_equals_single_steps(model, B, L):
    from distriflow_amd.data.synthetic import synthetic_mnist
    from distriflow_amd.models.zoo import build_model
    from distriflow_amd.parallel.data_parallel import epoch_permutations
    from distriflow_amd.parallel.fedavg import FedAvgTrainer

    dev = torch.device("cuda", 0)
    data, labels = synthetic_mnist(8192, seed=3, device=dev)
    stream = epoch_permutations(8192, B, 3 * L, dev, seed=4)
    res = []
    for multi in (True, False):
        net = build_model(model, device=dev, seed=0)
        tr = FedAvgTrainer(net, lr=0.05, local_steps=L, graph="full")
        tr.bind_dataset(data, labels, B, scale=1.0 / 255.0)
        tr.bind_index_stream(stream)
        for _ in range(3):
            if multi:
                tr.run_round()
            else:
                for _ in range(L):
                    tr.step()
                tr.average()
        torch.cuda.synchronize()
        if multi:
            assert tr._multi_u == min(L, 64), tr._multi_u
        res.append(net.store.master.clone())
    assert torch.equal(res[0], res[1])
