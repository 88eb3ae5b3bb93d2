"""ExampleRing: the preallocated FIFO behind FederatedClient.DistributedUpdate (reference concat/slice
buffer, /root/reference/src/client/federated_client.ts:70-86,125-130)."""
import pytest
import torch

from distriflow_amd.utils.tensors import ExampleRing


def test_ring_fifo_order_with_wraparound_and_growth():
    r = ExampleRing((2, 3), capacity=4)
    ref = []
    n = 0

    def rows(k):
        nonlocal n
        t = torch.arange(n, n + k, dtype=torch.float32)[:, None, None].expand(k, 2, 3).clone()
        n += k
        return t

    for k, take in [(3, 2), (3, 3), (1, 0), (2, 2), (5, 4), (0, 0), (6, 9)]:
        t = rows(k)
        r.push(t)
        ref += [float(v) for v in t[:, 0, 0]]
        assert len(r) == len(ref)
        if take:
            got = r.peek(take)
            assert [float(v) for v in got[:, 0, 0]] == ref[:take]
            assert got.shape == (take, 2, 3)
            r.pop(take)
            ref = ref[take:]
    assert len(r) == len(ref) == 0 and r.head == 0
    assert r.grows >= 1 and r.capacity >= 8


def test_ring_single_example_and_errors():
    r = ExampleRing((4,), dtype=torch.int64, capacity=2)
    r.push(torch.tensor([1, 2, 3, 4]))
    r.push(torch.tensor([[5, 6, 7, 8]]))
    assert r.peek(2).tolist() == [[1, 2, 3, 4], [5, 6, 7, 8]]
    r.pop(1)
    r.push(torch.tensor([[9, 9, 9, 9]]))  # wraps: peek gathers the two pieces
    assert r.peek(2).tolist() == [[5, 6, 7, 8], [9, 9, 9, 9]]
    assert r.grows == 0  # steady state allocates nothing
    with pytest.raises(ValueError):
        r.push(torch.zeros(3))
    with pytest.raises(IndexError):
        r.peek(3)
    with pytest.raises(IndexError):
        r.pop(3)
