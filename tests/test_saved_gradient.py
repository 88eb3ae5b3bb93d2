"""README DistriModel fields ``modelID`` and ``savedGradient`` (/root/reference/README.md:24-29): local
gradient accumulation over microbatches, applied as one averaged update."""
import uuid

import pytest
import torch

from distriflow_amd.models.distri_model import DynamicModel, EngineModel
from distriflow_amd.models.zoo import build_model


def _engine(seed=0):
    m = EngineModel(build_model("mlp_mnist", device="cpu", seed=seed), {"learningRate": 0.1})
    m.fetch_initial()
    return m


def test_model_id_is_stable_uuid():
    m = _engine()
    assert uuid.UUID(m.model_id).version == 4
    assert m.modelID == m.model_id
    assert _engine().model_id != m.model_id


def test_saved_gradient_mean_equals_full_batch_step():
    torch.manual_seed(0)
    x = torch.rand(32, 28, 28, 1)
    y = torch.randint(0, 10, (32,))
    a, b = _engine(), _engine()
    # two half-batch microbatches accumulated locally == one full-batch gradient (mean loss)
    a.accumulate(x[:16], y[:16])
    g0 = a.saved_gradient.clone()
    a.accumulate(x[16:], y[16:])
    assert a.saved_count == 2
    assert not torch.equal(a.saved_gradient, g0)  # copied out of the live buffer, then summed
    full = b.fit_flat(x, y).clone()
    torch.testing.assert_close(a.saved_gradient / 2, full, rtol=1e-4, atol=1e-6)
    assert a.apply_saved_gradient() == 2
    assert a.saved_gradient is None and a.saved_count == 0
    b.update_flat(full)
    torch.testing.assert_close(a.get_flat(), b.get_flat(), rtol=1e-5, atol=1e-6)
    assert a.apply_saved_gradient() == 0


def test_saved_gradient_on_dynamic_model_list_grads():
    w = torch.zeros(3, requires_grad=False)
    m = DynamicModel([w.clone()], predict=lambda x: x, loss=lambda y, p: ((p - y) ** 2),
                     input_shape=[3], output_shape=[], learning_rate=0.5)
    m.save_gradient([torch.ones(3)])
    m.save_gradient([3 * torch.ones(3)])
    assert m.apply_saved_gradient(mean=True) == 2
    torch.testing.assert_close(m.get_vars()[0], torch.full((3,), -1.0))


@pytest.mark.gpu
def test_saved_gradient_engine_gpu():
    """Same identity on the HIP engine (bf16 compute, fp32 gradients): two accumulated half batches,
    averaged, equal the full-batch gradient up to bf16 rounding of the per-microbatch sums."""
    from distriflow_amd import native

    native.require()
    torch.manual_seed(0)
    x = torch.rand(256, 28, 28, 1, device="cuda").to(torch.bfloat16)
    y = torch.randint(0, 10, (256,), device="cuda")
    a = EngineModel(build_model("lenet5", device="cuda:0", seed=0), {"learningRate": 0.05})
    b = EngineModel(build_model("lenet5", device="cuda:0", seed=0), {"learningRate": 0.05})
    a.fetch_initial(), b.fetch_initial()
    a.accumulate(x[:128], y[:128])
    a.accumulate(x[128:], y[128:])
    full = b.fit_flat(x, y).clone()
    assert a.saved_gradient.is_cuda and a.saved_count == 2
    torch.testing.assert_close(a.saved_gradient / 2, full, rtol=2e-2, atol=2e-4)
    a.apply_saved_gradient()
    b.update_flat(full)
    torch.testing.assert_close(a.get_flat(), b.get_flat(), rtol=1e-3, atol=1e-5)
