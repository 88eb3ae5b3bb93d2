"""EngineModel.evaluate: compiled loss + accuracy (reference models.ts:106-115).  CPU: the torch loss
registry; GPU: one metrics launch (csrc/metrics.hip) against the registry on the same outputs."""
import warnings

import pytest
import torch

from distriflow_amd import ops
from distriflow_amd.models.distri_model import EngineModel

KINDS = ["meanSquaredError", "absoluteDifference", "hingeLoss", "huberLoss", "logLoss", "sigmoidCrossEntropy",
         "softmaxCrossEntropy", "categorical_crossentropy"]


def _ref(z, y, loss, softmax):
    out = torch.zeros(2)
    return ops.classifier_metrics(z.cpu(), y.cpu(), loss, softmax, out)


def test_engine_model_warns_once_for_non_ce_loss():
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        EngineModel("mlp_mnist", {"loss": "hingeLoss"}, device="cpu")
        EngineModel("mlp_mnist", {"loss": "hingeLoss"}, device="cpu")
    assert sum("softmax cross-entropy" in str(x.message) for x in w) == 1
    with pytest.raises(ValueError):
        EngineModel("mlp_mnist", {"loss": "meanSquaredError"}, device="cpu", strict_loss=True)
    EngineModel("mlp_mnist", {"loss": "softmaxCrossEntropy"}, device="cpu", strict_loss=True)


def test_evaluate_cpu_matches_registry():
    m = EngineModel("mlp_mnist", {"loss": "meanSquaredError"}, device="cpu")
    x = torch.rand(40, 28, 28, 1)
    y = torch.randint(0, 10, (40,))
    loss, acc = m.evaluate(x, y)
    probs = m.predict(x)
    oh = torch.nn.functional.one_hot(y, 10).float()
    assert abs(loss - float(((oh - probs) ** 2).mean(1).mean())) < 1e-6
    assert abs(acc - float((probs.argmax(1) == y).float().mean())) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("softmax", [True, False])
def test_metrics_kernel_matches_registry(kind, softmax):
    torch.manual_seed(0)
    z = torch.randn(300, 10) * 2
    if kind == "logLoss" and not softmax:
        z = torch.rand(300, 10)  # logLoss needs probabilities in (0, 1)
    y = torch.randint(0, 10, (300,), dtype=torch.int32)
    out = torch.zeros(2, device="cuda")
    g = ops.classifier_metrics(z.cuda(), y.cuda(), kind, softmax, out).cpu()
    r = _ref(z, y, kind, softmax)
    torch.testing.assert_close(g, r, rtol=2e-4, atol=2e-3)


@pytest.mark.gpu
def test_engine_evaluate_gpu_matches_cpu_path():
    m = EngineModel("lenet5", {"loss": "meanSquaredError"}, device="cuda")
    x = torch.rand(200, 28, 28, 1)
    y = torch.randint(0, 10, (200,))
    loss, acc = m.evaluate(x, y)
    probs = m.predict(x).float().cpu()
    oh = torch.nn.functional.one_hot(y, 10).float()
    assert abs(loss - float(((oh - probs) ** 2).mean(1).mean())) < 1e-4
    assert abs(acc - float((probs.argmax(1) == y).float().mean())) < 1e-6
