"""Loss registry (reference ``lossesMap``, /root/reference/src/common/utils.ts:19-30).

Every function has the tf.js signature ``fn(labels, predictions, weights=None) -> per-example loss``
(mean over the non-batch axes) and works on any torch device.  These back ``DistriModel.evaluate``
and the ``DynamicModel`` path; the engine's *training* loss is the fused softmax cross-entropy
kernel on logits (the reference calls softmaxCrossEntropy with swapped arguments on already
softmaxed outputs, SURVEY §2.9 item 1 — not reproduced).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.nn.functional as F


def _reduce(v: torch.Tensor) -> torch.Tensor:
    return v.reshape(v.shape[0], -1).mean(dim=1) if v.dim() > 1 else v


def _w(v, weights):
    return v * weights if weights is not None else v


def absolute_difference(labels, predictions, weights=None):
    return _reduce(_w((labels.float() - predictions.float()).abs(), weights))


def compute_weighted_loss(losses, weights=None, *_):
    return _reduce(_w(losses.float(), weights))


def hinge_loss(labels, predictions, weights=None):
    y = 2.0 * labels.float() - 1.0
    return _reduce(_w(torch.relu(1.0 - y * predictions.float()), weights))


def huber_loss(labels, predictions, weights=None, delta: float = 1.0):
    return _reduce(_w(F.huber_loss(predictions.float(), labels.float(), reduction="none", delta=delta), weights))


def log_loss(labels, predictions, weights=None, eps: float = 1e-7):
    p = predictions.float()
    y = labels.float()
    return _reduce(_w(-(y * torch.log(p + eps) + (1 - y) * torch.log(1 - p + eps)), weights))


def mean_squared_error(labels, predictions, weights=None):
    return _reduce(_w((labels.float() - predictions.float()) ** 2, weights))


def sigmoid_cross_entropy(labels, logits, weights=None):
    return _reduce(_w(F.binary_cross_entropy_with_logits(logits.float(), labels.float(), reduction="none"), weights))


def softmax_cross_entropy(labels, logits, weights=None):
    """labels one-hot (or class indices), logits pre-softmax."""
    z = logits.float()
    if labels.dim() == 1 or labels.shape != z.shape:
        v = F.cross_entropy(z, labels.long().view(-1), reduction="none")
    else:
        v = -(labels.float() * F.log_softmax(z, dim=1)).sum(dim=1)
    return _w(v, weights)


def categorical_crossentropy(labels, probs, weights=None, eps: float = 1e-7):
    """Keras categorical_crossentropy on probabilities (the model.json training_config loss)."""
    p = probs.float().clamp(eps, 1.0)
    if labels.dim() == 1:
        v = -torch.log(p.gather(1, labels.long().view(-1, 1)).squeeze(1))
    else:
        v = -(labels.float() * torch.log(p)).sum(dim=1)
    return _w(v, weights)


LOSSES: dict[str, Callable] = {
    "absoluteDifference": absolute_difference,
    "computeWeightedLoss": compute_weighted_loss,
    "hingeLoss": hinge_loss,
    "huberLoss": huber_loss,
    "logLoss": log_loss,
    "meanSquaredError": mean_squared_error,
    "sigmoidCrossEntropy": sigmoid_cross_entropy,
    "softmaxCrossEntropy": softmax_cross_entropy,
    "categorical_crossentropy": categorical_crossentropy,
    "categoricalCrossentropy": categorical_crossentropy,
    "mse": mean_squared_error,
}
lossesMap = LOSSES


def get_loss(name: str) -> Callable:
    if name not in LOSSES:
        raise KeyError(f"unknown loss {name!r}; available: {sorted(LOSSES)}")
    return LOSSES[name]


def accuracy(labels, predictions) -> torch.Tensor:
    """Keras 'accuracy' for categorical outputs: argmax(pred) == argmax(labels) (labels may be indices)."""
    pred = predictions.argmax(dim=1)
    lab = labels.long().view(-1) if labels.dim() == 1 else labels.argmax(dim=1)
    return (pred == lab).float()
