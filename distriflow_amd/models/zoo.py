"""Model zoo: the reference's models plus the BASELINE.json benchmark architectures.

* ``mlp_mnist``   — 784 -> Dense 10 relu -> Dense 10 softmax, 7,960 params
                    (/root/reference/experiment/mnist/mnist_server.ts:16-22, mnist_client.ts:15-21)
* ``keras_cnn``   — the Keras 2.1.4 CNN of /root/reference/experiment/mnist/model.json:1
                    (conv3x3x32, conv3x3x32, maxpool2, dropout .25, dense 128, dropout .5, dense 5; 600,165 params)
* ``lenet5``      — LeNet-5 for MNIST (BASELINE.json configs[1]/[2]): conv5x5x6 'same' + relu, maxpool2,
                    conv5x5x16 + relu, maxpool2, dense 120 relu, dense 84 relu, dense 10; 61,706 params
* ``resnet18_cifar`` — ResNet-18 for CIFAR-10 (BASELINE.json configs[3]): 3x3 stem, 4 stages x 2 basic
                    blocks (64/128/256/512), global average pool, dense 10; 11.17M params
"""
from __future__ import annotations

import json
import os

from .keras import layers_from_keras
from .layers import (Activation, BatchNorm, Conv2D, Dense, Dropout, Flatten, GlobalAveragePooling2D,
                     MaxPooling2D, ResidualBlock)
from .net import Net

REFERENCE_MODEL_JSON = "/root/reference/experiment/mnist/model.json"
_BUNDLED_TOPOLOGY = os.path.join(os.path.dirname(__file__), "keras_cnn_topology.json")


def mlp_mnist_layers():
    return [Flatten(name="flatten_1"), Dense(10, "relu", name="dense_1"), Dense(10, "softmax", name="dense_2")], (28, 28, 1)


def lenet5_layers():
    return [
        Conv2D(6, 5, 1, "same", "relu", name="conv2d_1"),
        MaxPooling2D(2, name="max_pooling2d_1"),
        Conv2D(16, 5, 1, "valid", "relu", name="conv2d_2"),
        MaxPooling2D(2, name="max_pooling2d_2"),
        Flatten(name="flatten_1"),
        Dense(120, "relu", name="dense_1"),
        Dense(84, "relu", name="dense_2"),
        Dense(10, "softmax", name="dense_3"),
    ], (28, 28, 1)


def keras_cnn_topology() -> dict:
    """modelTopology of the reference's model.json (bundled copy of the topology JSON; no weights)."""
    for p in (_BUNDLED_TOPOLOGY, REFERENCE_MODEL_JSON):
        if os.path.exists(p):
            with open(p) as f:
                d = json.load(f)
            return d.get("modelTopology", d)
    raise FileNotFoundError("keras CNN topology not found")


def keras_cnn_layers():
    return layers_from_keras(keras_cnn_topology())


def resnet18_cifar_layers(num_classes: int = 10):
    ls = [Conv2D(64, 3, 1, 1, use_bias=False, name="stem/conv", kernel_initializer="he_normal"),
          BatchNorm(relu=True, name="stem/bn")]
    cin = 64
    for stage, (f, s) in enumerate([(64, 1), (128, 2), (256, 2), (512, 2)]):
        for b in range(2):
            ls.append(ResidualBlock(f, s if b == 0 else 1, name=f"layer{stage + 1}.{b}"))
            cin = f
    ls += [GlobalAveragePooling2D(name="gap"), Dense(num_classes, "linear", name="fc")]
    return ls, (32, 32, 3)


MODELS = {
    "mlp_mnist": mlp_mnist_layers,
    "lenet5": lenet5_layers,
    "keras_cnn": keras_cnn_layers,
    "resnet18_cifar": resnet18_cifar_layers,
}


def build_model(name: str, device="cuda", seed: int = 0) -> Net:
    if name not in MODELS:
        raise KeyError(f"unknown model {name!r}; choose from {sorted(MODELS)}")
    layers, in_shape = MODELS[name]()
    return Net(layers, in_shape, device=device, name=name, seed=seed)
