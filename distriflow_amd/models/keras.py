"""Keras / tf.js ``LayersModel`` topology <-> engine layers.

Reads the ``modelTopology`` of a tf.js ``model.json`` (Keras 2.x Sequential, as shipped in
/root/reference/experiment/mnist/model.json:1) and writes it back, so a DistriFlow user's model files
load directly.  Supported classes: InputLayer, Conv2D, Dense, Activation, MaxPooling2D, Dropout,
Flatten, BatchNormalization (channels_last only).
"""
from __future__ import annotations

from .layers import Activation, BatchNorm, Conv2D, Dense, Dropout, Flatten, Layer, MaxPooling2D


def _init_name(cfg):
    ki = cfg.get("kernel_initializer") or {}
    cls = ki.get("class_name", "VarianceScaling") if isinstance(ki, dict) else str(ki)
    c = ki.get("config", {}) if isinstance(ki, dict) else {}
    if cls in ("GlorotUniform", "glorot_uniform"):
        return "glorot_uniform"
    if cls == "VarianceScaling":
        mode, dist, scale = c.get("mode", "fan_avg"), c.get("distribution", "uniform"), c.get("scale", 1.0)
        if mode == "fan_avg" and "uniform" in dist and scale == 1.0:
            return "glorot_uniform"
        if mode == "fan_in" and scale == 2.0:
            return "he_normal"
        if mode == "fan_in" and scale == 1.0 and "uniform" in dist:
            return "lecun_uniform"
    if cls in ("HeNormal", "he_normal"):
        return "he_normal"
    return "glorot_uniform"


def layers_from_keras(model_config: dict) -> tuple[list[Layer], tuple]:
    """-> (layers, input_shape HWC/F) from ``modelTopology.model_config`` (or ``modelTopology`` itself)."""
    if "model_config" in model_config:
        model_config = model_config["model_config"]
    cls = model_config.get("class_name")
    cfg = model_config.get("config")
    if cls not in ("Sequential", None):
        raise NotImplementedError(f"only Sequential models are supported, got {cls}")
    layer_cfgs = cfg["layers"] if isinstance(cfg, dict) else cfg
    layers: list[Layer] = []
    input_shape = None
    for lc in layer_cfgs:
        c = lc["config"]
        name = c.get("name")
        if input_shape is None and c.get("batch_input_shape"):
            input_shape = tuple(int(v) for v in c["batch_input_shape"][1:])
        k = lc["class_name"]
        if k == "InputLayer":
            continue
        if c.get("data_format", "channels_last") != "channels_last":
            raise NotImplementedError("channels_first layers")
        if k == "Conv2D":
            if tuple(c.get("dilation_rate", [1, 1])) != (1, 1):
                raise NotImplementedError("dilated conv")
            layers.append(Conv2D(c["filters"], tuple(c["kernel_size"]), tuple(c.get("strides", [1, 1])),
                                 c.get("padding", "valid"), c.get("activation", "linear"), c.get("use_bias", True),
                                 name=name, kernel_initializer=_init_name(c)))
        elif k == "Dense":
            layers.append(Dense(c["units"], c.get("activation", "linear"), c.get("use_bias", True), name=name,
                                kernel_initializer=_init_name(c)))
        elif k == "Activation":
            layers.append(Activation(c["activation"], name=name))
        elif k == "MaxPooling2D":
            if c.get("padding", "valid") != "valid":
                raise NotImplementedError("MaxPooling2D padding='same'")
            layers.append(MaxPooling2D(tuple(c.get("pool_size", [2, 2])), c.get("strides"), name=name))
        elif k == "Dropout":
            layers.append(Dropout(c["rate"], name=name))
        elif k == "Flatten":
            layers.append(Flatten(name=name))
        elif k == "BatchNormalization":
            layers.append(BatchNorm(momentum=1.0 - c.get("momentum", 0.99), eps=c.get("epsilon", 1e-3), name=name))
        else:
            raise NotImplementedError(f"Keras layer {k}")
    if input_shape is None:
        raise ValueError("model_config has no batch_input_shape")
    return layers, input_shape


def keras_config_from_layers(layers: list[Layer], input_shape: tuple, name: str = "sequential") -> dict:
    """Inverse of :func:`layers_from_keras` (Keras 2.x Sequential JSON, as tf.js writes it)."""
    out = []
    first = True
    for l in layers:
        c: dict = {"name": l.name, "trainable": True}
        if first:
            c["batch_input_shape"] = [None, *input_shape]
            c["dtype"] = "float32"
            first = False
        if isinstance(l, Conv2D):
            cls = "Conv2D"
            c.update(l.config())
            c.update({"data_format": "channels_last", "dilation_rate": [1, 1],
                      "kernel_initializer": {"class_name": "VarianceScaling",
                                             "config": {"scale": 1.0, "mode": "fan_avg", "distribution": "uniform",
                                                        "seed": None}},
                      "bias_initializer": {"class_name": "Zeros", "config": {}}})
        elif isinstance(l, Dense):
            cls = "Dense"
            c.update(l.config())
            c.update({"kernel_initializer": {"class_name": "VarianceScaling",
                                             "config": {"scale": 1.0, "mode": "fan_avg", "distribution": "uniform",
                                                        "seed": None}},
                      "bias_initializer": {"class_name": "Zeros", "config": {}}})
        elif isinstance(l, Activation):
            cls = "Activation"
            c.update(l.config())
        elif isinstance(l, MaxPooling2D):
            cls = "MaxPooling2D"
            c.update(l.config())
            c["data_format"] = "channels_last"
        elif isinstance(l, Dropout):
            cls = "Dropout"
            c.update(l.config())
        elif isinstance(l, Flatten):
            cls = "Flatten"
        elif isinstance(l, BatchNorm):
            cls = "BatchNormalization"
            c.update({"momentum": 1.0 - l.momentum, "epsilon": l.eps, "axis": -1})
        else:
            raise NotImplementedError(f"cannot export {type(l).__name__} to Keras JSON")
        out.append({"class_name": cls, "config": c})
    return {"class_name": "Sequential", "config": {"name": name, "layers": out}}
