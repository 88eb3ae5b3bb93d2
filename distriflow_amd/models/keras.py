"""Keras / tf.js ``LayersModel`` topology <-> engine layers.

Reads the ``modelTopology`` of a tf.js ``model.json`` and writes it back, so a DistriFlow user's model
files load directly.  The reference wraps any ``tf.LayersModel`` fetched by URL
(/root/reference/src/common/utils.ts:236-244, src/common/models.ts:92-100); its shipped model is a
Keras 2.1.4 Sequential (/root/reference/experiment/mnist/model.json:1).  Supported:

* ``Sequential`` models, and functional ``Model`` / ``Functional`` graphs that are a single chain
  (every layer consumes the previous one: what a Sequential exported through the functional API is);
* InputLayer, Conv2D, Dense, Activation (relu, relu6, sigmoid, tanh, elu, selu, softplus, softsign,
  hard_sigmoid, swish / silu, exponential, linear; softmax / sigmoid as the output), MaxPooling2D and
  AveragePooling2D (any pool / strides, 'valid' or 'same'), GlobalAveragePooling2D,
  GlobalMaxPooling2D, Dropout, Flatten, BatchNormalization — channels_last only.
"""
from __future__ import annotations

from .layers import (Activation, AveragePooling2D, BatchNorm, Conv2D, Dense, Dropout, Flatten,
                     GlobalAveragePooling2D, GlobalMaxPooling2D, Layer, MaxPooling2D)


def _chain_order(layer_cfgs: list, model_cfg: dict) -> list:
    """Layers of a functional graph in execution order; raises unless the graph is one chain."""
    by_name = {lc.get("name") or lc["config"].get("name"): lc for lc in layer_cfgs}

    def parents(lc):
        nodes = lc.get("inbound_nodes") or []
        if not nodes:
            return []
        if len(nodes) != 1:
            raise NotImplementedError(f"layer {lc['config'].get('name')!r} is applied more than once (shared layer)")
        node = nodes[0]
        if isinstance(node, dict):  # Keras 3 style {"args": [...], "kwargs": {}}
            args = node.get("args", [])
            names = [a["config"]["keras_history"][0] for a in args if isinstance(a, dict) and "config" in a]
        else:  # Keras 2 style [[name, node_index, tensor_index, kwargs], ...]
            names = [inb[0] for inb in node]
        return names

    outs = model_cfg.get("output_layers") or []
    if len(outs) != 1:
        raise NotImplementedError("functional models must have exactly one output")
    order = []
    name = outs[0][0] if isinstance(outs[0], (list, tuple)) else outs[0]
    seen = set()
    while True:
        if name in seen:
            raise ValueError("cycle in the layer graph")
        seen.add(name)
        lc = by_name[name]
        order.append(lc)
        ps = parents(lc)
        if not ps:
            break
        if len(ps) != 1:
            raise NotImplementedError(f"layer {name!r} has {len(ps)} inputs: only single-chain graphs are supported "
                                      "(no Add / Concatenate joins)")
        name = ps[0]
    order.reverse()
    if len(order) != len(layer_cfgs):
        raise NotImplementedError("functional graph has branches that do not reach the output")
    return order


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
    layer_cfgs = cfg["layers"] if isinstance(cfg, dict) else cfg
    if cls in ("Model", "Functional"):
        layer_cfgs = _chain_order(layer_cfgs, cfg)
    elif cls not in ("Sequential", None):
        raise NotImplementedError(f"model class {cls!r} (supported: Sequential, single-chain functional Model)")
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
        elif k in ("MaxPooling2D", "AveragePooling2D"):
            cls_ = MaxPooling2D if k == "MaxPooling2D" else AveragePooling2D
            layers.append(cls_(tuple(c.get("pool_size", [2, 2])), c.get("strides"), c.get("padding", "valid"),
                               name=name))
        elif k == "GlobalAveragePooling2D":
            layers.append(GlobalAveragePooling2D(name=name))
        elif k == "GlobalMaxPooling2D":
            layers.append(GlobalMaxPooling2D(name=name))
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
        elif isinstance(l, GlobalMaxPooling2D):
            cls = "GlobalMaxPooling2D"
            c["data_format"] = "channels_last"
        elif isinstance(l, MaxPooling2D):
            cls = "AveragePooling2D" if isinstance(l, AveragePooling2D) else "MaxPooling2D"
            c.update(l.config())
            c["data_format"] = "channels_last"
        elif isinstance(l, GlobalAveragePooling2D):
            cls = "GlobalAveragePooling2D"
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
