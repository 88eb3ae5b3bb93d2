"""Keras / tf.js ``LayersModel`` topology <-> engine layers.

Reads the ``modelTopology`` of a tf.js ``model.json`` and writes it back, so a DistriFlow user's model
files load directly.  The reference wraps any ``tf.LayersModel`` fetched by URL
(/root/reference/src/common/utils.ts:236-244, src/common/models.ts:92-100); its shipped model is a
Keras 2.1.4 Sequential (/root/reference/experiment/mnist/model.json:1).  Supported:

* ``Sequential`` models, and functional ``Model`` / ``Functional`` graphs with one input and one output:
  chains, and branching graphs whose branches join in merge layers (Add, Subtract, Multiply, Average,
  Maximum, Minimum, Concatenate on the channel axis) or fan out from one layer to several (the
  branching region runs as one :class:`~distriflow_amd.models.graph.GraphLayer`, models/graph.py);
  the logits layer (the output) must be a Dense fed by a single chain;
* InputLayer, Conv2D (any kernel size / strides pair, 'valid' or 'same' -- an odd 'same' total pads the
  bottom / right, as TensorFlow does), Dense, Activation (relu, relu6, sigmoid, tanh, elu, selu, softplus, softsign,
  hard_sigmoid, swish / silu, exponential, linear; softmax / sigmoid as the output), MaxPooling2D and
  AveragePooling2D (any pool / strides, 'valid' or 'same'), GlobalAveragePooling2D,
  GlobalMaxPooling2D, Dropout, Flatten, BatchNormalization — channels_last only.
"""
from __future__ import annotations

from .graph import GraphLayer, Merge, split_chain
from .layers import (Activation, AveragePooling2D, BatchNorm, Conv2D, Dense, Dropout, Flatten,
                     GlobalAveragePooling2D, GlobalMaxPooling2D, Layer, MaxPooling2D)

_MERGES = ("Add", "Subtract", "Multiply", "Average", "Maximum", "Minimum", "Concatenate")


def _inbound_names(lc) -> list:
    """Names of the layers feeding ``lc`` (Keras 2 and Keras 3 JSON); raises for shared layers."""
    nodes = lc.get("inbound_nodes") or []
    if not nodes:
        return []
    if len(nodes) != 1:
        raise NotImplementedError(f"layer {lc['config'].get('name')!r} is applied more than once (shared layer)")
    node = nodes[0]
    if isinstance(node, dict):  # Keras 3 style {"args": [...], "kwargs": {}}
        names = []
        for a in node.get("args", []):
            items = a if isinstance(a, list) else [a]
            names += [x["config"]["keras_history"][0] for x in items if isinstance(x, dict) and "config" in x]
        return names
    return [inb[0] for inb in node]  # Keras 2 style [[name, node_index, tensor_index, kwargs], ...]


def _graph_order(layer_cfgs: list, model_cfg: dict) -> tuple:
    """(configs in topological order, {name: [input names]}) of a one-input, one-output functional
    graph, keeping only what reaches the output."""
    by_name = {lc.get("name") or lc["config"].get("name"): lc for lc in layer_cfgs}
    outs = model_cfg.get("output_layers") or []
    ins = model_cfg.get("input_layers") or []
    if len(outs) != 1:
        raise NotImplementedError("functional models must have exactly one output")
    if len(ins) > 1:
        raise NotImplementedError("functional models must have exactly one input")
    name_of = lambda ref: ref[0] if isinstance(ref, (list, tuple)) else ref  # noqa: E731
    parents = {n: _inbound_names(lc) for n, lc in by_name.items()}
    order, state = [], {}

    def visit(n):  # depth-first post-order from the output
        if state.get(n) == 1:
            raise ValueError("cycle in the layer graph")
        if state.get(n) == 2:
            return
        state[n] = 1
        for p in parents[n]:
            visit(p)
        state[n] = 2
        order.append(n)

    visit(name_of(outs[0]))
    return [by_name[n] for n in order], parents


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


def _make_layer(k: str, c: dict) -> Layer:
    """Engine layer of Keras class ``k`` with config ``c``."""
    name = c.get("name")
    if c.get("data_format", "channels_last") != "channels_last":
        raise NotImplementedError("channels_first layers")
    if k == "Conv2D":
        if tuple(c.get("dilation_rate", [1, 1])) != (1, 1):
            raise NotImplementedError("dilated conv")
        return Conv2D(c["filters"], tuple(c["kernel_size"]), tuple(c.get("strides", [1, 1])), c.get("padding", "valid"),
                      c.get("activation", "linear"), c.get("use_bias", True), name=name,
                      kernel_initializer=_init_name(c))
    if k == "Dense":
        return Dense(c["units"], c.get("activation", "linear"), c.get("use_bias", True), name=name,
                     kernel_initializer=_init_name(c))
    if k == "Activation":
        return Activation(c["activation"], name=name)
    if k in ("MaxPooling2D", "AveragePooling2D"):
        cls_ = MaxPooling2D if k == "MaxPooling2D" else AveragePooling2D
        return cls_(tuple(c.get("pool_size", [2, 2])), c.get("strides"), c.get("padding", "valid"), name=name)
    if k == "GlobalAveragePooling2D":
        return GlobalAveragePooling2D(name=name)
    if k == "GlobalMaxPooling2D":
        return GlobalMaxPooling2D(name=name)
    if k == "Dropout":
        return Dropout(c["rate"], name=name)
    if k == "Flatten":
        return Flatten(name=name)
    if k == "BatchNormalization":
        return BatchNorm(momentum=1.0 - c.get("momentum", 0.99), eps=c.get("epsilon", 1e-3), name=name)
    if k in _MERGES:
        # the axis is checked against the inputs' rank when the graph is built (Merge.build_multi)
        return Merge(k, name=name, axis=int(c.get("axis", -1)) if k == "Concatenate" else -1)
    raise NotImplementedError(f"Keras layer {k}")


def _input_shape_of(lc) -> tuple | None:
    c = lc["config"]
    shp = c.get("batch_input_shape") or c.get("batch_shape")
    return tuple(int(v) for v in shp[1:]) if shp else None


def _graph_layers(order: list, parents: dict) -> tuple:
    """Engine layers of a functional graph: the sequential head and tail as chain layers, the branching
    region in between as one GraphLayer.  Non-relu activations of a Conv2D / Dense INSIDE the branching
    region become their own Activation node (as the chain planner does for chain layers)."""
    input_shape, nodes, value = None, [], {}
    for lc in order:
        k, c = lc["class_name"], lc["config"]
        name = c.get("name")
        if k == "InputLayer" or not parents[name]:
            if k != "InputLayer":
                raise NotImplementedError(f"layer {name!r} has no input")
            input_shape = _input_shape_of(lc)
            value[name] = 0
            continue
        l = _make_layer(k, c)
        srcs = [value[p] for p in parents[name]]
        if isinstance(l, Merge) != (len(srcs) > 1):
            raise NotImplementedError(f"layer {name!r} ({k}) with {len(srcs)} inputs")
        nodes.append((l, srcs))
        value[name] = len(nodes)
    if input_shape is None:
        raise ValueError("the graph has no InputLayer with a batch shape")
    head, mid, tail = split_chain(nodes)
    if mid is None:
        return head, input_shape
    out, newid = [], {0: 0}
    for j, (l, ins) in enumerate(mid, start=1):
        out.append((l, [newid[i] for i in ins]))
        act = getattr(l, "activation", None) if isinstance(l, (Dense, Conv2D)) else None
        if act not in (None, "linear", "relu"):
            if act == "softmax":
                raise NotImplementedError("a softmax activation inside a branching region")
            out.append((Activation(act, name=f"{l.name}/{act}", implicit=True), [len(out)]))
        newid[j] = len(out)  # consumers of node j read its activation's output when one was added
    return head + [GraphLayer(out, name="graph")] + tail, input_shape


def layers_from_keras(model_config: dict) -> tuple[list[Layer], tuple]:
    """-> (layers, input_shape HWC/F) from ``modelTopology.model_config`` (or ``modelTopology`` itself)."""
    if "model_config" in model_config:
        model_config = model_config["model_config"]
    cls = model_config.get("class_name")
    cfg = model_config.get("config")
    layer_cfgs = cfg["layers"] if isinstance(cfg, dict) else cfg
    if cls in ("Model", "Functional"):
        return _graph_layers(*_graph_order(layer_cfgs, cfg))
    if cls not in ("Sequential", None):
        raise NotImplementedError(f"model class {cls!r} (supported: Sequential, functional Model)")
    layers: list[Layer] = []
    input_shape = None
    for lc in layer_cfgs:
        if input_shape is None:
            input_shape = _input_shape_of(lc)
        if lc["class_name"] == "InputLayer":
            continue
        l = _make_layer(lc["class_name"], lc["config"])
        if isinstance(l, Merge):
            raise NotImplementedError("a merge layer in a Sequential model")
        layers.append(l)
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
