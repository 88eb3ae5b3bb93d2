"""Branching Keras functional graphs: merge layers and the graph layer that runs a DAG of engine layers.

The reference trains whatever ``tf.LayersModel`` its ``fetchModel`` returns (/root/reference/src/common/
utils.ts:236-244, src/common/models.ts:92-100): Sequential models and functional graphs alike.  Keras
functional graphs join branches with merge layers (Add, Subtract, Multiply, Average, Maximum, Minimum,
Concatenate) and let one layer's output feed several consumers.  The engine's planner (models/net.py)
schedules a chain of layers; a branching region of a graph becomes ONE :class:`GraphLayer` in that chain:

* forward: its nodes in topological order, each an engine layer (same kernels, same preallocated
  buffers) or a merge node (csrc/merge.hip, one launch);
* backward: reverse topological order; a node's output gradient is the sum of its consumers'
  contributions (native add), relu' of a fused-ReLU producer is applied to each contribution by the
  graph (the layers inside run with ``in_relu`` off), merge nodes split their gradient per input.

The sequential head and tail of a graph stay ordinary chain layers, so the planner's fusions (fused
conv+pool, the fused dense head with softmax-CE) still apply to them.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import ops
from .layers import Activation, BatchNorm, Conv2D, Dense, Layer


class Merge(Layer):
    """A Keras merge layer: ``kind`` in ops.MERGE_KINDS; inputs share the batch and spatial shape
    (Concatenate: channels, the last axis, side by side)."""

    def __init__(self, kind: str, name=None, axis: int = -1):
        if kind not in ops.MERGE_KINDS:
            raise NotImplementedError(f"Keras merge layer {kind}")
        super().__init__(name or kind.lower())
        self.kind = kind
        self.axis = int(axis)  # Keras axis, batch axis included (Concatenate only)
        self.in_shapes: list = []

    def build_multi(self, shapes: list) -> tuple:
        shapes = [tuple(s) for s in shapes]
        if len(shapes) < 2 or len(shapes) > 8:
            raise NotImplementedError(f"{self.kind} of {len(shapes)} inputs (2..8 supported)")
        if self.kind == "Subtract" and len(shapes) != 2:
            raise ValueError("Subtract takes exactly two inputs")
        if self.kind == "Concatenate":
            # Keras counts the batch axis: rank-r inputs (r = len(shape) + 1) concatenate on the last axis
            # when axis is -1 or r - 1; any other axis is not the channel / feature axis
            ranks = {len(s) + 1 for s in shapes}
            if len(ranks) != 1:
                raise ValueError(f"Concatenate inputs of different rank: {shapes}")
            r = ranks.pop()
            if self.axis not in (-1, r - 1):
                raise NotImplementedError(f"Concatenate on axis {self.axis} of rank-{r} inputs (only the last axis)")
            lead = {s[:-1] for s in shapes}
            if len(lead) != 1:
                raise ValueError(f"Concatenate inputs differ outside the channel axis: {shapes}")
            out = shapes[0][:-1] + (sum(s[-1] for s in shapes),)
        else:
            if len(set(shapes)) != 1:
                raise ValueError(f"{self.kind} inputs must share one shape: {shapes}")
            out = shapes[0]
        self.in_shapes = shapes
        self.in_shape = shapes[0]
        self.out_shape = out
        return out

    def alloc(self, B, device, dtype, ws):
        self.out = torch.empty((B,) + self.out_shape, device=device, dtype=dtype)
        self.grads = [torch.empty((B,) + s, device=device, dtype=dtype) for s in self.in_shapes]

    def forward_multi(self, xs: list, training: bool):
        self.xs = xs
        ops.merge_fwd(xs, self.out, self.kind)
        return self.out

    def backward_multi(self, dy) -> list:
        ops.merge_bwd(self.xs, dy, self.grads, self.kind)
        return self.grads

    def config(self):
        return {"axis": -1} if self.kind == "Concatenate" else {}


class GraphLayer(Layer):
    """A DAG of engine layers.  ``nodes``: [(layer, [input ids])] in topological order, where input id 0
    is the graph input and id k >= 1 is node k - 1's output; the last node is the graph output."""
    has_params = True

    def __init__(self, nodes: list, name: Optional[str] = None):
        super().__init__(name or "graph")
        self.nodes = [(l, list(ins)) for l, ins in nodes]
        for l, ins in self.nodes:
            if isinstance(l, Merge) != (len(ins) > 1):
                raise ValueError(f"node {l.name}: merge layers take several inputs, other layers exactly one")

    def sublayers(self) -> list:
        return [l for l, _ in self.nodes]

    def bind_store(self, store):
        self.store = store
        for l in self.sublayers():
            l.store = store

    def specs(self):
        out = []
        for l in self.sublayers():
            out += l.specs()
        return out

    def build(self, in_shape):
        self.in_shape = tuple(in_shape)
        shapes = [self.in_shape]
        for l, ins in self.nodes:
            if isinstance(l, Merge):
                shapes.append(l.build_multi([shapes[i] for i in ins]))
            else:
                shapes.append(l.build(shapes[ins[0]]))
        self.out_shape = shapes[-1]
        self.relu = bool(self.nodes[-1][0].relu)  # the chain consumer applies relu' of the graph output
        # consumers of every value (0 = graph input) and whether a value is a fused-ReLU output
        self.consumers = {k: [] for k in range(len(self.nodes) + 1)}
        for n, (l, ins) in enumerate(self.nodes):
            for i in ins:
                self.consumers[i].append(n)
        return self.out_shape

    def alloc(self, B, device, dtype, ws):
        n = len(self.nodes)
        for k, (l, ins) in enumerate(self.nodes):
            # relu' of a producer is applied by the graph to each gradient contribution (a layer's own
            # in_relu fusion covers one consumer; here a value may have several)
            l.in_relu = False
            l.grad_premasked = False
            # a node needs its input gradient unless every input is the graph input and the graph itself
            # needs none
            l.need_dx = self.need_dx or any(i != 0 for i in ins)
            l.alloc(B, device, dtype, ws)
        # gradient accumulators of values with several consumers (value 0: the graph input)
        self.acc = {}
        for v in range(n + 1):
            if len(self.consumers[v]) > 1 and (v > 0 or self.need_dx):
                shape = self.in_shape if v == 0 else self.nodes[v - 1][0].out_shape
                self.acc[v] = torch.empty((B,) + tuple(shape), device=device, dtype=dtype)
        self.out = self.nodes[-1][0].out
        self.dx = None

    def _value_relu(self, v: int) -> bool:
        return v > 0 and bool(self.nodes[v - 1][0].relu)

    def forward(self, x, training):
        self.x = x
        vals = [x]
        for l, ins in self.nodes:
            if isinstance(l, Merge):
                vals.append(l.forward_multi([vals[i] for i in ins], training))
            else:
                vals.append(l.forward(vals[ins[0]], training))
        self.vals = vals
        self.out = vals[-1]
        return self.out

    def backward(self, dy):
        n = len(self.nodes)
        grads: dict = {n: dy}
        pending = {v: len(c) for v, c in self.consumers.items()}
        for k in range(n - 1, -1, -1):
            l, ins = self.nodes[k]
            g = grads.pop(k + 1, None)
            if g is None:  # a dead branch (its output reaches nothing): no gradient flows
                continue
            if isinstance(l, Merge):
                contrib = l.backward_multi(g)
            else:
                d = l.backward(g)
                contrib = [d]
            for i, c in zip(ins, contrib):
                if c is None or (i == 0 and not self.need_dx):
                    continue
                if self._value_relu(i):
                    ops.relu_bwd(self.vals[i], c, c)  # relu' of the producer (c is this consumer's buffer)
                if i in self.acc:
                    if i not in grads:
                        grads[i] = self.acc[i]
                        grads[i].copy_(c)
                    else:
                        ops.add_act(grads[i], c, grads[i])
                else:
                    grads[i] = c
                pending[i] -= 1
        self.dx = grads.get(0)
        if self.dx is not None and self.in_relu:  # the graph input is a fused-ReLU output of the chain
            ops.relu_bwd(self.x, self.dx, self.dx)
        return self.dx

    def config(self):
        return {}


def split_chain(nodes: list) -> tuple:
    """(head, middle, tail) of a node list [(layer, [input ids])] (ids as in GraphLayer): head / tail are
    the maximal single-input, single-consumer chains at either end (ordinary engine layers), middle the
    branching region in between as GraphLayer nodes re-numbered from its own input, or None."""
    n = len(nodes)
    cons = {k: 0 for k in range(n + 1)}
    for _, ins in nodes:
        for i in ins:
            cons[i] += 1
    # head: node k takes exactly value k (its predecessor) and value k has one consumer
    h = 0
    while h < n and nodes[h][1] == [h] and cons[h] == 1 and not isinstance(nodes[h][0], Merge):
        h += 1
    # tail: walking back from the output while the node's single input is the previous node's value and
    # that value has one consumer
    t = n
    while t - 1 > h and nodes[t - 1][1] == [t - 1] and cons[t - 1] == 1 and not isinstance(nodes[t - 1][0], Merge):
        t -= 1
    if h == n:
        return [l for l, _ in nodes], None, []
    head = [l for l, _ in nodes[:h]]
    tail = [l for l, _ in nodes[t:]]
    mid = []
    for l, ins in nodes[h:t]:
        if any(i < h for i in ins):
            raise NotImplementedError("a branch reads a value from before the branching region")
        mid.append((l, [i - h for i in ins]))
    return head, mid, tail
