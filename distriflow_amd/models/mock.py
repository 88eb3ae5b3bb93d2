"""MockModel — protocol-test double (reference /root/reference/src/test/mock_model.ts:5-46).

Implements both the server and client model contracts; ``fit`` returns the variables themselves as
"gradients", ``update`` is a no-op, ``save`` bumps a timestamp version, ``predict`` is the identity and
``evaluate`` returns ``[0]`` — so role tests exercise the protocol without any training math.
"""
from __future__ import annotations

import time

import torch

from .distri_model import DistriModel


class MockModel(DistriModel):
    is_distri_client_model = True
    is_distri_server_model = True

    def __init__(self, vars, input_shape=(1,), output_shape=(1,)):
        self.vars = [torch.as_tensor(v).clone().float() for v in vars]
        self.version = "0"
        self._in, self._out = list(input_shape), list(output_shape)
        self.device = "cpu"

    def setup(self):
        pass

    def save(self):
        last = int(self.version) if str(self.version).isdigit() else 0
        self.version = str(max(int(time.time() * 1000), last + 1))
        return self.version

    def fit(self, x, y):
        return [v.clone() for v in self.vars]

    def update(self, grads):
        pass

    def update_flat(self, flat_grad, scale=1.0):
        pass

    def set_vars(self, vals):
        for v, n in zip(self.vars, vals):
            v.copy_(torch.as_tensor(n).reshape(v.shape))

    def get_vars(self):
        return self.vars

    def predict(self, x):
        return x

    def evaluate(self, x, y):
        return [0]

    @property
    def input_shape(self):
        return self._in

    @property
    def output_shape(self):
        return self._out
