"""Keras optimizers (reference keras/optimizers.py) -> fused HIP SGD / Adam of flexflow_amd.core."""
from __future__ import annotations

from ..core.optimizers import AdamOptimizer, SGDOptimizer


class Optimizer:
    ffhandle = None

    def create_ffhandle(self, ffmodel):
        raise NotImplementedError

    def set_learning_rate(self, lr):
        self.learning_rate = float(lr)
        if self.ffhandle is not None:
            self.ffhandle.set_learning_rate(lr)


class SGD(Optimizer):
    def __init__(self, learning_rate=0.01, momentum=0.0, nesterov=False, weight_decay=0.0, **kw):
        self.learning_rate = float(kw.pop("lr", learning_rate))
        self.momentum, self.nesterov, self.weight_decay = float(momentum), bool(nesterov), float(weight_decay)

    def create_ffhandle(self, ffmodel):
        self.ffhandle = SGDOptimizer(ffmodel, self.learning_rate, self.momentum, self.nesterov, self.weight_decay)
        return self.ffhandle


class Adam(Optimizer):
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-8, weight_decay=0.0, **kw):
        self.learning_rate = float(kw.pop("lr", learning_rate))
        self.beta_1, self.beta_2, self.epsilon, self.weight_decay = beta_1, beta_2, epsilon, weight_decay

    def create_ffhandle(self, ffmodel):
        self.ffhandle = AdamOptimizer(ffmodel, self.learning_rate, self.beta_1, self.beta_2, self.weight_decay,
                                      self.epsilon)
        return self.ffhandle


def get(spec):
    if isinstance(spec, Optimizer):
        return spec
    return {"sgd": SGD, "adam": Adam}[str(spec).lower()]()
