"""Weight regularizers (reference keras/regularizers.py). Applied by the executor as a gradient
term before the optimizer step: L2 adds 2*l2*w, L1 adds l1*sign(w)."""
from __future__ import annotations


class Regularizer:
    l1 = 0.0
    l2 = 0.0

    def grad_terms(self):
        return self.l1, self.l2


class L1(Regularizer):
    def __init__(self, l1=0.01):
        self.l1 = float(l1)


class L2(Regularizer):
    def __init__(self, l2=0.01):
        self.l2 = float(l2)


class L1L2(Regularizer):
    def __init__(self, l1=0.0, l2=0.0):
        self.l1, self.l2 = float(l1), float(l2)


def l1(v=0.01):
    return L1(v)


def l2(v=0.01):
    return L2(v)


def get(spec):
    if spec is None or isinstance(spec, Regularizer):
        return spec
    raise TypeError(f"unsupported regularizer {spec!r}")
