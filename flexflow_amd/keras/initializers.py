"""Keras initializers -> flexflow_amd.core initializers (reference keras/initializers.py)."""
from __future__ import annotations

from ..core import initializers as core_init


class Initializer:
    def ff(self):
        raise NotImplementedError


class DefaultInitializer(Initializer):
    def ff(self):
        return None  # the op's own default (Glorot-uniform weights, zero bias)


class Zeros(Initializer):
    def ff(self):
        return core_init.ZeroInitializer()


class Ones(Initializer):
    def ff(self):
        return core_init.ConstantInitializer(1.0)


class Constant(Initializer):
    def __init__(self, value=0.0):
        self.value = float(value)

    def ff(self):
        return core_init.ConstantInitializer(self.value)


class GlorotUniform(Initializer):
    def __init__(self, seed=0):
        self.seed = int(seed or 0)

    def ff(self):
        return core_init.GlorotUniformInitializer(self.seed)


class RandomUniform(Initializer):
    def __init__(self, minval=-0.05, maxval=0.05, seed=0):
        self.minval, self.maxval, self.seed = minval, maxval, int(seed or 0)

    def ff(self):
        return core_init.UniformInitializer(self.seed, self.minval, self.maxval)


class RandomNormal(Initializer):
    def __init__(self, mean=0.0, stddev=0.05, seed=0):
        self.mean, self.stddev, self.seed = mean, stddev, int(seed or 0)

    def ff(self):
        return core_init.NormInitializer(self.seed, self.mean, self.stddev)


_BY_NAME = {"glorot_uniform": GlorotUniform, "zeros": Zeros, "ones": Ones, "uniform": RandomUniform,
            "random_uniform": RandomUniform, "normal": RandomNormal, "random_normal": RandomNormal}


def get(spec):
    if spec is None:
        return None
    if isinstance(spec, Initializer):
        return spec
    if isinstance(spec, str):
        return _BY_NAME[spec]()
    raise TypeError(f"unsupported initializer {spec!r}")
