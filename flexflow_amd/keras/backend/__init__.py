"""Keras backend functions as layers (reference keras/backend/backend_functions.py + internal.py)."""
from __future__ import annotations

from ..layers import Layer


class _Unary(Layer):
    op = "exp"

    def __init__(self, scalar=None, **kw):
        super().__init__(**kw)
        self.scalar = scalar

    def _lower(self, ff, xs):
        fn = getattr(ff, self.op)
        t = fn(xs[0], self.scalar) if self.scalar is not None else fn(xs[0])
        return [self._track(ff, t)]


class Sin(_Unary):
    op = "sin"


class Cos(_Unary):
    op = "cos"


class Exp(_Unary):
    op = "exp"


class Rsqrt(_Unary):
    op = "rsqrt"


class Pow(_Unary):
    op = "pow"


class ReduceSum(Layer):
    def __init__(self, axis=None, keepdims=False, **kw):
        super().__init__(**kw)
        self.axis, self.keepdims = axis, keepdims

    def compute_output_shape(self, in_shapes):
        s = list(in_shapes[0])
        axes = [self.axis] if isinstance(self.axis, int) else list(self.axis)
        axes = [a - 1 if a > 0 else len(s) + a for a in axes]  # keras axes count the batch dim
        if self.keepdims:
            for a in axes:
                s[a] = 1
            return [tuple(s)]
        return [tuple(d for i, d in enumerate(s) if i not in axes)]

    def _lower(self, ff, xs):
        axes = [self.axis] if isinstance(self.axis, int) else list(self.axis)
        axes = [a if a >= 0 else len(xs[0].dims) + a for a in axes]
        return [self._track(ff, ff.reduce_sum(xs[0], axes, self.keepdims))]


class BatchMatmul(Layer):
    def compute_output_shape(self, in_shapes):
        a, b = in_shapes
        return [a[:-1] + (b[-1],)]

    def _lower(self, ff, xs):
        return [self._track(ff, ff.batch_matmul(xs[0], xs[1]))]


class Gather(Layer):
    """torch.gather semantics along a non-batch `axis` (keras axes count the batch dim):
    out[b, i, j] = x[b, idx[b, i, j], j] for axis 1 (reference keras/backend/internal.py gather)."""

    def __init__(self, axis=1, **kw):
        super().__init__(**kw)
        self.axis = int(axis)

    def compute_output_shape(self, in_shapes):
        return [tuple(in_shapes[1])]

    def output_dtypes(self, in_dtypes):
        return [in_dtypes[0]]

    def _lower(self, ff, xs):
        ax = self.axis if self.axis >= 0 else len(xs[0].dims) + self.axis
        return [self._track(ff, ff.gather(xs[0], xs[1], ax))]


def gather(x, index, axis=1):
    return Gather(axis)([x, index])


def backend():
    return "flexflow_amd"


_IMAGE_DATA_FORMAT = ["channels_first"]


def image_data_format():
    return _IMAGE_DATA_FORMAT[0]


def set_image_data_format(fmt):
    if fmt != "channels_first":
        raise NotImplementedError("only channels_first (NCHW) tensors, as the reference")
    _IMAGE_DATA_FORMAT[0] = fmt


def get_value(x):
    """Weights of a layer / the value of a weight as numpy (tensors are symbolic until compiled)."""
    import numpy as np
    if hasattr(x, "get_weights"):
        return x.get_weights()
    return np.asarray(x)


def set_value(x, value):
    if hasattr(x, "set_weights"):
        x.set_weights(value if isinstance(value, (list, tuple)) else [value])
        return
    raise TypeError("set_value: expects a layer")


def batch_dot(x, y):
    return BatchMatmul()([x, y])


def sin(x):
    return Sin()(x)


def cos(x):
    return Cos()(x)


def exp(x):
    return Exp()(x)


def rsqrt(x):
    return Rsqrt()(x)


def pow(x, a):
    return Pow(a)(x)


def sum(x, axis=None, keepdims=False):
    return ReduceSum(axis, keepdims)(x)
