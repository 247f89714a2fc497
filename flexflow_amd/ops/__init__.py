"""Operator library. Importing this package registers every op in `OPS`."""
from .base import OPS, OpCtx, OpImpl, WeightSpec, register, torch_dtype  # noqa: F401
from . import attention, conv, elementwise, embedding, linear, misc, norm, parallel_ops, rnn, shape, softmax  # noqa: F401
