"""Keras losses (reference keras/losses.py) -> LossType."""
from __future__ import annotations

from ..type import DataType, LossType


class Loss:
    type = None
    label_dtype = DataType.DT_FLOAT


class CategoricalCrossentropy(Loss):
    type = LossType.LOSS_CATEGORICAL_CROSSENTROPY


class SparseCategoricalCrossentropy(Loss):
    type = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY
    label_dtype = DataType.DT_INT32


class MeanSquaredError(Loss):
    type = LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE


class Identity(Loss):
    type = LossType.LOSS_IDENTITY


_BY_NAME = {"categorical_crossentropy": CategoricalCrossentropy,
            "sparse_categorical_crossentropy": SparseCategoricalCrossentropy,
            "mean_squared_error": MeanSquaredError, "mse": MeanSquaredError, "identity": Identity}


def get(spec):
    if isinstance(spec, Loss):
        return spec
    if spec not in _BY_NAME:
        raise ValueError(f"unsupported loss {spec!r}")
    return _BY_NAME[spec]()
