"""keras_exp Tensor (reference python/flexflow/keras_exp/models/tensor.py): the symbolic input of
a keras_exp model, bound to an FFModel tensor at compile."""
from __future__ import annotations

from ...type import DataType

_NP_DT = {"float32": DataType.DT_FLOAT, "int32": DataType.DT_INT32, "int64": DataType.DT_INT64,
          "float64": DataType.DT_DOUBLE, "float16": DataType.DT_HALF}


class Tensor:
    def __init__(self, ffconfig=None, key=0, shape=None, batch_shape=None, dtype="float32"):
        self.key = key
        self.ffconfig = ffconfig
        if batch_shape is None:
            bs = ffconfig.batch_size if ffconfig is not None else None
            batch_shape = (bs,) + tuple(int(s) for s in (shape or ())[1:] if s is not None) \
                if shape is not None and len(shape) and shape[0] is None else (bs,) + tuple(shape or ())
        self.batch_shape = tuple(batch_shape)
        self.dtype_str = dtype if isinstance(dtype, str) else str(dtype)
        self.dtype = _NP_DT.get(self.dtype_str, dtype if isinstance(dtype, DataType) else DataType.DT_FLOAT)
        self.ffhandle = None

    @property
    def num_dims(self):
        return len(self.batch_shape)

    def create_ff_tensor(self, ffmodel):
        self.ffhandle = ffmodel.create_tensor(list(self.batch_shape), self.dtype)
        return self.ffhandle
