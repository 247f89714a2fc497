"""User-facing Tensor / Parameter handles (reference include/flexflow/tensor.h, python
flexflow_cffi.py Tensor:576-850 / Parameter:851-886).

A Tensor is a node in the layer graph (pre-parallelization). After `FFModel.compile()` it is
backed by per-rank shards owned by the executor; `get_tensor`/`set_tensor` gather/scatter the
full logical value through the executor (reference parallel_tensor.cc set_tensor/get_tensor).
"""
from __future__ import annotations

import itertools
from typing import Optional

import numpy as np

from ..type import DataType

_guid = itertools.count(3000000)

NP_DT = {DataType.DT_FLOAT: np.float32, DataType.DT_DOUBLE: np.float64, DataType.DT_INT32: np.int32,
         DataType.DT_INT64: np.int64, DataType.DT_HALF: np.float16, DataType.DT_BOOLEAN: np.bool_,
         DataType.DT_BF16: np.float32}


class Tensor:
    def __init__(self, dims, data_type: DataType = DataType.DT_FLOAT, owner_layer=None, owner_idx: int = 0,
                 create_grad: bool = True, name: Optional[str] = None):
        self.dims = tuple(int(d) for d in dims)
        self.data_type = data_type
        self.owner_layer = owner_layer
        self.owner_idx = owner_idx
        self.create_grad = create_grad
        self.guid = next(_guid)
        self.name = name or f"tensor_{self.guid}"
        self._model = None
        self.mapped = False
        self._attached: Optional[np.ndarray] = None

    # reference API spellings
    @property
    def num_dims(self) -> int:
        return len(self.dims)

    @property
    def shape(self):
        return self.dims

    def get_dims(self):
        return list(self.dims)

    def get_dim(self, i):
        return self.dims[i]

    def is_mapped(self):
        return self.mapped

    # ------------------------------------------------------------------ value access
    def set_tensor(self, ffmodel, np_array):
        ffmodel._set_tensor_value(self, np.asarray(np_array))

    def get_tensor(self, ffmodel):
        return ffmodel._get_tensor_value(self)

    def get_gradients(self, ffmodel, comm_type=None):
        return ffmodel._get_tensor_grad(self)

    def get_model_output_gradients(self, ffmodel, comm_type=None):
        return ffmodel._get_tensor_grad(self)

    def get_model_output_tensor(self, ffmodel):
        return ffmodel._get_tensor_value(self)

    def attach_numpy_array(self, ffmodel, ffconfig=None, np_array=None):
        if np_array is None:  # reference signature (ffconfig, np_array)
            np_array = ffconfig
        self._attached = np.ascontiguousarray(np_array)
        if getattr(ffmodel, "_compiled", False):
            try:
                ffmodel._set_tensor_value(self, self._attached)  # a graph input: feed it now
            except KeyError:
                pass  # not part of the compiled graph (e.g. a whole dataset for a data loader)
        self.mapped = True

    def detach_numpy_array(self, ffconfig=None):
        self._attached = None
        self.mapped = False

    def inline_map(self, ffmodel=None, ffconfig=None):
        self.mapped = True

    def inline_unmap(self, ffmodel=None, ffconfig=None):
        self.mapped = False

    def get_array(self, ffmodel, ffconfig=None):
        """The tensor's values as numpy. Before compile (or when called with an FFConfig, as the
        reference's `get_array(ffconfig, dtype)` after `inline_map`) this is the host array the
        tensor is attached to — writable, and fed to the model at compile."""
        if getattr(ffmodel, "_compiled", False):
            try:
                return self.get_tensor(ffmodel)
            except KeyError:
                pass  # not part of the compiled graph: the host array it is attached to
        if self._attached is None:
            self._attached = np.zeros(tuple(self.dims), dtype=np.int32 if self.data_type in (
                DataType.DT_INT32, DataType.DT_INT64) else np.float32)
        return self._attached

    def get_flat_array(self, ffmodel, ffconfig=None):
        return self.get_tensor(ffmodel).reshape(-1)

    def __repr__(self):
        return f"Tensor({self.name}, dims={list(self.dims)}, {self.data_type.name})"


class Parameter(Tensor):
    """A weight tensor (reference Parameter: set_weights/get_weights)."""

    def __init__(self, dims, data_type=DataType.DT_FLOAT, owner_layer=None, owner_idx=0, name=None,
                 initializer=None):
        super().__init__(dims, data_type, owner_layer, owner_idx, True, name)
        self.initializer = initializer

    def set_weights(self, ffmodel, np_array):
        ffmodel._set_weight_value(self, np.asarray(np_array))

    def get_weights(self, ffmodel):
        return ffmodel._get_weight_value(self)


class RegionNdarray:
    """A numpy-array view of raw memory (reference flexflow_cffi.py RegionNdarray: a region's
    base pointer, shape and byte strides exposed through __array_interface__), e.g.
    np.asarray(RegionNdarray((4, 8), DataType.DT_FLOAT, ptr, (32, 4), False))."""
    __slots__ = ["__array_interface__"]

    def __init__(self, shape, data_type, base_ptr, strides, read_only):
        from ..type import DataType
        typestr = {DataType.DT_FLOAT: "<f4", DataType.DT_INT32: "<i4", DataType.DT_INT64: "<i8",
                   DataType.DT_DOUBLE: "<f8", DataType.DT_HALF: "<f2"}.get(data_type)
        assert typestr is not None, f"RegionNdarray: unsupported data type {data_type}"
        self.__array_interface__ = {"version": 3, "shape": tuple(shape), "typestr": typestr,
                                    "data": (int(base_ptr), bool(read_only)),
                                    "strides": tuple(strides) if strides is not None else None}
