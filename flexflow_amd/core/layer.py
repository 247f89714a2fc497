"""Layer: a node of the pre-parallelization graph (reference include/flexflow/layer.h:8-63).

Holds op type, attributes (the reference's int/float/vector properties), input/output Tensors and
weight Parameters. The op semantics live in flexflow_amd.ops (`OPS[op_type]`).
"""
from __future__ import annotations

import itertools
from typing import Any, Dict, List, Optional

from ..type import DataType, OperatorType
from .tensor import Parameter, Tensor

_layer_guid = itertools.count(1000000)


class Layer:
    def __init__(self, model, op_type: OperatorType, name: Optional[str], inputs: List[Tensor],
                 attrs: Dict[str, Any]):
        from ..ops import OPS  # late import (registry)
        self.model = model
        self.op_type = op_type
        self.guid = next(_layer_guid)
        base = op_type.name[3:].lower()
        self.name = name or f"{base}_{self.guid - 1000000}"
        self.inputs = list(inputs)
        self.attrs = dict(attrs)
        self.outputs: List[Tensor] = []
        self.weights: List[Parameter] = []
        impl_cls = OPS[op_type]
        out_dims, out_dtypes, wspecs = impl_cls.infer(self.attrs, [t.dims for t in self.inputs],
                                                      [t.data_type for t in self.inputs])
        for i, (d, dt) in enumerate(zip(out_dims, out_dtypes)):
            self.outputs.append(Tensor(d, dt, owner_layer=self, owner_idx=i, name=f"{self.name}:out{i}"))
        for i, ws in enumerate(wspecs):
            p = Parameter(ws.dims, ws.dtype, owner_layer=self, owner_idx=i, name=f"{self.name}.{ws.name}",
                          initializer=ws.init)
            p.trainable = ws.trainable
            p.short_name = ws.name
            self.weights.append(p)
        self.impl = impl_cls(self)

    # reference Op python API (flexflow_cffi.py Op:57-100)
    def get_number_parameters(self):
        return len(self.weights)

    def get_parameter_by_id(self, i):
        return self.weights[i]

    def get_number_inputs(self):
        return len(self.inputs)

    def get_input_by_id(self, i):
        return self.inputs[i]

    def get_number_outputs(self):
        return len(self.outputs)

    def get_output_by_id(self, i):
        return self.outputs[i]

    def get_output_tensor(self):
        return self.outputs[0]

    def init(self, model):
        """Re-initialise this op's weights with their initializers (reference Op.init)."""
        model.executor.init_weights(model.config.seed, only=[self])

    def forward(self, model):
        """Run this op alone on the current values of its inputs (reference Op.forward)."""
        model.executor.forward_layer(self)

    def _add_to_model(self, model):
        """Layers join their model when they are built (reference Op._add_to_model)."""
        assert self in model.layers

    def get_input_tensor(self):
        return self.inputs[0]

    def get_weight_tensor(self):
        return self.weights[0] if self.weights else None

    def get_bias_tensor(self):
        return self.weights[1] if len(self.weights) > 1 else None

    def __repr__(self):
        return f"Layer({self.name}, {self.op_type.name}, in={[list(t.dims) for t in self.inputs]}, " \
               f"out={[list(t.dims) for t in self.outputs]})"


# Per-operator layer classes of the reference Python API (flexflow_cffi.py: Exp, Conv2D, Linear, ...,
# returned by get_layer_by_id / get_layers through convert_op_handle_to_op). Here every layer is a
# Layer; the op-specific class is a marker subclass assigned at creation, so isinstance checks and
# type(layer).__name__ behave as in the reference.
_OP_CLASS_NAMES = {
    "OP_EXP": "Exp", "OP_SIN": "Sin", "OP_COS": "Cos", "OP_EW_ADD": "Add", "OP_EW_SUB": "Subtract",
    "OP_EW_MUL": "Multiply", "OP_EW_DIV": "Divide", "OP_EW_MAX": "Max", "OP_EW_MIN": "Min",
    "OP_REDUCE_SUM": "ReduceSum", "OP_CONV2D": "Conv2D", "OP_POOL2D": "Pool2D", "OP_LINEAR": "Linear",
    "OP_FLAT": "Flat", "OP_SOFTMAX": "Softmax", "OP_EMBEDDING": "Embedding", "OP_CONCAT": "Concat",
    "OP_BATCHNORM": "BatchNorm", "OP_LAYERNORM": "LayerNorm", "OP_DROPOUT": "Dropout",
    "OP_SCALAR_MULTIPLY": "ScalarMultiply", "OP_SCALAR_ADD": "ScalarAdd", "OP_SCALAR_SUB": "ScalarSub",
    "OP_SCALAR_TRUE_DIV": "ScalarTrueDiv", "OP_RSQRT": "Rsqrt", "OP_POW": "Pow", "OP_MEAN": "Mean",
    "OP_RELU": "Relu", "OP_GELU": "Gelu", "OP_SIGMOID": "Sigmoid", "OP_TANH": "Tanh", "OP_ELU": "Elu",
    "OP_BATCHMATMUL": "Batch_Matmul", "OP_SPLIT": "Split", "OP_RESHAPE": "Reshape", "OP_GATHER": "Gather",
    "OP_IDENTITY": "Identity", "OP_TRANSPOSE": "Transpose", "OP_REVERSE": "Reverse",
    "OP_MULTIHEAD_ATTENTION": "MultiHeadAttention",
}
OP_CLASSES: Dict[OperatorType, type] = {}
for _op, _cls in _OP_CLASS_NAMES.items():
    if hasattr(OperatorType, _op):
        OP_CLASSES[getattr(OperatorType, _op)] = type(_cls, (Layer,), {"__doc__": f"{_cls} layer (reference flexflow_cffi.{_cls})."})
Batch_Norm = OP_CLASSES.get(OperatorType.OP_BATCHNORM)


def op_class(op_type: OperatorType) -> type:
    return OP_CLASSES.get(op_type, Layer)
