"""Element-wise unary / scalar / binary ops, dropout and cast.

Reference: src/ops/element_unary.cc (+.cu), src/ops/element_binary.cc, src/ops/dropout.cc,
src/ops/cast.cc. All run on the vectorised HIP kernels of csrc/kernels/elementwise.hip. Binary
ops broadcast numpy-style; a broadcast (size-1) input dim is replicated along that axis and its
gradient is reduced back by the executor's edge transfer + local reduction.
"""
from __future__ import annotations

import torch

from .. import kernels as K
from ..type import DataType, OperatorType
from .base import OpImpl, register, torch_dtype

UNARY = {
    OperatorType.OP_RELU: "relu", OperatorType.OP_SIGMOID: "sigmoid", OperatorType.OP_TANH: "tanh",
    OperatorType.OP_ELU: "elu", OperatorType.OP_GELU: "gelu", OperatorType.OP_EXP: "exp",
    OperatorType.OP_SIN: "sin", OperatorType.OP_COS: "cos", OperatorType.OP_RSQRT: "rsqrt",
    OperatorType.OP_POW: "pow", OperatorType.OP_IDENTITY: "identity",
    OperatorType.OP_SCALAR_MULTIPLY: "scalar_multiply", OperatorType.OP_SCALAR_ADD: "scalar_add",
    OperatorType.OP_SCALAR_SUB: "scalar_sub", OperatorType.OP_SCALAR_TRUE_DIV: "scalar_true_divide",
    OperatorType.OP_SCALAR_FLOOR_DIV: "scalar_floor_divide", OperatorType.OP_LOG: "log",
    OperatorType.OP_SQRT: "sqrt", OperatorType.OP_LEAKYRELU: "leaky_relu",
}


# functions whose gradient can be computed from the output alone, so the output may overwrite the
# input (reference in-place optimisation, model.cc:2885-2919 / Op::can_inplace_output)
INPLACE_OK = {"relu", "sigmoid", "tanh", "exp", "scalar_multiply", "scalar_add", "scalar_sub",
              "scalar_true_divide"}


@register(*UNARY.keys())
class ElementUnary(OpImpl):
    def __init__(self, layer):
        super().__init__(layer)
        self.fn = UNARY[layer.op_type]
        self.op_type = layer.op_type

    @property
    def scalar(self):
        return float(self.attrs.get("scalar", 0.0))

    def forward(self, ctx, xs, ws):
        x = xs[0]
        if self.fn == "identity":
            return [x]
        if ctx.extra.get("fused_into_producer"):
            # the producing binary op already applied this ReLU (executor._plan_binary_relu); the
            # gradient needs the output only
            if ctx.training:
                ctx.saved["x"] = x
                ctx.saved["y"] = x
            return [x]
        if ctx.extra.get("inplace") and x.is_contiguous():
            y = K.unary_fwd(self.fn, x, self.scalar, out=x)
            if ctx.training:
                ctx.saved["x"] = y  # the input was overwritten; the gradient needs y only
                ctx.saved["y"] = y
            return [y]
        y = K.unary_fwd(self.fn, x, self.scalar)
        if ctx.training:
            ctx.saved["x"] = x
            ctx.saved["y"] = y
        return [y]

    def can_inplace(self):
        return self.fn in INPLACE_OK

    def saves_output(self):
        return True

    def backward(self, ctx, douts):
        dy = douts[0]
        if self.fn == "identity":
            return [dy]
        x, y = ctx.saved.pop("x"), ctx.saved.pop("y")
        return [K.unary_bwd(self.fn, x, y, dy, self.scalar)]


BINARY = {OperatorType.OP_EW_ADD: "add", OperatorType.OP_EW_SUB: "sub", OperatorType.OP_EW_MUL: "mul",
          OperatorType.OP_EW_DIV: "div", OperatorType.OP_EW_MAX: "max", OperatorType.OP_EW_MIN: "min"}


@register(*BINARY.keys())
class ElementBinary(OpImpl):
    def saves_output(self):
        return False  # backward reads inputs / its own saved buffers only

    def __init__(self, layer):
        super().__init__(layer)
        self.fn = BINARY[layer.op_type]
        self.op_type = layer.op_type

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        out = tuple(torch.broadcast_shapes(tuple(in_dims[0]), tuple(in_dims[1])))
        return [out], [in_dtypes[0]], []

    def input_maps(self):
        out = self.layer.outputs[0].dims
        n = len(out)
        maps = []
        for t in self.layer.inputs:
            m = []
            off = n - len(t.dims)
            for j, s in enumerate(t.dims):
                m.append(None if (s == 1 and out[off + j] != 1) else off + j)
            maps.append(tuple(m))
        return maps

    def forward(self, ctx, xs, ws):
        a, b = xs
        c = K.binary_fwd(self.fn, a, b, relu=bool(ctx.extra.get("fused_relu")))
        if ctx.training:
            ctx.saved["a"], ctx.saved["b"] = a, b
        return [c]

    def backward(self, ctx, douts):
        a, b = ctx.saved.pop("a"), ctx.saved.pop("b")
        dc = douts[0]
        if self.fn == "add" and tuple(a.shape) == tuple(b.shape) == tuple(dc.shape):
            return [dc, dc]
        da, db = K.binary_bwd(self.fn, a, b, dc)
        return [da, db]


@register(OperatorType.OP_DROPOUT)
class Dropout(OpImpl):
    op_type = OperatorType.OP_DROPOUT

    def forward(self, ctx, xs, ws):
        x = xs[0]
        rate = float(self.attrs.get("rate", 0.0))
        if not ctx.training or rate <= 0.0:
            return [x]
        seed = int(self.attrs.get("seed", 0)) + ctx.seed
        # per-step, per-part stream offset: deterministic and distinct across shards
        offset = (ctx.step * 1000003 + hash(ctx.part_coords) % 1000003) * x.numel()
        y, mask = K.dropout_fwd(x, rate, seed, offset)
        ctx.saved["mask"] = mask
        return [y]

    def backward(self, ctx, douts):
        rate = float(self.attrs.get("rate", 0.0))
        if rate <= 0.0 or "mask" not in ctx.saved:
            return [douts[0]]
        return [K.dropout_bwd(douts[0], ctx.saved.pop("mask"), rate)]


@register(OperatorType.OP_CAST)
class Cast(OpImpl):
    op_type = OperatorType.OP_CAST

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        return [in_dims[0]], [attrs["dtype"]], []

    def forward(self, ctx, xs, ws):
        dt = self.attrs["dtype"]
        x = xs[0]
        if dt in (DataType.DT_FLOAT, DataType.DT_HALF, DataType.DT_DOUBLE) and x.is_floating_point():
            return [x]  # float casts are absorbed by the compute dtype policy
        ctx.saved["dtype"] = x.dtype
        return [x.to(torch_dtype(dt))]

    def backward(self, ctx, douts):
        dt = ctx.saved.pop("dtype", None)
        if dt is None:
            return [douts[0]]
        if not dt.is_floating_point:
            return [None]
        return [douts[0].to(dt)]
