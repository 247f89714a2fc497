"""Embedding lookup with optional bag aggregation (reference src/ops/embedding.cc, .cu).

Input: integer ids [..., bag] (AGGR_MODE_SUM/AVG reduce the trailing bag dim, as DLRM uses) or
[...] (AGGR_MODE_NONE appends the embedding dim). Weight [num_entries, out_dim].

Parallel axes: output dims (batch = sample parallelism, last = embedding columns) plus a *vocab*
axis: each part owns a contiguous row range of the table, looks up only the ids it owns and
emits a partial sum (the DLRM parameter-parallel embedding of the reference, without whole-table
placement restrictions). Kernels: csrc/kernels/embedding.hip (gather fwd, fp32 atomic bwd).
"""
from __future__ import annotations

import math

import torch

from .. import kernels as K
from ..type import AggrMode, DataType, OperatorType
from .base import OpImpl, WeightSpec, register


@register(OperatorType.OP_EMBEDDING)
class Embedding(OpImpl):
    op_type = OperatorType.OP_EMBEDDING

    def saves_output(self):
        return False  # backward reads inputs / its own saved buffers only

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        d = in_dims[0]
        aggr = attrs.get("aggr", AggrMode.AGGR_MODE_NONE)
        if aggr == AggrMode.AGGR_MODE_NONE:
            out = tuple(d) + (attrs["out_dim"],)
        else:
            out = tuple(d[:-1]) + (attrs["out_dim"],)
        dt = attrs.get("data_type") or DataType.DT_FLOAT
        ws = [WeightSpec("weight", (attrs["num_entries"], attrs["out_dim"]), dt, attrs.get("kernel_init"))]
        return [out], [dt], ws

    @property
    def bag(self):
        aggr = self.attrs.get("aggr", AggrMode.AGGR_MODE_NONE)
        return 1 if aggr == AggrMode.AGGR_MODE_NONE else self.layer.inputs[0].dims[-1]

    @property
    def vocab_axis(self):
        return len(self.layer.outputs[0].dims)

    def extra_axis_sizes(self):
        return [self.attrs["num_entries"]]

    def axis_kinds(self):
        n = len(self.layer.outputs[0].dims)
        return ["sample"] + ["attribute"] * (n - 2) + ["parameter", "parameter"]

    def input_maps(self):
        n = len(self.layer.outputs[0].dims)
        aggr = self.attrs.get("aggr", AggrMode.AGGR_MODE_NONE)
        ni = len(self.layer.inputs[0].dims)
        if aggr == AggrMode.AGGR_MODE_NONE:
            return [tuple(range(ni))]
        return [tuple(range(ni - 1)) + (None,)]

    def weight_maps(self):
        n = len(self.layer.outputs[0].dims)
        return [(self.vocab_axis, n - 1)]

    def forward(self, ctx, xs, ws):
        idx = xs[0]
        table = ws[0]
        bag = self.bag
        avg = self.attrs.get("aggr") == AggrMode.AGGR_MODE_AVG
        vdeg = ctx.degree(self.vocab_axis)
        if vdeg > 1:
            lo = ctx.coord(self.vocab_axis) * table.shape[0]
            idx = idx.to(torch.int64) - lo  # out-of-range ids are skipped by the kernel (contribute 0)
        out = K.embedding_fwd(idx, table, bag, avg)
        if ctx.training:
            ctx.saved["idx"] = idx
        lead = idx.shape if bag == 1 and self.attrs.get("aggr", AggrMode.AGGR_MODE_NONE) == AggrMode.AGGR_MODE_NONE \
            else idx.shape[:-1]
        return [out.reshape(tuple(lead) + (table.shape[1],))]

    def backward(self, ctx, douts):
        idx = ctx.saved.pop("idx")
        ctx.extra["touched_idx"] = idx  # rows this step touched (Executor row-sparse SGD update)
        if ctx.wgrads and ctx.wgrads[0] is not None:
            dim = ctx.wgrads[0].shape[1]
            K.embedding_bwd(idx, douts[0].reshape(-1, dim), ctx.wgrads[0], self.bag,
                            self.attrs.get("aggr") == AggrMode.AGGR_MODE_AVG)
        return [None]

    def needs_input_grad(self, i):
        return False

    def flops(self, in_shapes, out_shapes, w_shapes):
        return float(math.prod(out_shapes[0]) * self.bag)

    def mem_bytes(self, in_shapes, out_shapes, w_shapes, elem=2):
        return float(elem * math.prod(out_shapes[0]) * (self.bag + 1))
