"""Softmax over one dim (reference src/ops/softmax.cc, kernels/softmax.cu).

When the softmax output feeds a cross-entropy loss the loss already produced the gradient w.r.t.
the softmax *input* ((p - y)/batch, reference loss_functions.cu), so backward is a pass-through in
that case (`ctx.extra['loss_fused']`), exactly as the reference's Softmax::backward copies.
"""
from __future__ import annotations

import math

from .. import kernels as K
from ..type import OperatorType
from .base import OpImpl, register


@register(OperatorType.OP_SOFTMAX)
class Softmax(OpImpl):
    op_type = OperatorType.OP_SOFTMAX

    @property
    def dim(self):
        d = self.attrs.get("dim", -1)
        return d % len(self.layer.outputs[0].dims)

    def axis_kinds(self):
        k = super().axis_kinds()
        k[self.dim] = "none"
        return k

    def supports_axis(self, axis):
        return axis != self.dim

    def forward(self, ctx, xs, ws):
        x = xs[0]
        if ctx.training and ctx.extra.get("loss_fused") and self.dim == x.dim() - 1:
            # The loss consumes the LOGITS (fused softmax + cross-entropy kernel), so the
            # [tokens x classes] probability tensor is never written; probabilities are produced
            # on demand if the user reads this tensor (executor.get_value).
            ctx.extra["emitted_logits"] = True
            return [x]
        ctx.extra["emitted_logits"] = False
        xm = x.movedim(self.dim, -1) if self.dim != x.dim() - 1 else x
        shp = xm.shape
        y = K.softmax_fwd(xm.reshape(-1, shp[-1]).contiguous()).reshape(shp)
        if self.dim != x.dim() - 1:
            y = y.movedim(-1, self.dim).contiguous()
        if ctx.training:
            ctx.saved["y"] = y
        return [y]

    def backward(self, ctx, douts):
        dy = douts[0]
        if ctx.extra.get("loss_fused"):
            ctx.saved.pop("y", None)
            return [dy]
        y = ctx.saved.pop("y")
        if self.dim != y.dim() - 1:
            ym, dym = y.movedim(self.dim, -1), dy.movedim(self.dim, -1)
            shp = ym.shape
            dx = K.softmax_bwd(ym.reshape(-1, shp[-1]).contiguous(), dym.reshape(-1, shp[-1]).contiguous())
            return [dx.reshape(shp).movedim(-1, self.dim).contiguous()]
        shp = y.shape
        return [K.softmax_bwd(y.reshape(-1, shp[-1]), dy.reshape(-1, shp[-1]).contiguous()).reshape(shp)]

    def flops(self, in_shapes, out_shapes, w_shapes):
        return 5.0 * math.prod(out_shapes[0])
