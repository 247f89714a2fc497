"""LayerNorm and BatchNorm.

LayerNorm normalises over the trailing `axes` (reference src/ops/layer_norm.cc; the reference HIP
build has its fast path disabled, layer_norm.cpp:46-52). Normalised dims cannot be partitioned;
every other dim can. Runs on csrc/kernels/norm.hip (one wave per row, row kept in VGPRs).

BatchNorm (NCHW, reference src/ops/batch_norm.cc) normalises per channel over N,H,W with
per-shard statistics when the batch is partitioned — the reference's cuDNN per-partition
semantics (csrc/kernels/cnn.hip).

RMSNorm (extension: the T5 / LLaMA "LayerNorm" without centering, which the HuggingFace import
path of the torch frontend meets) normalises the last dimension: y = x * rsqrt(mean(x^2) + eps) * w
(csrc/kernels/norm.hip).
"""
from __future__ import annotations

import math

import torch

from .. import kernels as K
from ..type import DataType, OperatorType
from .base import OpImpl, WeightSpec, register


@register(OperatorType.OP_LAYERNORM)
class LayerNorm(OpImpl):
    op_type = OperatorType.OP_LAYERNORM

    def saves_output(self):
        return False  # backward reads inputs / its own saved buffers only

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        d = in_dims[0]
        axes = sorted(a % len(d) for a in attrs["axes"])
        attrs["axes"] = axes
        ws = []
        if attrs.get("elementwise_affine", True):
            nd = tuple(d[a] for a in axes)
            from ..core.initializers import ConstantInitializer, ZeroInitializer
            ws = [WeightSpec("gamma", nd, in_dtypes[0], ConstantInitializer(1.0)),
                  WeightSpec("beta", nd, in_dtypes[0], ZeroInitializer())]
        return [d], [in_dtypes[0]], ws

    def axis_kinds(self):
        kinds = super().axis_kinds()
        for a in self.attrs["axes"]:
            kinds[a] = "none"
        return kinds

    def supports_axis(self, axis):
        return axis not in self.attrs["axes"]

    def weight_maps(self):
        return [tuple([None] * len(w.dims)) for w in self.layer.weights]

    def forward(self, ctx, xs, ws):
        # 2 inputs = residual-fused LayerNorm(x + res), produced by the fuse_add_layernorm
        # substitution: one kernel reads x and res and writes y (+ the sum kept for backward)
        x = xs[0]
        res = xs[1] if len(xs) > 1 else None
        nrm = int(math.prod(x.shape[a] for a in self.attrs["axes"]))
        assert self.attrs["axes"] == list(range(x.dim() - len(self.attrs["axes"]), x.dim())), \
            "LayerNorm axes must be trailing"
        x2 = x.reshape(-1, nrm)
        r2 = res.reshape(-1, nrm).contiguous() if res is not None else None
        g = ws[0].reshape(-1) if ws else None
        b = ws[1].reshape(-1) if ws else None
        y, xs_, mean, rstd = K.layernorm_fwd(x2.contiguous(), r2, g, b, float(self.attrs.get("eps", 1e-5)), False)
        if ctx.training:
            ctx.saved.update(x=xs_, mean=mean, rstd=rstd, g=g)
        return [y.reshape(x.shape)]

    def backward(self, ctx, douts):
        dy = douts[0]
        s = ctx.saved
        x2 = s.pop("x")
        dg = ctx.wgrads[0].reshape(-1) if ctx.wgrads else None
        db = ctx.wgrads[1].reshape(-1) if ctx.wgrads else None
        # fused bias gradient of the Linear that produced an input (executor pass fuse_bias_grads)
        dsum = ctx.extra.get("colsum_out")
        dx = K.layernorm_bwd(dy.reshape(x2.shape).contiguous(), x2, s.pop("g"), s.pop("mean"), s.pop("rstd"), dg, db,
                             dsum=dsum)
        dx = dx.reshape(dy.shape)
        return [dx, dx] if len(self.layer.inputs) > 1 else [dx]

    def flops(self, in_shapes, out_shapes, w_shapes):
        return 8.0 * math.prod(out_shapes[0])


@register(OperatorType.OP_BATCHNORM)
class BatchNorm(OpImpl):
    op_type = OperatorType.OP_BATCHNORM

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        d = in_dims[0]
        from ..core.initializers import ConstantInitializer, ZeroInitializer
        c = d[1]
        ws = [WeightSpec("scale", (c,), in_dtypes[0], ConstantInitializer(1.0)),
              WeightSpec("bias", (c,), in_dtypes[0], ZeroInitializer())]
        return [d], [in_dtypes[0]], ws

    def axis_kinds(self):
        # N (sample) and C (parameter) partitionable; spatial dims need cross-shard statistics
        return ["sample", "parameter"] + ["none"] * (len(self.layer.outputs[0].dims) - 2)

    def supports_axis(self, axis):
        return axis in (0, 1)

    def weight_maps(self):
        return [(1,), (1,)]

    def forward(self, ctx, xs, ws):
        """Batch statistics in training (running statistics updated, momentum 0.1), running
        statistics in inference; fused ReLU per the reference's batch_norm(relu=True) default.
        HIP kernels: csrc/kernels/cnn.hip (split Welford statistics + normalize pass)."""
        x = K.act_dense(xs[0])  # channel-last on the device (kernels.CHANNELS_LAST)
        c = x.shape[1]
        rm = ctx.extra.setdefault("running_mean", torch.zeros(c, device=x.device))
        rv = ctx.extra.setdefault("running_var", torch.ones(c, device=x.device))
        g, b = ws[0].reshape(-1), ws[1].reshape(-1)
        relu = bool(self.attrs.get("relu", True))
        y, mean, rstd = K.batchnorm_fwd(x, g, b, rm, rv, ctx.training, relu)
        if ctx.training:
            ctx.saved.update(x=x, g=g, b=b, mean=mean, rstd=rstd)
        return [y]

    def backward(self, ctx, douts):
        s = ctx.saved
        dg = ctx.wgrads[0].reshape(-1) if ctx.wgrads else None
        db = ctx.wgrads[1].reshape(-1) if ctx.wgrads and len(ctx.wgrads) > 1 else None
        dx = K.batchnorm_bwd(s.pop("x"), douts[0], s.pop("g"), s.pop("b"), s.pop("mean"), s.pop("rstd"), dg, db,
                             bool(self.attrs.get("relu", True)))
        return [dx]


@register(OperatorType.OP_RMS_NORM)
class RMSNorm(OpImpl):
    op_type = OperatorType.OP_RMS_NORM

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        d = in_dims[0]
        from ..core.initializers import ConstantInitializer
        return [d], [in_dtypes[0]], [WeightSpec("weight", (d[-1],), in_dtypes[0], ConstantInitializer(1.0))]

    def axis_kinds(self):
        kinds = super().axis_kinds()
        kinds[-1] = "none"
        return kinds

    def supports_axis(self, axis):
        return axis != len(self.layer.outputs[0].dims) - 1

    def weight_maps(self):
        return [(None,)]

    def forward(self, ctx, xs, ws):
        x = xs[0].contiguous()
        d = x.shape[-1]
        y, rstd = K.rmsnorm_fwd(x.reshape(-1, d), ws[0].reshape(-1), float(self.attrs.get("eps", 1e-6)))
        if ctx.training:
            ctx.saved.update(x=x, w=ws[0].reshape(-1), rstd=rstd)
        return [y.reshape(x.shape)]

    def backward(self, ctx, douts):
        s = ctx.saved
        x, w, rstd = s.pop("x"), s.pop("w"), s.pop("rstd")
        d = x.shape[-1]
        dw = ctx.wgrads[0].reshape(-1) if ctx.wgrads else None
        dx = K.rmsnorm_bwd(x.reshape(-1, d), w, douts[0].reshape(-1, d).contiguous(), rstd, dw)
        return [dx.reshape(x.shape)]

    def flops(self, in_shapes, out_shapes, w_shapes):
        return 5.0 * math.prod(out_shapes[0])
