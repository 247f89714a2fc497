"""Linear (dense) layer: y = act(x . W^T + b).

Parallel axes: every output dim (batch/sequence = sample/attribute parallelism, the last dim =
output channels = parameter parallelism) plus a reduction axis over input channels whose output
is a partial sum (reference Linear parallel-dim mappings, src/ops/linear.cc:1058-1072 and the
Reduction parallel op). Weight W is [out, in]; bias only on reduction coordinate 0 so the
reduced sum adds it once.

Kernels: bf16 MFMA GEMM with fused bias+activation epilogue (pre-activation saved for the
backward), split-K fp32 wgrad straight into the fp32 gradient arena, fused act'+bias-grad.
Reference: src/ops/linear.cc, src/ops/kernels/linear_kernels.cu.
"""
from __future__ import annotations

import math
import os

from .. import kernels as K
from ..type import ActiMode, DataType, OperatorType
from .base import OpImpl, WeightSpec, register


@register(OperatorType.OP_LINEAR)
class Linear(OpImpl):
    op_type = OperatorType.OP_LINEAR

    def saves_output(self):
        return False  # backward reads inputs / its own saved buffers only

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        d = in_dims[0]
        out = tuple(d[:-1]) + (attrs["out_dim"],)
        ws = [WeightSpec("kernel", (attrs["out_dim"], d[-1]), in_dtypes[0], attrs.get("kernel_init"))]
        if attrs.get("use_bias", True):
            ws.append(WeightSpec("bias", (attrs["out_dim"],), in_dtypes[0], attrs.get("bias_init")))
        return [out], [attrs.get("data_type") or in_dtypes[0]], ws

    def extra_axis_sizes(self):
        return [self.layer.inputs[0].dims[-1]]

    @property
    def red_axis(self):
        return len(self.layer.outputs[0].dims)

    def axis_kinds(self):
        n = len(self.layer.outputs[0].dims)
        return ["sample"] + ["attribute"] * (n - 2) + ["parameter", "parameter"]

    def supports_axis(self, axis):
        if axis == self.red_axis:
            return self.act == ActiMode.AC_MODE_NONE.value
        return True

    @property
    def act(self):
        return self.attrs.get("activation", ActiMode.AC_MODE_NONE).value

    def input_maps(self):
        n = len(self.layer.outputs[0].dims)
        return [tuple(range(n - 1)) + (self.red_axis,)]

    def weight_maps(self):
        n = len(self.layer.outputs[0].dims)
        maps = [(n - 1, self.red_axis)]
        if len(self.layer.weights) > 1:
            maps.append((n - 1,))
        return maps

    def forward(self, ctx, xs, ws):
        x = xs[0]
        w = ws[0]
        b = ws[1] if len(ws) > 1 else None
        if b is not None and ctx.degree(self.red_axis) > 1 and ctx.coord(self.red_axis) != 0:
            b = None
        Kl = x.shape[-1]
        x2 = x.reshape(-1, Kl)
        # FF_DACT_STORE_GRAD=1: when the consumer's dgrad applies this op's act' (Executor.
        # _plan_dact_fusion), the forward stores act'(z) instead of z and the backward only
        # multiplies by it. Off by default: the forward pass then writes y AND act'(z) (384 instead
        # of 256 MB per BERT-Large FFN1 call, bias_act_fwd 1.23 -> 1.61 ms per step) while the
        # backward pass moves the same bytes either way (its act' VALU hides under HBM time).
        sg = bool(ctx.training and ctx.extra.get("dact_fused") and self.act != K.ACT_NONE
                  and os.environ.get("FF_DACT_STORE_GRAD", "0") == "1")
        wt = None
        if ctx.training and ctx.extra.get("need_dx0", True):
            # the dgrad GEMM reads W^T K-contiguous (kernels.weight_t)
            wt = K.weight_t(ctx.extra.setdefault("wt_store", {}), w)
        y, z = K.linear_fwd(x2, w, b, self.act, save_z=ctx.training, store_grad=sg)
        if ctx.training:
            ctx.saved["wt"] = wt
            ctx.saved["x"] = x2
            ctx.saved["z"] = z
            ctx.saved["z_is_grad"] = sg
            ctx.saved["w"] = w
            ctx.saved["has_b"] = b is not None
        return [y.reshape(tuple(x.shape[:-1]) + (w.shape[0],))]

    def backward(self, ctx, douts):
        dy = douts[0]
        x2, z, w = ctx.saved["x"], ctx.saved["z"], ctx.saved["w"]
        dy2 = dy.reshape(-1, w.shape[0]).contiguous()
        dw = ctx.wgrads[0] if ctx.wgrads else None
        db = ctx.wgrads[1] if (len(ctx.wgrads) > 1 and ctx.saved["has_b"]) else None
        act = self.act
        if ctx.extra.get("bias_grad_fused"):  # the consuming LayerNorm's backward already summed it
            db = None
        if ctx.extra.get("dact_fused"):
            # the consuming Linear's dgrad GEMM already applied act' and summed the bias gradient
            act, z, db = K.ACT_NONE, None, None
        acc = (ctx.extra.get("dx_accum") or {}).get(0)
        dact = None
        src = ctx.extra.get("dact_src")  # (producer's ctx, its act) when this op's dgrad is fused
        if src is not None:
            # planned by Executor._plan_dact_fusion: sole consumer, so no accumulated dx exists
            assert ctx.extra.get("need_dx0", True) and acc is None, "dact fusion needs a fresh dx"
            pctx, pact = src
            pdb = None
            if len(pctx.wgrads) > 1 and pctx.saved.get("has_b") and not pctx.extra.get("bias_grad_fused"):
                pdb = pctx.wgrads[1]
            if pctx.saved.get("z_is_grad"):
                pact = K.ACT_GRADMUL
            dact = (pctx.saved["z"].reshape(-1, x2.shape[1]), pact, pdb)
        ready = ctx.extra.get("dx_ready")
        out_shape = tuple(dy.shape[:-1]) + (x2.shape[1],)
        on_dx = None
        if ready is not None:
            def on_dx(d):  # the executor starts dx's transfer before the wgrad GEMM
                ready(0, acc if acc is not None else d.reshape(out_shape))
        dx = K.linear_bwd(dy2, x2, w, z, act, dw, db, need_dx=ctx.extra.get("need_dx0", True),
                          dw_beta=0.0 if ctx.extra.get("wgrad_overwrite") else 1.0,
                          dx_out=acc.view(-1, x2.shape[1]) if acc is not None else None, dact=dact, on_dx=on_dx,
                          wt=ctx.saved.get("wt"))
        ctx.saved.clear()
        if dx is None:
            return [None]
        return [acc if acc is not None else dx.reshape(out_shape)]

    def accumulates_dx(self):
        return True

    def overwrites_wgrad(self, i):
        return i == 0  # dW GEMM with dw_beta = 0 under wgrad_overwrite; the bias gradient accumulates

    def flops(self, in_shapes, out_shapes, w_shapes):
        return 2.0 * math.prod(out_shapes[0]) * in_shapes[0][-1]

    def uses_mfma(self):
        return True
