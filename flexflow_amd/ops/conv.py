"""Conv2D and Pool2D (NCHW logical shapes; channel-last memory on the device, kernels.CHANNELS_LAST),
reference src/ops/conv_2d.cc, src/ops/pool_2d.cc (cuDNN).

Parallel axes: N (sample), C_out (parameter; conv only), H and W (attribute parallelism: each part
computes an output row/col block and reads its input block plus a halo of the receptive field,
provided by the edge transfer), and for conv a C_in reduction axis with partial-sum outputs.
Attribute parallelism requires stride-aligned blocks (checked in supports_axis).

Math: Conv2D runs our implicit-GEMM MFMA kernels (csrc/kernels/conv.hip) or MIOpen, timed per
geometry (kernels.conv2d_fwd / conv2d_bwd); Pool2D runs csrc/kernels/cnn.hip. Groups, no dilation
(as the reference).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .. import kernels as K
from ..type import ActiMode, OperatorType, PoolType
from .base import OpImpl, WeightSpec, register


def _out_size(i, k, s, p):
    return (i + 2 * p - k) // s + 1


class _Spatial(OpImpl):
    def _kp(self):
        a = self.attrs
        return a["kernel_h"], a["kernel_w"], a["stride_h"], a["stride_w"], a["padding_h"], a["padding_w"]

    def input_halo(self, idx, degrees):
        if idx != 0:
            return None
        kh, kw, sh, sw, ph, pw = self._kp()
        return (0, 0, kh if degrees[2] > 1 else 0, kw if degrees[3] > 1 else 0)

    def _spatial_ok(self, axis):
        kh, kw, sh, sw, ph, pw = self._kp()
        ih, iw = self.layer.inputs[0].dims[2:4]
        oh, ow = self.layer.outputs[0].dims[2:4]
        # block-aligned tiling: output block [a, b) reads input block [a*s, b*s) plus a halo of at
        # most k rows on each side (the input layout's halo)
        if axis == 2:
            return ih == oh * sh and ph < kh
        if axis == 3:
            return iw == ow * sw and pw < kw
        return True

    def _local_input(self, ctx, x, axis_base=2):
        """Crop the halo'd input block to exactly what this output block needs (+ zero pad at edges)."""
        kh, kw, sh, sw, ph, pw = self._kp()
        pads = [pw, pw, ph, ph]
        if ctx.degree(2) == 1 and ctx.degree(3) == 1:
            return x, (ph, pw)
        ih, iw = self.layer.inputs[0].dims[2:4]
        # region bookkeeping supplied by the executor
        reg = ctx.extra["in_region0"]
        out_reg = ctx.extra["out_region"]
        res = []
        for d, (k, s, p, full) in zip((2, 3), ((kh, sh, ph, ih), (kw, sw, pw, iw))):
            olo, ohi = out_reg[d]
            need_lo, need_hi = olo * s - p, (ohi - 1) * s - p + k
            have_lo, have_hi = reg[d]
            lo_pad = max(0, have_lo - need_lo) if need_lo < 0 else 0
            hi_pad = max(0, need_hi - have_hi) if need_hi > full else 0
            a = max(need_lo, have_lo) - have_lo
            b = min(need_hi, have_hi) - have_lo
            res.append((a, b, lo_pad, hi_pad))
        (a2, b2, lp2, hp2), (a3, b3, lp3, hp3) = res
        xc = x[:, :, a2:b2, a3:b3]
        xc = F.pad(xc, (lp3, hp3, lp2, hp2))
        return xc, (0, 0)

    def _local_block(self, ctx, x):
        """Like _local_input, but the block is cropped only and its edge padding returned as
        (top, bottom, left, right) for kernels that pad implicitly (max pooling pads with -inf,
        average pooling must not count padding it does not include). Also returns the crop
        window (a2, b2, a3, b3) in the halo'd block for the backward's scatter."""
        kh, kw, sh, sw, ph, pw = self._kp()
        if ctx.degree(2) == 1 and ctx.degree(3) == 1:
            return x, (ph, ph, pw, pw), None
        ih, iw = self.layer.inputs[0].dims[2:4]
        reg = ctx.extra["in_region0"]
        out_reg = ctx.extra["out_region"]
        res = []
        for d, (k, s, p, full) in zip((2, 3), ((kh, sh, ph, ih), (kw, sw, pw, iw))):
            olo, ohi = out_reg[d]
            need_lo, need_hi = olo * s - p, (ohi - 1) * s - p + k
            have_lo, have_hi = reg[d]
            lo_pad = max(0, have_lo - need_lo) if need_lo < 0 else 0
            hi_pad = max(0, need_hi - have_hi) if need_hi > full else 0
            a = max(need_lo, have_lo) - have_lo
            b = min(need_hi, have_hi) - have_lo
            res.append((a, b, lo_pad, hi_pad))
        (a2, b2, lp2, hp2), (a3, b3, lp3, hp3) = res
        return x[:, :, a2:b2, a3:b3], (lp2, hp2, lp3, hp3), (a2, b2, a3, b3)


@register(OperatorType.OP_CONV2D)
class Conv2D(_Spatial):
    op_type = OperatorType.OP_CONV2D

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        n, c, h, w = in_dims[0]
        oh = _out_size(h, attrs["kernel_h"], attrs["stride_h"], attrs["padding_h"])
        ow = _out_size(w, attrs["kernel_w"], attrs["stride_w"], attrs["padding_w"])
        g = attrs.get("groups", 1)
        ws = [WeightSpec("kernel", (attrs["out_channels"], c // g, attrs["kernel_h"], attrs["kernel_w"]),
                         in_dtypes[0], attrs.get("kernel_init"))]
        if attrs.get("use_bias", True):
            ws.append(WeightSpec("bias", (attrs["out_channels"],), in_dtypes[0], attrs.get("bias_init")))
        return [(n, attrs["out_channels"], oh, ow)], [in_dtypes[0]], ws

    def extra_axis_sizes(self):
        return [self.layer.inputs[0].dims[1]]

    def axis_kinds(self):
        return ["sample", "parameter", "attribute", "attribute", "parameter"]

    def supports_axis(self, axis):
        if self.attrs.get("groups", 1) != 1 and axis in (1, 4):
            return False
        if axis == 4:
            return self.attrs.get("activation", ActiMode.AC_MODE_NONE) == ActiMode.AC_MODE_NONE
        return self._spatial_ok(axis)

    def input_maps(self):
        return [(0, 4, 2, 3)]

    def weight_maps(self):
        m = [(1, 4, None, None)]
        if len(self.layer.weights) > 1:
            m.append((1,))
        return m

    def forward(self, ctx, xs, ws):
        """Implicit-GEMM MFMA convolution (csrc/kernels/conv.hip) with bias and ReLU fused into its
        store, or MIOpen where the per-geometry timing found it faster (kernels.conv2d_fwd).
        Activations other than ReLU are applied after the convolution."""
        x = xs[0]
        w = ws[0]
        b = ws[1] if len(ws) > 1 else None
        if b is not None and ctx.degree(4) > 1 and ctx.coord(4) != 0:
            b = None
        kh, kw, sh, sw, ph, pw = self._kp()
        xc, pad = self._local_input(ctx, x)
        groups = self.attrs.get("groups", 1)
        xc = K.cl_dense(xc, K.cl_ok(xc, xc.shape[1] // groups))  # the layout the kernels take (saved as such)
        act = self.attrs.get("activation", ActiMode.AC_MODE_NONE)
        relu = act == ActiMode.AC_MODE_RELU
        pk = {} if ctx.training else None
        z = K.conv2d_fwd(xc, w, b, (sh, sw), pad, groups, relu, bwd_pack=pk)
        y = z if act in (ActiMode.AC_MODE_NONE, ActiMode.AC_MODE_RELU) else K.act_ref(z, act.value)
        if ctx.training:
            ctx.saved.update(xc=xc, w=w, z=z, y=y, pad=pad, x_shape=x.shape, has_b=b is not None, wpack=pk.get("w"))
        return [y]

    def backward(self, ctx, douts):
        s = ctx.saved
        xc, w, z, y, pad, x_shape, has_b, wpack = (s.pop(k) for k in ("xc", "w", "z", "y", "pad", "x_shape", "has_b",
                                                                        "wpack"))
        act = self.attrs.get("activation", ActiMode.AC_MODE_NONE)
        dy = douts[0].to(y.dtype)
        db = ctx.wgrads[1] if (has_b and len(ctx.wgrads) > 1) else None
        if ctx.extra.get("dact_fused"):
            # the consuming convolution's dgrad already applied this op's ReLU and summed its bias
            # gradient (Executor._plan_dact_fusion): dy is the pre-activation gradient
            dz = dy
        else:
            if act not in (ActiMode.AC_MODE_NONE, ActiMode.AC_MODE_RELU):
                dy = (dy.float() * K.act_grad_ref(z.float(), act.value)).to(y.dtype)
            dz = K.conv_bias_relu_bwd(dy, y if act == ActiMode.AC_MODE_RELU else None, db)
        kh, kw, sh, sw, ph, pw = self._kp()
        g = K.conv_geometry(xc, w, (sh, sw), pad, self.attrs.get("groups", 1))
        dw = ctx.wgrads[0] if ctx.wgrads else None
        acc = (ctx.extra.get("dx_accum") or {}).get(0)
        if acc is not None and tuple(xc.shape) != tuple(x_shape):
            acc = None  # attribute-parallel crop: dx is scattered into a fresh block below
        dact = None
        src = ctx.extra.get("dact_src")  # (producer's ctx,): this op's dgrad applies its ReLU
        if src is not None:
            pctx = src[0]
            pdb = pctx.wgrads[1] if (pctx.saved.get("has_b") and len(pctx.wgrads) > 1) else None
            assert acc is None and tuple(xc.shape) == tuple(x_shape), "conv dact fusion needs a fresh, uncropped dx"
            dact = (pctx.saved["y"], pdb)
        dx = K.conv2d_bwd(xc, w, dz, g, dw, ctx.extra.get("need_dx0", True), dx_acc=acc, wpack=wpack, dact=dact)
        if dx is None:  # the input needs no gradient (the data, or a frozen producer)
            return [None]
        if tuple(dx.shape) != tuple(x_shape):  # attribute-parallel: scatter crop back into halo'd block
            full = torch.zeros(x_shape, dtype=dx.dtype, device=dx.device)
            full = self._uncrop(ctx, full, dx)
            dx = full
        return [dx]

    def _uncrop(self, ctx, full, dxc):
        kh, kw, sh, sw, ph, pw = self._kp()
        ih, iw = self.layer.inputs[0].dims[2:4]
        reg = ctx.extra["in_region0"]
        out_reg = ctx.extra["out_region"]
        sl = []
        for d, (k, s_, p, fullsz) in zip((2, 3), ((kh, sh, ph, ih), (kw, sw, pw, iw))):
            olo, ohi = out_reg[d]
            need_lo, need_hi = olo * s_ - p, (ohi - 1) * s_ - p + k
            have_lo, have_hi = reg[d]
            a = max(need_lo, have_lo) - have_lo
            b = min(need_hi, have_hi) - have_lo
            lo_pad = (have_lo - need_lo) if need_lo < have_lo else 0
            sl.append((a, b, lo_pad))
        (a2, b2, l2), (a3, b3, l3) = sl
        full[:, :, a2:b2, a3:b3] += dxc[:, :, l2:l2 + (b2 - a2), l3:l3 + (b3 - a3)]
        return full

    def accumulates_dx(self):
        return True  # the dgrad kernel adds into an existing input gradient (kernels.conv2d_bwd)

    def accum_target_ok(self, t):
        return t.is_contiguous() or K.is_nhwc(t)

    def flops(self, in_shapes, out_shapes, w_shapes):
        w = w_shapes[0]
        return 2.0 * math.prod(out_shapes[0]) * w[1] * w[2] * w[3]

    def uses_mfma(self):
        return True


@register(OperatorType.OP_POOL2D)
class Pool2D(_Spatial):
    op_type = OperatorType.OP_POOL2D

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        n, c, h, w = in_dims[0]
        oh = _out_size(h, attrs["kernel_h"], attrs["stride_h"], attrs["padding_h"])
        ow = _out_size(w, attrs["kernel_w"], attrs["stride_w"], attrs["padding_w"])
        return [(n, c, oh, ow)], [in_dtypes[0]], []

    def axis_kinds(self):
        return ["sample", "attribute", "attribute", "attribute"]

    def supports_axis(self, axis):
        return self._spatial_ok(axis)

    def _fused(self):
        act = self.attrs.get("activation", ActiMode.AC_MODE_NONE)
        return act in (ActiMode.AC_MODE_NONE, ActiMode.AC_MODE_RELU), act == ActiMode.AC_MODE_RELU

    def forward(self, ctx, xs, ws):
        """HIP pooling (csrc/kernels/cnn.hip) with the ReLU the reference allows fused; other
        activations run through torch (not used by the reference's models)."""
        x = xs[0]
        kh, kw, sh, sw, ph, pw = self._kp()
        is_max = self.attrs.get("pool_type", PoolType.POOL_MAX) == PoolType.POOL_MAX
        include_pad = bool(self.attrs.get("count_include_pad", True))
        fused, relu = self._fused()
        if not fused:
            return self._forward_torch(ctx, x)
        xc, pads, crop = self._local_block(ctx, x)
        xc = K.act_dense(xc)
        y, idx = K.pool2d_fwd(xc, kh, kw, sh, sw, pads, is_max, include_pad, relu, ctx.training)
        if ctx.training:
            ctx.saved.update(xc=xc, y=y, idx=idx, pads=pads, crop=crop, x_shape=x.shape)
        return [y]

    def backward(self, ctx, douts):
        s = ctx.saved
        if "xr" in s:
            return self._backward_torch(ctx, douts)
        kh, kw, sh, sw, ph, pw = self._kp()
        is_max = self.attrs.get("pool_type", PoolType.POOL_MAX) == PoolType.POOL_MAX
        _, relu = self._fused()
        xc, y, idx, pads, crop, x_shape = (s.pop(k) for k in ("xc", "y", "idx", "pads", "crop", "x_shape"))
        dx = K.pool2d_bwd(xc, y, douts[0].to(xc.dtype), idx, kh, kw, sh, sw, pads, is_max,
                          bool(self.attrs.get("count_include_pad", True)), relu)
        if crop is not None:  # attribute-parallel: scatter the block back into the halo'd input
            a2, b2, a3, b3 = crop
            full = torch.zeros(x_shape, dtype=dx.dtype, device=dx.device)
            full[:, :, a2:b2, a3:b3] = dx
            dx = full
        return [dx]

    def _forward_torch(self, ctx, x):
        kh, kw, sh, sw, ph, pw = self._kp()
        xc, pad = self._local_input(ctx, x)
        xr = xc.detach().requires_grad_(ctx.training)
        act = self.attrs.get("activation", ActiMode.AC_MODE_NONE).value
        with torch.enable_grad() if ctx.training else torch.no_grad():
            if self.attrs.get("pool_type", PoolType.POOL_MAX) == PoolType.POOL_MAX:
                xp = F.pad(xr, (pad[1], pad[1], pad[0], pad[0]), value=float("-inf")) if any(pad) else xr
                y = F.max_pool2d(xp, (kh, kw), (sh, sw))
            else:
                y = F.avg_pool2d(xr, (kh, kw), (sh, sw), pad,
                                 count_include_pad=self.attrs.get("count_include_pad", True))
            y = K.act_ref(y, act)
        if ctx.training:
            ctx.saved.update(xr=xr, y=y, x_shape=x.shape)
        return [y.detach()]

    def _backward_torch(self, ctx, douts):
        s = ctx.saved
        xr, y, x_shape = s.pop("xr"), s.pop("y"), s.pop("x_shape")
        (dx,) = torch.autograd.grad(y, (xr,), douts[0].to(y.dtype))
        if tuple(dx.shape) != tuple(x_shape):
            full = torch.zeros(x_shape, dtype=dx.dtype, device=dx.device)
            dx = Conv2D._uncrop(self, ctx, full, dx)
        return [dx]

    def flops(self, in_shapes, out_shapes, w_shapes):
        return float(math.prod(out_shapes[0]) * self.attrs["kernel_h"] * self.attrs["kernel_w"])
