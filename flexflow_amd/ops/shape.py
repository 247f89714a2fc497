"""Shape / data-movement ops: input, noop, flat, reshape, transpose, concat, split, reverse, gather.

Reference: src/ops/{noop,flat,reshape,transpose,concat,split,reverse,gather}.cc. These are
layout-only on the local shard; which dims may be partitioned follows from which dims survive the
op unchanged (e.g. Reshape/Flat keep the batch dim, Concat/Split/Reverse/Softmax-like ops keep
every dim except the one they act on).
"""
from __future__ import annotations

import math
import os

import torch

from .. import kernels as K
from ..parallel import boxcopy
from ..type import DataType, OperatorType
from .base import OpImpl, register

_CHECK_INDICES = os.environ.get("FF_CHECK_INDICES", "0") == "1"


@register(OperatorType.OP_INPUT)
class Input(OpImpl):
    op_type = OperatorType.OP_INPUT

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        return [tuple(attrs["dims"])], [attrs["data_type"]], []

    def forward(self, ctx, xs, ws):  # value injected by the executor
        raise RuntimeError("input op is fed by the executor")

    def backward(self, ctx, douts):
        return []


@register(OperatorType.OP_NOOP)
class NoOp(OpImpl):
    op_type = OperatorType.OP_NOOP

    def forward(self, ctx, xs, ws):
        return [xs[0]]

    def backward(self, ctx, douts):
        return [douts[0]]

    def flops(self, *a):
        return 0.0


def _batch_only_kinds(n):
    return ["sample"] + ["none"] * (n - 1)


@register(OperatorType.OP_FLAT)
class Flat(OpImpl):
    op_type = OperatorType.OP_FLAT

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        d = in_dims[0]
        return [(d[0], int(math.prod(d[1:])))], [in_dtypes[0]], []

    def axis_kinds(self):
        return _batch_only_kinds(2)

    def supports_axis(self, axis):
        return axis == 0

    def input_maps(self):
        return [(0,) + (None,) * (len(self.layer.inputs[0].dims) - 1)]

    def forward(self, ctx, xs, ws):
        x = xs[0]
        ctx.saved["shape"] = x.shape
        return [x.reshape(x.shape[0], -1)]

    def backward(self, ctx, douts):
        return [douts[0].reshape(ctx.saved.pop("shape"))]

    def flops(self, *a):
        return 0.0


@register(OperatorType.OP_RESHAPE)
class Reshape(OpImpl):
    op_type = OperatorType.OP_RESHAPE

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        shape = list(attrs["shape"])
        n = math.prod(in_dims[0])
        if -1 in shape:
            i = shape.index(-1)
            shape[i] = n // -math.prod(shape)
        assert math.prod(shape) == n, (shape, in_dims[0])
        attrs["shape"] = tuple(shape)
        return [tuple(shape)], [in_dtypes[0]], []

    def _keeps_batch(self):
        i, o = self.layer.inputs[0].dims, self.layer.outputs[0].dims
        return i[0] == o[0]

    def axis_kinds(self):
        k = _batch_only_kinds(len(self.layer.outputs[0].dims))
        if not self._keeps_batch():
            k[0] = "none"
        return k

    def supports_axis(self, axis):
        return axis == 0 and self._keeps_batch()

    def input_maps(self):
        return [(0,) + (None,) * (len(self.layer.inputs[0].dims) - 1)]

    def forward(self, ctx, xs, ws):
        x = xs[0]
        ctx.saved["shape"] = x.shape
        shp = list(self.attrs["shape"])
        shp[0] = x.shape[0] if self._keeps_batch() else shp[0]
        return [x.reshape(shp)]

    def backward(self, ctx, douts):
        return [douts[0].reshape(ctx.saved.pop("shape"))]

    def flops(self, *a):
        return 0.0


@register(OperatorType.OP_TRANSPOSE)
class Transpose(OpImpl):
    op_type = OperatorType.OP_TRANSPOSE

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        perm = tuple(attrs["perm"])
        return [tuple(in_dims[0][p] for p in perm)], [in_dtypes[0]], []

    def input_maps(self):
        perm = self.attrs["perm"]
        inv = [0] * len(perm)
        for o, i in enumerate(perm):
            inv[i] = o
        return [tuple(inv)]

    def forward(self, ctx, xs, ws):
        return [xs[0].permute(*self.attrs["perm"]).contiguous()]

    def backward(self, ctx, douts):
        perm = self.attrs["perm"]
        inv = [0] * len(perm)
        for o, i in enumerate(perm):
            inv[i] = o
        return [douts[0].permute(*inv).contiguous()]


@register(OperatorType.OP_CONCAT)
class Concat(OpImpl):
    op_type = OperatorType.OP_CONCAT

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        ax = attrs["axis"] % len(in_dims[0])
        attrs["axis"] = ax
        out = list(in_dims[0])
        out[ax] = sum(d[ax] for d in in_dims)
        return [tuple(out)], [in_dtypes[0]], []

    def axis_kinds(self):
        k = super().axis_kinds()
        k[self.attrs["axis"]] = "none"
        return k

    def supports_axis(self, axis):
        return axis != self.attrs["axis"]

    def input_maps(self):
        n = len(self.layer.outputs[0].dims)
        return [tuple(range(n)) for _ in self.layer.inputs]

    def forward(self, ctx, xs, ws):
        ax = self.attrs["axis"]
        ctx.saved["sizes"] = [x.shape[ax] for x in xs]
        if len(xs) > 1 and xs[0].is_cuda and os.environ.get("FF_CAT_KERNEL", "1") == "1":
            out = _concat_rows(list(xs), ax)
            if out is not None:
                return [out]
        # FF_BOX_CONCAT=1: the generic box-kernel concat (measured 12.5 -> 12.9 ms per Inception-v3
        # b64 step, profiles/concat_box_ab_r5.txt)
        if len(xs) > 1 and _box_ok(xs[0]) and os.environ.get("FF_BOX_CONCAT", "0") == "1" \
                and all(x.dtype == xs[0].dtype for x in xs):
            out = boxcopy.concat(self.__dict__.setdefault("_box_plans", {}), list(xs), ax)
            if out is not None:
                return [out]
        return [torch.cat(xs, ax)]

    def backward(self, ctx, douts):
        sizes = ctx.saved.pop("sizes")
        dy = douts[0]
        if len(sizes) > 1 and _box_ok(dy) and os.environ.get("FF_BOX_SPLIT", "1") == "1":
            return _split_dense(self, dy, sizes, self.attrs["axis"])
        return list(torch.split(dy, sizes, self.attrs["axis"]))


def _concat_rows(xs, ax):
    """torch.cat(xs, ax) by transfer.hip's concat_rows kernel (one launch, up to 16 inputs): dense
    inputs of one dtype, either all contiguous (rows = the dims before ax) or all channel-last 4-D
    concatenated along C (rows = N*H*W pixels). None when that does not apply (the caller falls
    back). Reference: src/ops/kernels/concat_kernels.cu (one copy per input)."""
    if len(xs) > 16 or any(x.dtype != xs[0].dtype or x.dim() != xs[0].dim() for x in xs):
        return None
    n = xs[0].dim()
    shp = list(xs[0].shape)
    shp[ax] = sum(x.shape[ax] for x in xs)
    if all(x.is_contiguous() for x in xs):
        outer = math.prod(shp[:ax])
        lens = [x.shape[ax] * math.prod(x.shape[ax + 1:]) for x in xs]
        out = torch.empty(shp, dtype=xs[0].dtype, device=xs[0].device)
    elif n == 4 and ax == 1 and all(K.is_nhwc(x) for x in xs):
        outer = shp[0] * shp[2] * shp[3]
        lens = [x.shape[1] for x in xs]
        # (allocated channel-last directly: empty(...).contiguous(channels_last) is a full copy)
        out = torch.empty(shp, dtype=xs[0].dtype, device=xs[0].device, memory_format=torch.channels_last)
    else:
        return None
    if outer == 0 or min(lens) == 0:
        return None
    es = xs[0].element_size()
    for vb in (16, 8, 4, 2):
        if vb % es == 0 and all((l * es) % vb == 0 for l in lens) and \
                all(t.data_ptr() % vb == 0 for t in list(xs) + [out]):
            break
    else:
        return None
    if outer * max(lens) * es // vb + 8192 * 256 >= (1 << 31):
        return None
    K.ext().concat_rows(list(xs), [l * es // vb for l in lens], out, outer, vb)
    return out


def _split_dense(op, dy, sizes, ax):
    """torch.split of a concat's gradient into DENSE parts (each in dy's memory format, side by
    side in one buffer) by one box-copy launch (csrc/kernels/transfer.hip). The views torch.split
    returns are strided along the split dim (a channel slice of an NHWC gradient), and every
    consumer made its own ATen copy of one: Inception-v3 paid ~23 copy launches per backward
    (reference concat_kernels.cu backward: one copy per input as well)."""
    outs = boxcopy.split_dense(op.__dict__.setdefault("_box_plans", {}), dy, sizes, ax)
    return outs if outs is not None else list(torch.split(dy, sizes, ax))


def _box_ok(t) -> bool:
    return boxcopy.available(t) and os.environ.get("FF_BOX_SHAPE", "1") == "1"


@register(OperatorType.OP_SPLIT)
class Split(OpImpl):
    op_type = OperatorType.OP_SPLIT

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        d = in_dims[0]
        ax = attrs["axis"] % len(d)
        attrs["axis"] = ax
        sizes = attrs["sizes"]
        if isinstance(sizes, int):
            assert d[ax] % sizes == 0
            sizes = [d[ax] // sizes] * sizes
        attrs["sizes"] = list(sizes)
        outs = []
        for s in sizes:
            o = list(d)
            o[ax] = s
            outs.append(tuple(o))
        return outs, [in_dtypes[0]] * len(outs), []

    def axis_kinds(self):
        k = super().axis_kinds()
        k[self.attrs["axis"]] = "none"
        return k

    def supports_axis(self, axis):
        return axis != self.attrs["axis"]

    def output_maps(self):
        n = len(self.layer.outputs[0].dims)
        return [tuple(range(n)) for _ in self.layer.outputs]

    def forward(self, ctx, xs, ws):
        if len(self.attrs["sizes"]) > 1 and _box_ok(xs[0]):
            outs = boxcopy.split_dense(self.__dict__.setdefault("_box_plans", {}), xs[0], self.attrs["sizes"],
                                       self.attrs["axis"])
            if outs is not None:
                return outs
        return [K.dense(t) for t in torch.split(xs[0], self.attrs["sizes"], self.attrs["axis"])]

    def backward(self, ctx, douts):
        like = [d for d in douts if d is not None][0]
        parts = []
        for d, s in zip(douts, self.attrs["sizes"]):
            if d is None:
                shp = list(like.shape)
                shp[self.attrs["axis"]] = s
                d = torch.zeros(shp, dtype=like.dtype, device=like.device)
            parts.append(d)
        if len(parts) > 1 and _box_ok(parts[0]) and all(p.dtype == parts[0].dtype for p in parts):
            out = boxcopy.concat(self.__dict__.setdefault("_box_plans", {}), parts, self.attrs["axis"])
            if out is not None:
                return [out]
        return [torch.cat(parts, self.attrs["axis"])]


@register(OperatorType.OP_REVERSE)
class Reverse(OpImpl):
    op_type = OperatorType.OP_REVERSE

    def axis_kinds(self):
        k = super().axis_kinds()
        k[self.attrs["axis"] % len(k)] = "none"
        return k

    def supports_axis(self, axis):
        return axis != self.attrs["axis"] % len(self.layer.outputs[0].dims)

    def _flip(self, t):
        ax = self.attrs["axis"] % t.dim()
        if _box_ok(t):  # one box-copy launch walking the source backwards along the axis
            return boxcopy.reverse(self.__dict__.setdefault("_box_plans", {}), t, ax)
        return torch.flip(t, [ax])

    def forward(self, ctx, xs, ws):
        return [self._flip(xs[0])]

    def backward(self, ctx, douts):
        return [self._flip(douts[0])]


@register(OperatorType.OP_GATHER)
class Gather(OpImpl):
    """torch.gather semantics along `dim` (reference src/ops/gather.cc)."""
    op_type = OperatorType.OP_GATHER

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        return [tuple(in_dims[1])], [in_dtypes[0]], []

    def axis_kinds(self):
        k = _batch_only_kinds(len(self.layer.outputs[0].dims))
        if self.attrs["dim"] % len(k) == 0:
            k[0] = "none"
        return k

    def supports_axis(self, axis):
        return axis == 0 and self.attrs["dim"] % len(self.layer.outputs[0].dims) != 0

    def input_maps(self):
        n = len(self.layer.outputs[0].dims)
        return [(0,) + (None,) * (len(self.layer.inputs[0].dims) - 1), (0,) + (None,) * (n - 1)]

    def _geom(self, shape, dtype, on_gpu, idx):
        """(dsz, inner, xd) for the HIP kernels (transfer.hip), or None: a bf16 / fp32 x on the GPU,
        int32 / int64 indices, every dim but `dim` equal between x and idx."""
        n = len(shape)
        d = self.attrs["dim"] % n
        if not (on_gpu and dtype in (torch.bfloat16, torch.float32) and idx.dtype in (torch.int32, torch.int64)
                and idx.dim() == n and all(shape[k] == idx.shape[k] for k in range(n) if k != d)):
            return None
        g = (idx.shape[d], math.prod(shape[d + 1:]), shape[d])
        return g if min(g) > 0 else None

    def forward(self, ctx, xs, ws):
        x, idx = xs
        ctx.saved.update(shape=x.shape, idx=idx)
        g = self._geom(tuple(x.shape), x.dtype, x.is_cuda, idx)
        if g is not None:
            # the HIP kernels clamp an out-of-range index into [0, xd) (no out-of-bounds access)
            # where torch.gather raises; FF_CHECK_INDICES=1 restores the error (one device sync)
            if _CHECK_INDICES and bool(((idx < 0) | (idx >= g[2])).any()):
                raise IndexError(f"gather: index out of range for dim size {g[2]}")
            out = torch.empty(idx.shape, dtype=x.dtype, device=x.device)
            K.ext().gather_fwd(x.contiguous(), idx.contiguous(), out, *g)
            return [out]
        return [torch.gather(x, self.attrs["dim"], idx.long())]

    def backward(self, ctx, douts):
        shp, idx = ctx.saved.pop("shape"), ctx.saved.pop("idx")
        dy = douts[0]
        dx = torch.zeros(shp, dtype=torch.float32, device=dy.device)
        g = self._geom(tuple(shp), dy.dtype, dy.is_cuda, idx)
        if g is not None:  # fp32 atomics into dx (repeated indices), then one cast
            K.ext().gather_bwd(dy.contiguous(), idx.contiguous(), dx, *g)
        else:
            dx.scatter_add_(self.attrs["dim"], idx.long(), dy.float())
        return [dx.to(dy.dtype), None]

    def needs_input_grad(self, i):
        return i == 0
