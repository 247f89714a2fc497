"""BatchMatmul, reductions, TopK and the mixture-of-experts family (GroupBy / Aggregate /
AggregateSpec / Cache).

Reference: src/ops/batch_matmul.cc, reduce.cc, mean.cc (a stub that asserts in the reference),
topk.cc, group_by.cc, aggregate.cc, aggregate_spec.cc, cache.cc (also a stub there).
BatchMatmul runs on the bf16 MFMA GEMM (strided batch); TopK and the MoE routing ops run on the
HIP kernels of csrc/kernels/moe.hip on the device (no host synchronisation, so an MoE step can be
captured into a hipGraph) and on torch indexing on the CPU.
"""
from __future__ import annotations

import math

import torch

from .. import kernels as K
from ..type import DataType, OperatorType
from .base import OpImpl, register


@register(OperatorType.OP_BATCHMATMUL)
class BatchMatmul(OpImpl):
    """C[..., M, N] = A[..., M, K] . B[..., K, N] (reference batch_matmul semantics, torch order)."""
    op_type = OperatorType.OP_BATCHMATMUL

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        a, b = in_dims
        assert a[-1] == b[-2], (a, b)
        return [tuple(a[:-1]) + (b[-1],)], [in_dtypes[0]], []

    def extra_axis_sizes(self):
        return [self.layer.inputs[0].dims[-1]]

    def axis_kinds(self):
        n = len(self.layer.outputs[0].dims)
        return ["sample"] + ["attribute"] * (n - 3) + ["attribute", "parameter", "parameter"]

    def input_maps(self):
        n = len(self.layer.outputs[0].dims)
        lead = tuple(range(n - 2))
        return [lead + (n - 2, n), lead + (n, n - 1)]

    def forward(self, ctx, xs, ws):
        a, b = xs[0].contiguous(), xs[1].contiguous()
        c = K.bmm(a, b)
        if ctx.training:
            ctx.saved.update(a=a, b=b)
        return [c]

    def backward(self, ctx, douts):
        a, b = ctx.saved.pop("a"), ctx.saved.pop("b")
        dc = douts[0].contiguous()
        da = K.bmm(dc, b, trans_b=True)
        db = K.bmm(a, dc, trans_a=True)
        return [da, db]

    def flops(self, in_shapes, out_shapes, w_shapes):
        return 2.0 * math.prod(out_shapes[0]) * in_shapes[0][-1]

    def uses_mfma(self):
        return True


@register(OperatorType.OP_REDUCE_SUM, OperatorType.OP_MEAN, OperatorType.OP_REDUCE_MEAN)
class Reduce(OpImpl):
    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        d = list(in_dims[0])
        axes = sorted(a % len(d) for a in attrs["axes"])
        attrs["axes"] = axes
        keep = attrs.get("keepdims", False)
        out = [1 if i in axes else s for i, s in enumerate(d)] if keep else [s for i, s in enumerate(d) if i not in axes]
        if not out:
            out = [1]
        return [tuple(out)], [in_dtypes[0]], []

    def _mean(self):
        return self.layer.op_type in (OperatorType.OP_MEAN, OperatorType.OP_REDUCE_MEAN)

    def axis_kinds(self):
        return ["none"] * len(self.layer.outputs[0].dims)

    def input_maps(self):
        return [tuple([None] * len(self.layer.inputs[0].dims))]

    def forward(self, ctx, xs, ws):
        x = xs[0]
        axes = self.attrs["axes"]
        keep = self.attrs.get("keepdims", False)
        y = x.float().mean(axes, keepdim=keep) if self._mean() else x.float().sum(axes, keepdim=keep)
        ctx.saved["shape"] = x.shape
        return [y.reshape(self.layer.outputs[0].dims).to(x.dtype)]

    def backward(self, ctx, douts):
        shp = ctx.saved.pop("shape")
        axes = self.attrs["axes"]
        g = douts[0].float()
        kshape = [1 if i in axes else s for i, s in enumerate(shp)]
        g = g.reshape(kshape).expand(shp)
        if self._mean():
            g = g / math.prod(shp[a] for a in axes)
        return [g.to(douts[0].dtype).contiguous()]


@register(OperatorType.OP_TOPK)
class TopK(OpImpl):
    """Outputs (values, int32 indices) of the k largest along the last dim."""
    op_type = OperatorType.OP_TOPK

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        d = tuple(in_dims[0][:-1]) + (attrs["k"],)
        return [d, d], [in_dtypes[0], DataType.DT_INT32], []

    def axis_kinds(self):
        n = len(self.layer.outputs[0].dims)
        return ["sample"] + ["none"] * (n - 1)

    def output_maps(self):
        n = len(self.layer.outputs[0].dims)
        return [tuple(range(n)), tuple(range(n))]

    def forward(self, ctx, xs, ws):
        x = xs[0]
        if K.moe_on_device(x):  # HIP kernel (csrc/kernels/moe.hip): values descending, ties lowest index
            v, i = K.topk(x, self.attrs["k"])
            ctx.saved.update(idx=i, shape=x.shape, dtype=x.dtype)
            return [v, i]
        v, i = torch.topk(x.float(), self.attrs["k"], -1, largest=True, sorted=bool(self.attrs.get("sorted", False)))
        ctx.saved.update(idx=i, shape=x.shape, dtype=x.dtype)
        return [v.to(x.dtype), i.to(torch.int32)]

    def backward(self, ctx, douts):
        i, shp, dt = ctx.saved.pop("idx"), ctx.saved.pop("shape"), ctx.saved.pop("dtype")
        if douts[0] is None:
            return [torch.zeros(shp, dtype=dt, device=i.device)]
        if K.moe_on_device(douts[0]):
            return [K.topk_bwd(douts[0].to(dt), i.to(torch.int32), shp)]
        dx = torch.zeros(shp, dtype=torch.float32, device=i.device)
        dx.scatter_add_(-1, i.long(), douts[0].float())
        return [dx.to(douts[0].dtype)]


def _expert_slots(assign: torch.Tensor, n: int, cap: int):
    """Reference routing order: samples scanned in order, each expert fills rows 0..cap-1, overflow
    dropped. Returns (expert, row, valid) per (sample, choice)."""
    flat = assign.reshape(-1).long()
    onehot = torch.nn.functional.one_hot(flat.clamp(0, n - 1), n)
    pos = (torch.cumsum(onehot, 0) - 1).gather(1, flat.clamp(0, n - 1)[:, None]).squeeze(1)
    valid = (pos < cap) & (flat >= 0) & (flat < n)
    return flat, pos, valid


@register(OperatorType.OP_GROUP_BY)
class GroupBy(OpImpl):
    """Scatter rows of `data` [B, D] to n expert tensors [cap, D], cap = ceil(alpha*k/n*B)."""
    op_type = OperatorType.OP_GROUP_BY

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        data, assign = in_dims
        n, alpha = attrs["n"], attrs["alpha"]
        k = assign[-1]
        cap = int(math.ceil(alpha * k / n * data[0]))
        attrs["cap"] = cap
        return [(cap,) + tuple(data[1:])] * n, [in_dtypes[0]] * n, []

    def axis_kinds(self):
        return ["none"] * len(self.layer.outputs[0].dims)

    def input_maps(self):
        return [tuple([None] * len(t.dims)) for t in self.layer.inputs]

    def output_maps(self):
        return [tuple([None] * len(o.dims)) for o in self.layer.outputs]

    def forward(self, ctx, xs, ws):
        data, assign = xs
        n, cap = self.attrs["n"], self.attrs["cap"]
        k = assign.shape[-1]
        if K.moe_on_device(data, n):
            # device routing + row scatter, no host synchronisation (csrc/kernels/moe.hip)
            e, pos, _ = K.moe_route(assign, n, cap)
            outs = [torch.empty((cap,) + tuple(data.shape[1:]), dtype=data.dtype, device=data.device) for _ in range(n)]
            K.ext().groupby_fwd(data.contiguous(), e, pos, outs, cap, k)
            ctx.saved.update(dev=(e, pos), shape=data.shape, dtype=data.dtype, k=k)
            return outs
        e, pos, valid = _expert_slots(assign, n, cap)
        src = torch.arange(e.numel(), device=data.device) // k
        outs = []
        for j in range(n):
            o = torch.zeros((cap,) + tuple(data.shape[1:]), dtype=data.dtype, device=data.device)
            m = valid & (e == j)
            o[pos[m]] = data[src[m]]
            outs.append(o)
        ctx.saved.update(e=e, pos=pos, valid=valid, src=src, shape=data.shape)
        return outs

    def backward(self, ctx, douts):
        s = ctx.saved
        if "dev" in s:
            e, pos = s.pop("dev")
            shp, dt, k = s.pop("shape"), s.pop("dtype"), s.pop("k")
            dx = torch.empty(shp, dtype=dt, device=e.device)
            K.ext().groupby_bwd([d.to(dt).contiguous() if d is not None else None for d in douts], e, pos, dx,
                                self.attrs["cap"], k)
            return [dx, None]
        e, pos, valid, src, shp = s.pop("e"), s.pop("pos"), s.pop("valid"), s.pop("src"), s.pop("shape")
        like = [d for d in douts if d is not None][0]
        dx = torch.zeros(shp, dtype=torch.float32, device=like.device)
        for j, d in enumerate(douts):
            if d is None:
                continue
            m = valid & (e == j)
            dx.index_add_(0, src[m], d[pos[m]].float())
        return [dx.to(like.dtype), None]

    def needs_input_grad(self, i):
        return i == 0


@register(OperatorType.OP_AGGREGATE, OperatorType.OP_AGG_SPEC)
class Aggregate(OpImpl):
    """inputs: gate_preds [B,k], gate_assign [B,k], true_assign [B,k], full_gate_preds [B,n],
    exp_preds x n ([cap, D]). out[b] = sum_j gate_preds[b,j] * exp_pred[assign[b,j]][row].
    Backward (reference aggregate.cu): expert grads = gate * dout; full-gate grads = dout.exp_pred
    plus lambda_bal * n / B * expert load (the reference's scaling, aggregate.cu:194), made zero-mean
    per row. AggregateSpec skips the gate product."""

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        B = in_dims[0][0]
        D = in_dims[4][-1]
        return [(B, D)], [in_dtypes[4]], []

    def axis_kinds(self):
        return ["none", "none"]

    def input_maps(self):
        return [tuple([None] * len(t.dims)) for t in self.layer.inputs]

    def forward(self, ctx, xs, ws):
        gate, assign, true_assign, full_gate = xs[:4]
        exps = xs[4:]
        n = len(exps)
        cap = exps[0].shape[0]
        B, k = assign.shape
        spec = self.layer.op_type == OperatorType.OP_AGG_SPEC
        if K.moe_on_device(exps[0], n):
            dt = exps[0].dtype
            e, pos, load = K.moe_route(assign, n, cap)
            ex = [x.to(dt).contiguous() for x in exps]
            g = None if spec else gate.to(dt).contiguous()
            out = torch.empty((B, ex[0].shape[-1]), dtype=dt, device=ex[0].device)
            K.ext().aggregate_fwd(g, ex, e, pos, out, cap, k)
            ctx.saved.update(dev=(e, pos, load), exps=ex, gate=g, spec=spec, assign=assign.to(torch.int32).contiguous(),
                             true_assign=true_assign.to(torch.int32).contiguous(), gate_dtype=gate.dtype,
                             full_shape=full_gate.shape, full_dtype=full_gate.dtype, k=k, cap=cap)
            return [out]
        e, pos, valid = _expert_slots(assign, n, cap)
        stacked = torch.stack([x.float() for x in exps])  # [n, cap, D]
        rows = stacked[e.clamp(0, n - 1), pos.clamp(0, cap - 1)]  # [B*k, D]
        rows = rows * valid[:, None]
        spec = self.layer.op_type == OperatorType.OP_AGG_SPEC
        w = torch.ones_like(gate.float().reshape(-1)) if spec else gate.float().reshape(-1)
        out = (rows * w[:, None]).reshape(B, k, -1).sum(1)
        ctx.saved.update(e=e, pos=pos, valid=valid, rows=rows, w=w, B=B, k=k, n=n, cap=cap, spec=spec,
                         assign=assign, true_assign=true_assign, gate_dtype=gate.dtype, full_shape=full_gate.shape)
        return [out.to(exps[0].dtype)]

    def backward(self, ctx, douts):
        s = ctx.saved
        if "dev" in s:
            e, pos, load = s["dev"]
            ex, g, spec = s["exps"], s["gate"], s["spec"]
            dt = ex[0].dtype
            dout = douts[0].to(dt).contiguous()
            B, k, n = dout.shape[0], s["k"], len(ex)
            dexp = [torch.empty_like(x) for x in ex]
            dgate = None if spec else torch.empty((B, k), dtype=dt, device=dout.device)
            dfull = None if spec else torch.empty(tuple(s["full_shape"]), dtype=dt, device=dout.device)
            lam = float(self.attrs.get("lambda_bal", 0.0)) * n / max(B, 1)  # reference aggregate.cu:194
            K.ext().aggregate_bwd(dout, g, ex, dexp, e, pos, s["assign"], s["true_assign"], load,
                                  lam, dgate, dfull, s["cap"], k)
            gdt, fdt = s["gate_dtype"], s["full_dtype"]
            ctx.saved.clear()
            return [None if dgate is None else dgate.to(gdt), None, None,
                    None if dfull is None else dfull.to(fdt)] + dexp
        dout = douts[0].float()
        B, k, n, cap = s["B"], s["k"], s["n"], s["cap"]
        e, pos, valid, rows, w = s["e"], s["pos"], s["valid"], s["rows"], s["w"]
        dgrow = dout.repeat_interleave(k, 0)  # [B*k, D]
        dexp = []
        for j in range(n):
            g = torch.zeros(cap, dout.shape[1], dtype=torch.float32, device=dout.device)
            m = valid & (e == j)
            g[pos[m]] = (dgrow[m] * w[m][:, None])
            dexp.append(g.to(douts[0].dtype))
        dgate = None
        dfull = None
        if not s["spec"]:
            dgate = (dgrow * rows).sum(-1).reshape(B, k).to(s["gate_dtype"])
            lam = float(self.attrs.get("lambda_bal", 0.0)) * n / max(B, 1)  # reference aggregate.cu:194
            full = torch.zeros(s["full_shape"], dtype=torch.float32, device=dout.device)
            corr = (s["assign"] == s["true_assign"]).all(-1)
            contrib = (dgrow * rows).sum(-1) * corr.repeat_interleave(k)
            full.view(-1).index_add_(0, (torch.arange(B * k, device=dout.device) // k) * n + e.clamp(0, n - 1),
                                     contrib * valid)
            bal = torch.bincount(e.clamp(0, n - 1), minlength=n).float()
            full = full + lam * bal[None, :]
            full = full - full.mean(-1, keepdim=True)
            dfull = full.to(s["gate_dtype"])
        ctx.saved.clear()
        return [dgate, None, None, dfull] + dexp

    def needs_input_grad(self, i):
        return i not in (1, 2)


@register(OperatorType.OP_CACHE)
class Cache(OpImpl):
    """Caches the last `num_batches` batches of its input (reference cache.cc is a stub:
    FFModel::cache asserts). Forward passes through and records; `score()` compares the cached
    value with the current one (used by recompile triggers)."""
    op_type = OperatorType.OP_CACHE

    def forward(self, ctx, xs, ws):
        x = xs[0]
        buf = ctx.extra.setdefault("cache", [])
        buf.append(x.detach().clone())
        nb = int(self.attrs.get("num_batches", 1))
        if len(buf) > nb:
            buf.pop(0)
        return [x]

    def backward(self, ctx, douts):
        return [douts[0]]
